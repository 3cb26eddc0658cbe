"""Per-solve kernel time from a rocprofv3 kernel trace of tools/solve_time.py
(development tool): the last solve's total per kernel-name substring.
    python tools/trace_sum.py gpurun_out/x/run_kernel_trace.csv bisect pqr_kernel ..."""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
nsolve = sum('bulge_lds' in x['Kernel_Name'] for x in r)
print(f"{sys.argv[1]}: {nsolve} solves")
for key in sys.argv[2:]:
    ds = [int(x['End_Timestamp']) - int(x['Start_Timestamp']) for x in r if key in x['Kernel_Name']]
    per = len(ds) // max(nsolve, 1)
    last = ds[-per:] if per else []
    print(f"  {key:24s} calls/solve {per:5d}  last solve {sum(last) / 1e6:9.3f} ms")
