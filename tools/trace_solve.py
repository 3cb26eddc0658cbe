"""Kernel ranking of the last solve in a rocprofv3 kernel trace of
tools/solve_time.py (development tool).  A solve starts at the first panel-QR
launch after the previous solve's bulge chase.
    python tools/trace_solve.py gpurun_out/x/run_kernel_trace.csv [top]"""
import collections
import csv
import re
import sys

r = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
bul = [i for i, x in enumerate(r) if 'bulge_lds' in x['Kernel_Name']]
i0 = bul[-2] if len(bul) > 1 else 0
i0 = next(i for i in range(i0, len(r)) if 'pqr_kernel' in r[i]['Kernel_Name'])
win = r[i0:]


def short(name):
    name = name.replace('(anonymous namespace)::', '')
    return re.sub(r'\(.*', '', name)[:80]


tot, cnt = collections.Counter(), collections.Counter()
for x in win:
    k = short(x['Kernel_Name'])
    tot[k] += int(x['End_Timestamp']) - int(x['Start_Timestamp'])
    cnt[k] += 1
span = (int(win[-1]['End_Timestamp']) - int(win[0]['Start_Timestamp'])) / 1e6
print(f"last solve: span {span:.2f} ms, kernels busy {sum(tot.values()) / 1e6:.2f} ms")
for k, v in tot.most_common(top):
    print(f"{v / 1e6:8.3f} ms {cnt[k]:5d}  {k}")
