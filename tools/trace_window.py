"""Print the kernel timeline (start offset, duration, gap to the previous
kernel, name) of the last CALLS-th window of a rocprofv3 kernel trace
(development tool):  python tools/trace_window.py KERNEL_TRACE_CSV FIRST_KERNEL_SUBSTR [NTH]
The window starts at the NTH-from-last dispatch whose name contains
FIRST_KERNEL_SUBSTR and runs to the next such dispatch (or the end)."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    key = sys.argv[2]
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    a = idx[-nth]
    b = idx[-nth + 1] if nth > 1 else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f}  "
              f"{r['Kernel_Name'][:90]}")
        prev_end = max(prev_end, e)
    print(f"window {(prev_end - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
