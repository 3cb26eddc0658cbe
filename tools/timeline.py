"""Print the kernel timeline of the last N dispatches from a rocprofv3
kernel-trace CSV (development tool).

usage: timeline.py run_kernel_trace.csv [N] [start_regex]
With start_regex, prints from the last dispatch matching it."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
if len(sys.argv) > 3:
    idx = max(i for i, r in enumerate(rows) if re.search(sys.argv[3], r["Kernel_Name"]))
    rows = rows[idx:idx + n]
else:
    rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3
    print(f"{(s - t0) / 1e3:10.2f} +{(e - s) / 1e3:8.2f} us gap {gap:7.2f} q{r.get('Queue_Id', '?'):>2} "
          f"{re.sub(r'[(<].*', '', r['Kernel_Name'].replace('(anonymous namespace)::', ''))[:60]}")
    prev_end = max(prev_end, e)
    busy += e - s
print(f"span {(prev_end - t0) / 1e3:.1f} us, summed kernel time {busy / 1e3:.1f} us")
