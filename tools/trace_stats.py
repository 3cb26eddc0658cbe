"""Per-kernel totals inside one window of a rocprofv3 kernel trace (development tool).
    python tools/trace_stats.py TRACE.csv FIRST_REGEX LAST_REGEX [occurrence]"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.split(r"[(<]", name, maxsplit=1)[0][:40] + ("<" + name.split("<", 1)[1].split(">")[0][:22] + ">" if "<" in name.split("(")[0] else "")


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
occ = int(sys.argv[4]) if len(sys.argv) > 4 else 1
firsts = [i for i, r in enumerate(rows) if re.search(sys.argv[2], r["Kernel_Name"])]
lasts = [i for i, r in enumerate(rows) if re.search(sys.argv[3], r["Kernel_Name"])]
s = firsts[0]
for _ in range(occ):
    e = next(i for i in lasts if i >= s)
    seg, s = rows[s:e + 1], next((i for i in firsts if i > e), len(rows))
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[short(r["Kernel_Name"])]
    a[0] += 1
    a[1] += d
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
busy, cur = 0, None
for a, b in iv:
    if cur is None or a > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
        cur = [a, b]
    else:
        cur[1] = max(cur[1], b)
busy += cur[1] - cur[0]
print(f"window {(t1 - t0) / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms, {len(seg)} kernels")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:64s} n={v[0]:5d} tot={v[1] / 1e3:7.2f} ms avg={v[1] / v[0]:8.1f} us")
