"""Aggregate kernel time by name over a window of a rocprofv3 kernel trace
(development tool):  python tools/trace_agg.py TRACE_CSV START_SUBSTR [END_SUBSTR] [TOP]
The window runs from the last dispatch containing START_SUBSTR to the first
later dispatch containing END_SUBSTR (or the end of the trace)."""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace('(anonymous namespace)::', '')
    return re.sub(r'\(.*', '', name)[:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    a = max(i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"])
    end = sys.argv[3] if len(sys.argv) > 3 else None
    b = next((i for i in range(a + 1, len(rows)) if end and end in rows[i]["Kernel_Name"]), len(rows))
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    win = rows[a:b]
    tot, cnt = collections.Counter(), collections.Counter()
    for x in win:
        k = short(x["Kernel_Name"])
        tot[k] += int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
        cnt[k] += 1
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6
    print(f"window: {len(win)} dispatches, span {span:.3f} ms, kernels busy {sum(tot.values()) / 1e6:.3f} ms")
    for k, v in tot.most_common(top):
        print(f"{v / 1e6:8.3f} ms {cnt[k]:5d}  {k}")


if __name__ == "__main__":
    main()
