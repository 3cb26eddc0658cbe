"""Summarise stall-counter passes (tools/stall_passes.py) per kernel class.

usage: stall_summary.py OUT_JSON CLASS=SUBSTRING ... -- CSV ...
(CSV: rocprofv3 --pmc counter_collection.csv files, one per pass)

Per class: each counter's mean per launch (summed over the counter's
instances), and the ratios the X/M question needs:
  wave states   SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
                SQ_WAVE_CYCLES (parked on a wait count or barrier / issue
                stalled / issuing; they sum to ~1);
  TA busy       TA_TA_BUSY / (CUs x GRBM_GUI_ACTIVE / XCDs): the fraction of
                the launch the average CU's texture-address unit is busy
                (GRBM_GUI_ACTIVE is summed over the 8 XCDs);
  stalled by TC TA_*_STALLED_BY_TC over TA busy;
  L2 hit rate   TCC_HIT / (TCC_HIT + TCC_MISS);
  HBM latency   TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ: mean cycles a fabric
                read is outstanding.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

CUS, XCDS = 256, 8


def load(paths, sub):
    per = defaultdict(lambda: defaultdict(float))  # (file, dispatch) -> counter -> value
    for p in paths:
        for r in csv.DictReader(open(p)):
            if sub not in r["Kernel_Name"]:
                continue
            per[(p, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    sums, cnt = defaultdict(float), defaultdict(int)
    for vals in per.values():
        for c, v in vals.items():
            sums[c] += v
            cnt[c] += 1
    return {c: sums[c] / cnt[c] for c in sums}, {c: cnt[c] for c in cnt}


def pick(m, name):
    for k in (name, name + "_sum"):
        if k in m:
            return m[k]
    b = re.sub(r"_sum$", "", name)
    return m.get(b)


def main():
    args = sys.argv[1:]
    sep = args.index("--")
    out, specs, csvs = args[0], args[1:sep], args[sep + 1:]
    data = json.load(open(out)) if os.path.exists(out) else {}
    for spec in specs:
        cls, sub = spec.split("=", 1)
        m, n = load(csvs, sub)
        if not m:
            print(f"{cls}: no dispatches of {sub}")
            continue
        ent = {"kernel": sub, "per_launch": {k: round(v) for k, v in sorted(m.items())},
               "launches": n, "sources": csvs}
        wc = pick(m, "SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                v = pick(m, k)
                if v is not None:
                    ent[k.lower().replace("sq_", "frac_")] = round(v / wc, 4)
        g = pick(m, "GRBM_GUI_ACTIVE")
        ta = pick(m, "TA_TA_BUSY")
        if g and ta is not None:
            ent["ta_busy_frac"] = round(ta / (CUS * g / XCDS), 4)
            for k in ("TA_ADDR_STALLED_BY_TC_CYCLES", "TA_DATA_STALLED_BY_TC_CYCLES"):
                v = pick(m, k)
                if v is not None and ta:
                    ent[k.lower() + "_over_busy"] = round(v / ta, 4)
        h, mi = pick(m, "TCC_HIT"), pick(m, "TCC_MISS")
        if h is not None and mi is not None and h + mi > 0:
            ent["l2_hit_rate"] = round(h / (h + mi), 4)
        rq, lv = pick(m, "TCC_EA0_RDREQ"), pick(m, "TCC_EA0_RDREQ_LEVEL")
        if rq and lv is not None:
            ent["fabric_read_latency_cycles"] = round(lv / rq, 1)
        data[cls] = ent
        print(cls, json.dumps({k: v for k, v in ent.items() if k not in ("per_launch", "sources")}))
    json.dump(data, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
