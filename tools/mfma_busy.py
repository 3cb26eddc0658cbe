"""MFMA busy fraction per kernel class from a rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (development tool;
tools/profile_round.sh).

usage: mfma_busy.py COUNTER_CSV [OUT_JSON] CLASS=SUBSTRING ...

Per class, summed over its dispatches:
  busy_frac    = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs)
                 (GRBM_GUI_ACTIVE is summed over the 8 XCDs, so / 8 is the
                 launch's active cycles; 1024 SIMDs on MI355X);
  clock_GHz    = GRBM_GUI_ACTIVE / 8 / (End - Start timestamp): the
                 effective clock of the profiled launches (DVFS, MI355X guide).
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


def main():
    path = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and "=" not in sys.argv[2] else None
    specs = [a for a in sys.argv[2:] if "=" in a]
    rows = list(csv.DictReader(open(path)))
    res = {}
    for spec in specs:
        cls, sub = spec.split("=", 1)
        per = defaultdict(dict)
        span = {}
        for r in rows:
            if sub not in r["Kernel_Name"]:
                continue
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            span[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if not per:
            print(f"{cls}: no dispatches of {sub}")
            continue
        mfma = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in per.values())
        grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in per.values())
        ns = sum(span.values())
        ent = dict(kernel=sub, dispatches=len(per), mfma_busy_cycles=mfma, grbm_gui_active=grbm,
                   busy_frac=round(mfma / (SIMDS * grbm / XCDS), 4) if grbm else None,
                   clock_GHz=round(grbm / XCDS / ns, 3) if ns else None)
        res[cls] = ent
        print(cls, ent)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
