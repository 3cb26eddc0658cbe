"""Pick the stall-counter passes that this box's rocprofv3 offers.

usage: stall_passes.py LIST_FILE            (LIST_FILE: `rocprofv3 -L` output)
prints one line per pass: the space-separated counters, each pass within
the gfx950 per-block slot limits (SQ 8, TA 2, TD 2, TCP 4, TCC 4, GRBM 2;
a counter's _sum / _avr / _min / _max count once).  Candidates the box
does not list are dropped, so a pass never names an unknown counter.

Pass 1: wave-state split (SQ_WAIT_ANY = parked on s_waitcnt / barrier,
SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY; they sum to
SQ_WAVE_CYCLES) and the vector-memory instruction count.
Pass 2: the address / data path (TA busy and stalled-by-cache cycles, TD
busy, TCP stalls) and L2 hit / miss.
"""
import re
import sys

PASSES = [
    {"SQ": ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_INSTS_VMEM_RD", "SQ_BUSY_CYCLES", "SQ_WAVES", "SQ_INSTS_LDS"],
     "GRBM": ["GRBM_GUI_ACTIVE"]},
    {"TA": ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"],
     "TD": ["TD_TD_BUSY_sum", "TD_TC_STALL_sum"],
     "TCP": ["TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum",
             "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
             "TCP_TCC_READ_REQ_LATENCY_sum"],
     "TCC": ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_LEVEL_sum"],
     "GRBM": ["GRBM_GUI_ACTIVE"]},
]
LIMIT = {"SQ": 8, "TA": 2, "TD": 2, "TCP": 4, "TCC": 4, "GRBM": 2}


def base(name):
    return re.sub(r"_(sum|avr|min|max)$", "", name)


def main():
    text = open(sys.argv[1]).read()
    avail = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", text))
    for p in PASSES:
        picked = []
        for block, cands in p.items():
            used = set()
            for c in cands:
                if c not in avail and base(c) not in avail:
                    continue
                b = base(c)
                if b in used or len(used) >= LIMIT[block]:
                    continue
                used.add(b)
                # a derived _sum the box lists as its base only: ask for the base
                picked.append(c if c in avail else b)
        if picked:
            print(" ".join(picked))


if __name__ == "__main__":
    main()
