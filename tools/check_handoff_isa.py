#!/usr/bin/env python3
"""Build-time guard for the cross-workgroup hand-offs of the persistent
kernels (csrc/spin.h, DESIGN.md §3 "Persistent kernels").

The kernels hand data from one workgroup to another inside a launch in two
forms (MI355X_MICROARCH.md § visibility):

* write-through form (pqr_kernel, xm_kernel, the pivot kernels, the
  boundary chunks of q2_lds_kernel, q1_lds_kernel<false>): payload
  stored `sc1`, every storing wave drains `vmcnt(0)`, one lane signals (an
  agent-scope atomic add or `sc1` store); the consumer polls the word and
  reads the payload with `sc1` loads -- the guide's "Valid forms" row 1;
* one-L2 form (bulge_lds_kernel, bulge_df_kernel, bt_few_kernel, q1_lds_kernel<true>):
  the workers are the workgroups that landed on ONE XCD (HW_REG_XCC_ID
  election; the others exit before touching the data), the payload is
  stored plain (the lines stay in that XCD's L2, the point of coherence of
  its CUs), drained with `vmcnt(0)` before the signal, and the consumer
  reads it with `sc1` (L1-bypassing) loads from the same L2.  No agent-scope
  release or acquire: that would write the L2 back to HBM / invalidate L1 on
  every hand-off (>= 1.7 us each, thousands per launch).

Neither form is a C++ memory-model edge across workgroups, so this script
checks in the gfx950 code object what the forms rely on:

(A) drain before signal, every kernel in KERNELS: on EVERY path of the
    control-flow graph (a forward data-flow over basic blocks, loops
    included), between a vector-memory store and the next signal of the same
    wave -- a non-returning `global_atomic_add` (arrival) or a
    `global_store_dword` (progress word / flag) -- the wave executes
    `s_waitcnt vmcnt(0)`.  The give-up path of a bounded wait marks its stall
    word with `global_atomic_or` (spin.h stall_set), which is exempt: the
    launch's results are poisoned then;
(B) one-L2 kernels: the kernel reads HW_REG_XCC_ID, and every `buffer_load`
    (the hand-off payload loads) carries `sc1`; in the bulge kernels every
    vector load carries `sc1` (the band is their only global input);
(C) no `flat_` load in the kernels marked so (a flat load could be a
    hand-off load that bypasses both rules).  Words no wave of the launch
    waits on (ticket resets, path records) are written by atomic exchange
    (spin.h ctl_reset / ctl_record) and are not signals.

Exit status 0 = every rule holds; otherwise the offending paths are printed.
Run by ``__graft_entry__.build()`` after the library is built.
"""
import os
import re
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from check_xm_isa import code_object, disasm  # noqa: E402

BUILD = os.path.join(HERE, "..", "gptq-svd_amd", "build")
# object -> [(mangled-name fragment, one-L2 form, every vector load sc1, no flat loads)]
KERNELS = {
    "bulge.o": [("bulge_lds_kernel", True, True, True), ("bulge_df_kernel", True, True, True)],
    "backtr.o": [("bt_few_kernelILi1ELb1E", True, False, True),
                 ("bt_few_kernelILi2ELb1E", True, False, True),
                 ("bt_few_kernelILi1ELb0E", True, False, True),
                 ("bt_few_kernelILi2ELb0E", True, False, True),
                 ("q2_lds_kernelILi1E", False, False, True), ("q1_lds_kernelILb1E", True, False, True),
                 ("q1_lds_kernelILb0E", False, False, True)],
    # pqr: the hand-off words and payloads go through explicit address_space(1)
    # sc1 atomics (st_sc1 / ld_sc1); its flat accesses are the panel rows of
    # the launch's input and its outputs, reached through the LDS copy of the
    # arguments (rule A still covers every signal, the out-of-line fallback's too)
    "pqr.o": [("pqr_kernel", False, False, False), ("ph_householder", False, False, False)],
    "band.o": [("xm_kernelILi1E", False, False, True), ("xm_kernelILi2E", False, False, True)],
    "factor.o": [("piv_panel_kernelILi1E", False, False, True),
                 ("piv_panel_kernelILi2E", False, False, True),
                 ("piv_step_kernel", False, False, True)],
}
STORE = re.compile(r"^(global_store|buffer_store|global_atomic|flat_store|flat_atomic)")
EXEMPT = ("global_atomic_or", "global_atomic_swap")  # stall marks, resets, records
BRANCH_END = ("s_endpgm", "s_setpc_b64")


def is_signal(mn, ops):
    if mn == "global_store_dword":
        return True
    # arrival: non-returning add (a returning one, sc0, is a ticket / queue take)
    return mn == "global_atomic_add" and "sc0" not in " ".join(ops).split()


def drains(mn, ops):
    return mn == "s_waitcnt" and "vmcnt(0)" in " ".join(ops)


def blocks(insns):
    """Basic blocks: (start, end) index ranges and successor lists."""
    base = insns[0][0]
    idx = {a - base: i for i, (a, _, _, _) in enumerate(insns)}
    lead = {0}
    for i, (_, mn, _, tgt) in enumerate(insns):
        if tgt is not None:
            lead.add(idx[tgt])
        if (tgt is not None or mn in BRANCH_END) and i + 1 < len(insns):
            lead.add(i + 1)
    starts = sorted(lead)
    bl = []
    for k, s in enumerate(starts):
        e = (starts[k + 1] if k + 1 < len(starts) else len(insns)) - 1
        _, mn, _, tgt = insns[e]
        succ = []
        if tgt is not None:
            succ.append(starts.index(idx[tgt]))
        if mn not in BRANCH_END and mn != "s_branch" and k + 1 < len(starts):
            succ.append(k + 1)
        bl.append((s, e, succ))
    return bl


def check_drain(name, insns):
    """Rule A: forward data-flow of 'a store of this wave may be outstanding'."""
    bl = blocks(insns)
    state_in = [None] * len(bl)
    state_in[0] = False
    work = [0]
    errs = []
    reported = set()
    while work:
        b = work.pop()
        s, e, succ = bl[b]
        pend = state_in[b]
        for i in range(s, e + 1):
            addr, mn, ops, _ = insns[i]
            if drains(mn, ops):
                pend = False
            elif is_signal(mn, ops):
                if pend and addr not in reported:
                    reported.add(addr)
                    errs.append(f"{name}: signal {mn} {', '.join(ops)} at 0x{addr:x} reachable "
                                f"from a store without s_waitcnt vmcnt(0)")
                # the signal itself is a store: later signals need no new drain
                # for it (it is not payload), keep the state
            elif STORE.match(mn) and not mn.startswith(EXEMPT):
                pend = True
        for t in succ:
            new = pend if state_in[t] is None else (state_in[t] or pend)
            if new != state_in[t]:
                state_in[t] = new
                work.append(t)
    return errs


def check_one_l2(name, insns, all_loads_sc1):
    errs = []
    if not any(mn == "s_getreg_b32" and any("HW_REG_XCC_ID" in o for o in ops)
               for _, mn, ops, _ in insns):
        errs.append(f"{name}: one-L2 hand-off without an HW_REG_XCC_ID election")
    for addr, mn, ops, _ in insns:
        words = " ".join(ops).split()
        if mn.startswith("buffer_load") and "sc1" not in words:
            errs.append(f"{name}: {mn} {', '.join(ops)} at 0x{addr:x} without sc1")
        if all_loads_sc1 and mn.startswith("global_load") and "sc1" not in words:
            errs.append(f"{name}: {mn} {', '.join(ops)} at 0x{addr:x} without sc1")
    return errs


def main() -> int:
    errs, seen = [], 0
    for obj, kernels in KERNELS.items():
        with tempfile.TemporaryDirectory() as tmp:
            funcs = disasm(code_object(os.path.join(BUILD, obj), tmp))
        for frag, one_l2, all_sc1, no_flat in kernels:
            names = [n for n in funcs if frag in n]
            if not names:
                errs.append(f"{obj}: kernel {frag} not found")
                continue
            for name in names:
                insns = funcs[name]
                seen += 1
                short = frag
                if no_flat:
                    errs += [f"{short}: flat load {mn} at 0x{a:x}"
                             for a, mn, _, _ in insns if mn.startswith("flat_load")]
                errs += check_drain(short, insns)
                if one_l2:
                    errs += check_one_l2(short, insns, all_sc1)
    if errs:
        print("check_handoff_isa: FAILED", file=sys.stderr)
        for e in errs[:40]:
            print("  " + e, file=sys.stderr)
        return 1
    print(f"check_handoff_isa: {seen} persistent kernels: drain-before-signal on every path, "
          f"one-L2 hand-offs elected and read sc1")
    return 0


if __name__ == "__main__":
    sys.exit(main())
