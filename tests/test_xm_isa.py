"""tools/check_xm_isa.py (the build-time guard of the X/M kernel's inline-asm
K loop, csrc/band.hip xm_load_asm / xm_wait_slot): it passes on the built
library and catches a read before its wait, a spill-like extra memory op and
a wrong wait count on synthetic loops.  CPU only (disassembly)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_xm_isa as cx  # noqa: E402


def test_built_library_passes():
    if not os.path.exists(cx.OBJ):
        pytest.skip("gptq-svd_amd/build/band.o not built")
    assert cx.main() == 0


def _loop(nbc=1, da=2, wait=None, read_early=False, extra=None):
    """prologue of da slots, a loop body that waits per slot, uses the slot
    (an MFMA reading it) and reloads it; instructions as check_kernel sees
    them: (address, mnemonic, operands, branch target)."""
    per = nbc + 2
    wait = (da - 1) * per if wait is None else wait
    ins, a = [], 0

    def add(mn, ops, tgt=None):
        nonlocal a
        ins.append((a, mn, ops, tgt))
        a += 8

    add("s_mov_b32", ["s0", "0"])
    slot = lambda u, c: f"v[{10 + 2 * (u * per + c)}:{11 + 2 * (u * per + c)}]"
    for u in range(da):
        for c in range(per):
            add("global_load_dwordx2", [slot(u, c), "v[2:3]", "off"])
    head = a
    for u in range(da):
        if not (read_early and u == 0):
            add("s_waitcnt", [f"vmcnt({wait})"])
        add("v_mfma_f64_16x16x4_f64", ["v[100:107]", slot(u, 0), slot(u, 1), "v[100:107]"])
        if extra and u == 0:
            add(*extra)
        for c in range(per):
            add("global_load_dwordx2", [slot(u, c), "v[2:3]", "off"])
    if read_early:
        add("s_waitcnt", [f"vmcnt({wait})"])
    add("s_cbranch_scc1", ["label"], head)
    add("s_waitcnt", ["vmcnt(0)"])
    add("s_endpgm", [])
    return ins, da, wait


def test_synthetic_safe_loop_passes():
    ins, da, wait = _loop()
    assert cx.check_kernel("k", ins, 1, da, 3, wait, {"global_load_dwordx2"}) == []


def test_read_before_wait_is_caught():
    ins, da, wait = _loop(read_early=True)
    errs = cx.check_kernel("k", ins, 1, da, 3, wait, {"global_load_dwordx2"})
    assert any("before its load's wait" in e for e in errs), errs


def test_extra_memory_op_is_caught():
    ins, da, wait = _loop(extra=("scratch_store_dwordx2", ["off", "v[10:11]", "s0"]))
    errs = cx.check_kernel("k", ins, 1, da, 3, wait, {"global_load_dwordx2"})
    assert any("unexpected vector-memory op" in e for e in errs), errs


def test_too_loose_wait_is_caught():
    ins, da, _ = _loop(wait=3 * 2)   # waits that leave the slot's own loads in flight
    errs = cx.check_kernel("k", ins, 1, da, 3, 3 * 2, {"global_load_dwordx2"})
    assert any("before its load's wait" in e for e in errs), errs


def test_build_config_follows_the_source_defaults():
    cfg = cx.build_config()
    frag, da, lps, wait, lmn = cfg[2]
    assert frag == "xm_kernelILi2E" and wait == (da - 1) * lps and 0 < wait <= 63
    assert cfg[1][3] == (cfg[1][1] - 1) * 3
