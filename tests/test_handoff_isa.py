"""tools/check_handoff_isa.py (the build-time guard of the persistent
kernels' cross-workgroup hand-offs): it passes on the built library, and on
synthetic control-flow graphs it catches a signal reachable from a payload
store without a vmcnt(0) drain (straight line, one arm of a branch, around a
loop's back edge), accepts the drained forms and the exempt give-up / reset
atomics, and catches a one-L2 kernel that loads its payload without sc1 or
never elects an XCD.  CPU only (disassembly)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_handoff_isa as ch  # noqa: E402


def test_built_library_passes():
    if not os.path.exists(os.path.join(ch.BUILD, "bulge.o")):
        pytest.skip("gptq-svd_amd/build not built")
    assert ch.main() == 0


class Prog:
    """instructions as the checker sees them: (address, mnemonic, operands,
    branch target offset or None)"""

    def __init__(self):
        self.ins = []

    def add(self, mn, ops=(), tgt=None):
        self.ins.append((len(self.ins) * 8, mn, list(ops), tgt))
        return len(self.ins) * 8 - 8

    def label(self):
        return len(self.ins) * 8


STORE = ("buffer_store_dwordx4", ["v[0:3]", "v4", "s[0:3]", "0 offen"])
FLAG = ("global_store_dword", ["v5", "v6", "s[8:9]"])
DRAIN = ("s_waitcnt", ["vmcnt(0)"])


def test_straight_line():
    p = Prog()
    p.add(*STORE)
    p.add(*FLAG)
    p.add("s_endpgm")
    assert len(ch.check_drain("k", p.ins)) == 1
    p = Prog()
    p.add(*STORE)
    p.add(*DRAIN)
    p.add(*FLAG)
    p.add("s_endpgm")
    assert ch.check_drain("k", p.ins) == []


def test_arrival_and_ticket():
    p = Prog()
    p.add("global_store_dwordx2", ["v[0:1]", "v[2:3]", "off", "sc1"])
    p.add("global_atomic_add", ["v1", "v2", "s[0:1]", "sc0"])  # returning: a ticket
    p.add("s_endpgm")
    assert ch.check_drain("k", p.ins) == []
    p = Prog()
    p.add("global_store_dwordx2", ["v[0:1]", "v[2:3]", "off", "sc1"])
    p.add("global_atomic_add", ["v1", "v2", "s[0:1]"])  # fire-and-forget arrival
    p.add("s_endpgm")
    assert len(ch.check_drain("k", p.ins)) == 1


def test_undrained_branch_arm():
    # if (c) { store } ; signal -- the taken arm skips nothing, the store arm
    # reaches the signal undrained
    p = Prog()
    br = p.add("s_cbranch_scc1", ["x"], None)
    p.add(*STORE)
    join = p.label()
    p.add(*FLAG)
    p.add("s_endpgm")
    p.ins[br // 8] = (br, "s_cbranch_scc1", ["x"], join)
    assert len(ch.check_drain("k", p.ins)) == 1
    # drained in the store arm: fine
    p = Prog()
    br = p.add("s_cbranch_scc1", ["x"], None)
    p.add(*STORE)
    p.add(*DRAIN)
    join = p.label()
    p.add(*FLAG)
    p.add("s_endpgm")
    p.ins[br // 8] = (br, "s_cbranch_scc1", ["x"], join)
    assert ch.check_drain("k", p.ins) == []


def test_loop_back_edge():
    # loop { signal ; store } -- the second iteration's signal follows the
    # first iteration's store without a drain
    p = Prog()
    head = p.label()
    p.add(*FLAG)
    p.add(*STORE)
    p.add("s_cbranch_scc1", ["x"], head)
    p.add("s_endpgm")
    assert len(ch.check_drain("k", p.ins)) == 1
    p = Prog()
    head = p.label()
    p.add(*DRAIN)
    p.add(*FLAG)
    p.add(*STORE)
    p.add("s_cbranch_scc1", ["x"], head)
    p.add("s_endpgm")
    assert ch.check_drain("k", p.ins) == []


def test_exempt_atomics():
    p = Prog()
    p.add(*STORE)
    p.add("global_atomic_or", ["v1", "v2", "s[0:1]"])    # stall_set: give-up path
    p.add("global_atomic_swap", ["v1", "v2", "s[0:1]"])  # ctl_reset / ctl_record
    p.add(*DRAIN)
    p.add(*FLAG)
    p.add("s_endpgm")
    assert ch.check_drain("k", p.ins) == []


def test_one_l2_rules():
    p = Prog()
    p.add("s_getreg_b32", ["s2", "hwreg(HW_REG_XCC_ID", "0", "4)"])
    p.add("buffer_load_dwordx4", ["v[0:3]", "v4", "s[0:3]", "0 offen sc1"])
    p.add("global_load_dword", ["v5", "v6", "s[8:9]", "sc1"])
    p.add("s_endpgm")
    assert ch.check_one_l2("k", p.ins, True) == []
    p.ins[1] = (8, "buffer_load_dwordx4", ["v[0:3]", "v4", "s[0:3]", "0 offen"], None)
    assert len(ch.check_one_l2("k", p.ins, True)) == 1
    p.ins[0] = (0, "s_nop", ["0"], None)
    assert len(ch.check_one_l2("k", p.ins, False)) == 2
