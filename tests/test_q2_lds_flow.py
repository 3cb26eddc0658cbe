"""tools/q2_lds_sim.py: the LDS-resident Q2 back-transform's data flow
(csrc/backtr.hip q2_lds_kernel -- waits, ring slots, write-through hand-offs
between workgroups) reproduces the level-by-level block order exactly under
random wave interleavings, and the model does see a broken flow (the first
draft's missing last-row carry).  CPU only."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import q2_lds_sim as sim  # noqa: E402


@pytest.mark.parametrize("n,seed", [(64, 0), (600, 1), (1025, 2)])
def test_flow_matches_level_order(n, seed):
    assert sim.run(n, 2, seed) == 0.0


def test_model_catches_missing_carry():
    assert sim.run(600, 2, 0, buggy=True) > 1.0
