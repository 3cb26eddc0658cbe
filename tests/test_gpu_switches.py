"""Every path-selecting developer switch left in the library, on the GPU:
each alternative path must reproduce the default path on the same Hessian
(perm identical, U / R_x to 1e-10, the quantised weights bit-identical).
n = 2048 (rank 1536): large enough that the GEMMs take the 128-tile kernels
(TG_GEMM_IMPL=own selects the 4-wave one, TG_GEMM_TILE forces a tile) and
both spectral paths exist.  The switches are read per call."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def problem():
    import gptq_svd_amd.gptq_utils as g
    torch.manual_seed(5)
    n = 2048
    X = torch.randn(3 * n // 4, n).half().to(DEV)
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(X)
    H = acc.get_hessian()
    W = torch.randn(256, n, device=DEV)
    return g, H, W


def solve(g, H, W):
    U, R_x, perm, S, k = g.truncated_spectral_factor(H, 1e-4, "energy")
    q = g.Quantizer(4, 128, False)
    Wq, _ = g.gptq_fwrd(W, U, q, perm, block_size=1024)
    return dict(U=U.cpu().numpy(), R_x=R_x.cpu().numpy(), perm=perm.cpu().numpy(),
                Wq=Wq.cpu().numpy(), path=g.truncated_spectral_factor.last_path[0])


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("path", ["kept", "complement"])
@pytest.mark.parametrize("switches", [
    {"TG_PIVOT_OLD": "1"},
    {"TG_PIVOT_OLD": "1", "TG_PIVOT_STEPWISE": "1"},
    {"TG_INVIT_REG": "1"},
    {"TG_INVIT_REFACTOR": "1"},
    {"TG_BT_MULTI": "1"},
    {"TG_BT_Q2_WAVE": "1"},
    {"TG_URX_TWOCHOL": "1"},
    {"TG_GEMM_IMPL": "own"},
    {"TG_GEMM_TILE": "128"},
    {"TG_GEMM_TILE": "12864"},
    {"TG_GEMM_TILE": "64"},
    {"TG_GEMM_SWZ": "0", "TG_GEMM_TILE": "128"},
    {"TG_SB_PAIR": "1"},
    {"TG_SB_PAIR": "0"},
    {"TG_SB_PAIR": "1", "TG_XM_NBC": "2"},
    {"TG_SB_PAIR": "1", "TG_XM_NBC": "2", "TG_SB_PAIR_SIDE": "1"},
    {"TG_SYR2K_PERSIST": "0"},
    {"TG_SYR2K_PERSIST": "0", "TG_SB_PAIR": "1"},
    {"TG_XM_ASM": "0"},
    {"TG_XM_ASM": "0", "TG_XM_NBC": "2"},
    {"TG_XM_NBC": "2"},
    {"TG_XM_FUSE_W": "1"},
    {"TG_XM_KSPLIT": "1"},
    {"TG_XM_KSPLIT": "3"},
    {"TG_URX_SMALLM": "1"},
    {"TG_URX_INV": "1"},
    {"TG_SCHUR_MIRROR": "1"},
    {"TG_PIV_CC": "1"},
    {"TG_BT_Q2_LDS": "0"},
    {"TG_BT_Q1_LDS": "0"},
    {"TG_BT_TF_SIDE": "0"},
    {"TG_BT_SLABS": "0"},
    {"TG_CHOL_FUSED": "0"},
    {"TG_BISECT_NOGRID": "1"},
    {"TG_BISECT_CHUNK": "1"},
    {"TG_ORTH_MGS": "1"},
], ids=lambda d: "+".join(f"{k}={v}" for k, v in d.items()))
def test_switch_matches_default(problem, path, switches, monkeypatch):
    g, H, W = problem
    monkeypatch.setenv("TG_SPECTRAL_PATH", path)
    ref = solve(g, H, W)
    assert ref["path"] == path
    for k, v in switches.items():
        monkeypatch.setenv(k, v)
    got = solve(g, H, W)
    assert got["path"] == path
    assert np.array_equal(got["perm"], ref["perm"])
    assert rel(got["U"], ref["U"]) <= 1e-10
    assert rel(got["R_x"], ref["R_x"]) <= 1e-10
    mism = float(np.mean(got["Wq"] != ref["Wq"]))
    assert mism <= 1e-5, mism  # U agrees to ~1e-15: at most a rounding-tie flip


def test_small_m_u_factor_near_full_rank(monkeypatch):
    """A near-full-rank H (rows 2n, the real layers' case: k = n - m with m
    tiny) takes the small-m U factor by default (C = R11^-1 R12 by block back
    substitution, N = R11^T R11 by a triangular SYRK + a rank-2m term); U
    matches the explicit-inverse form (TG_URX_SMALLM=0) to 1e-10, perm and R_x
    identical."""
    import gptq_svd_amd.gptq_utils as g
    torch.manual_seed(7)
    n = 2048
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(torch.randn(2 * n, n).half().to(DEV))
    H = acc.get_hessian()
    W = torch.randn(128, n, device=DEV)
    monkeypatch.setenv("TG_SPECTRAL_PATH", "complement")
    got = solve(g, H, W)
    k = got["R_x"].shape[0]
    assert (n - k) * 16 <= k, k
    monkeypatch.setenv("TG_URX_SMALLM", "0")
    ref = solve(g, H, W)
    assert np.array_equal(got["perm"], ref["perm"])
    assert rel(got["R_x"], ref["R_x"]) == 0.0
    assert rel(got["U"], ref["U"]) <= 1e-10


def test_explicit_u_factor_odd_widths(monkeypatch):
    """The explicit-form U factor (m > k/16) with an odd rank and an odd
    complement (k = 1001, m = 499: R12's rows and C's ld are not 16-byte
    aligned, so Z's product runs on padded copies) against the explicit
    inverse form (TG_URX_INV=1): perm and R_x identical, U to 1e-10.  n = 1536
    (a whole number of 128-column groups), 1001 calibration rows."""
    import gptq_svd_amd.gptq_utils as g
    torch.manual_seed(8)
    n, rows = 1536, 1001
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(torch.randn(rows, n).half().to(DEV))
    H = acc.get_hessian()
    W = torch.randn(64, n, device=DEV)
    monkeypatch.setenv("TG_SPECTRAL_PATH", "complement")
    got = solve(g, H, W)
    k = got["R_x"].shape[0]
    assert k % 2 == 1 and (n - k) % 2 == 1 and (n - k) * 16 > k, k
    monkeypatch.setenv("TG_URX_INV", "1")
    ref = solve(g, H, W)
    assert np.array_equal(got["perm"], ref["perm"])
    assert rel(got["R_x"], ref["R_x"]) == 0.0
    assert rel(got["U"], ref["U"]) <= 1e-10
