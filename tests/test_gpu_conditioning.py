"""U factor under ill-conditioning (tg_u_factor, tg_u_factor_rx).

Both U paths form U from the Cholesky factor of a Gram matrix, which squares
the condition number relative to the reference's Householder QR
(gptq_utils.py:120).  The library guards it (factor.hip, "Conditioning
guard"): a breakdown or a large diagonal range of the first factor triggers
CholeskyQR refinement (shifted CholeskyQR3 after a breakdown); a factor that
still breaks down raises RuntimeError instead of returning NaN.

Bars: the s_ golden vectors (energy eps 1e-7, graded / cliff spectra, made
by the reference itself) -- k and perm identical, U within 1e-5 relative
Frobenius (their eigenvectors are determined to ~eps ||H|| / gap ~1e-7 by any
LAPACK; the north-star bar is 1e-3).  Direct factor tests against LAPACK
Householder QR of the same A: 1e-5 at cond(A) = 1e9 (breakdown of the plain
CholeskyQR), 1e-8 at cond(A) = 1e6.
"""
import numpy as np
import pytest
import scipy.linalg
import torch

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def g():
    import gptq_svd_amd.gptq_utils as g
    return g


@pytest.fixture(scope="module")
def lib():
    from gptq_svd_amd import _lib
    return _lib


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("refine", ["auto", "0", "1"])
@pytest.mark.parametrize("path", ["auto", "kept", "complement"])
@pytest.mark.parametrize("name", golden_names("s_"))
def test_spectrum_golden(g, name, path, refine, monkeypatch):
    monkeypatch.setenv("TG_SPECTRAL_PATH", path)
    if refine != "auto":
        monkeypatch.setenv("TG_U_REFINE", refine)
    d = load_golden(name)
    U, R_x, perm, S, k = g.truncated_spectral_factor(t(d["H"]), float(d["eps"]), str(d["method"]))
    taken = g.truncated_spectral_factor.last_path[0]
    if path == "auto" and name.startswith("s_n512_w4a_graded"):
        # dropped eigenvalues down to rounding level stay in H - B_c^T B_c:
        # the auto rule takes the exact kept path
        assert taken == "kept"
    assert k == int(d["k"])
    assert np.array_equal(perm.cpu().numpy(), d["perm"])
    assert rel(S.cpu().numpy(), d["S"]) < 1e-10
    err = rel(U.cpu().numpy(), d["U"])
    print(f"{name} {path}->{taken} refine={refine}: |U - U_ref| / |U_ref| = {err:.2e}")
    # the forced complement form on the graded spectrum is off by ~left/lambda_k
    # (~1e-13 / 1e-7, measured 2.2e-5): inside the 1e-3 bar, not the 1e-5 one
    forced_inexact = path == "complement" and name.startswith("s_n512_w4a_graded")
    assert err < (1e-4 if forced_inexact else 1e-5)
    assert rel(R_x.cpu().numpy(), d["Rx"]) < (1e-4 if forced_inexact else 1e-5)
    q = g.Quantizer(int(d["bits"]), int(d["group"]), bool(d["sym"]))
    Wq, _ = g.gptq_fwrd(t(d["W"]), U, q, perm, block_size=int(d["block_size"]))
    mism = float(np.mean(Wq.cpu().numpy() != d["final_W"]))
    print(f"   code mismatch vs reference {mism:.2e}")
    assert mism <= 2e-3


def factor_problem(n, k, s_hi, s_lo, seed):
    """Orthonormal Vh (k x n), S log-spaced s_hi .. s_lo (cond(A) = 10^(s_hi - s_lo)),
    perm and R_x from LAPACK dgeqp3 of diag(S) Vh, and the reference U =
    sign-normalised R of Householder QR(diag(1/S) Vh[:, perm])."""
    rng = np.random.default_rng(seed)
    Vh = np.linalg.qr(rng.standard_normal((n, n)))[0][:, :k].T.copy()
    S = np.logspace(s_hi, s_lo, k)
    _, Rx, perm = scipy.linalg.qr(S[:, None] * Vh, pivoting=True, mode="economic")
    Rx = Rx * np.sign(np.diag(Rx))[:, None]
    R = np.linalg.qr((1.0 / S)[:, None] * Vh[:, perm], mode="r")
    R = R * np.sign(np.diag(R))[:, None]
    return Vh, S, perm.astype(np.int64), Rx, R


def u_factor(lib, Vh, S, perm):
    k, n = Vh.shape
    U = torch.empty((k, n), dtype=torch.float64, device=DEV)
    ws = lib.workspace(lib.lib.tg_ufactor_workspace_size(n, k), DEV)
    dV, dS, dp = t(Vh), t(S), t(perm)
    lib.call("tg_u_factor", lib.stream(), lib.ptr(dV), n, lib.ptr(dS), lib.ptr(dp), n, k,
             lib.ptr(U), n, lib.ptr(ws), ws.numel())
    return U.cpu().numpy()


def u_factor_rx(lib, Rx):
    k, n = Rx.shape
    U = torch.empty((k, n), dtype=torch.float64, device=DEV)
    ws = lib.workspace(lib.lib.tg_ufactor_rx_workspace_size(n, k), DEV)
    dR = t(Rx)
    lib.call("tg_u_factor_rx", lib.stream(), lib.ptr(dR), n, n, k, lib.ptr(U), n, lib.ptr(ws),
             ws.numel())
    return U.cpu().numpy()


@pytest.mark.parametrize("refine", ["auto", "1"])
@pytest.mark.parametrize("n,k,s_hi,s_lo,tol", [(384, 320, 4.0, -5.0, 1e-5),   # plain breaks down
                                               (384, 320, 3.0, -3.0, 1e-8),
                                               (512, 256, 1.5, -2.0, 1e-10),
                                               (300, 300, 4.0, -4.0, 1e-8)])  # k = n
def test_u_factor_conditioning(lib, monkeypatch, refine, n, k, s_hi, s_lo, tol):
    if refine != "auto":
        monkeypatch.setenv("TG_U_REFINE", refine)
    Vh, S, perm, _, R = factor_problem(n, k, s_hi, s_lo, n + k)
    U = u_factor(lib, Vh, S, perm)
    assert np.all(np.isfinite(U))
    assert np.allclose(np.tril(U[:, :k], -1), 0.0)
    assert np.all(np.diag(U) > 0)
    err = rel(U, R)
    print(f"tg_u_factor n={n} k={k} cond=1e{s_hi - s_lo:g}: {err:.2e}")
    assert err < tol


@pytest.mark.parametrize("refine", ["auto", "1"])
@pytest.mark.parametrize("n,k,s_hi,s_lo,tol", [(384, 320, 4.0, -5.0, 1e-5),
                                               (384, 320, 3.0, -3.0, 1e-7),
                                               (512, 256, 1.5, -2.0, 1e-8),   # unrefined: 2.7e-9
                                               (300, 300, 4.0, -4.0, 1e-7)])
def test_u_factor_rx_conditioning(lib, monkeypatch, refine, n, k, s_hi, s_lo, tol):
    """Complement form U = R(QR(S^-1 R_x)), S = R_x R_x^T, against Householder
    QR of diag(1/S) Vh P (identity (ii))."""
    if refine != "auto":
        monkeypatch.setenv("TG_U_REFINE", refine)
    _, _, _, Rx, R = factor_problem(n, k, s_hi, s_lo, 7 * n + k)
    U = u_factor_rx(lib, Rx)
    assert np.all(np.isfinite(U))
    assert np.all(np.diag(U) > 0)
    err = rel(U, R)
    print(f"tg_u_factor_rx n={n} k={k} cond=1e{s_hi - s_lo:g}: {err:.2e}")
    assert err < tol


def test_u_factor_breakdown_raises(lib):
    """A factor that cannot be repaired raises instead of returning NaN."""
    Vh, S, perm, Rx, _ = factor_problem(128, 96, 1.0, -1.0, 5)
    Vh[3, 7] = np.nan
    with pytest.raises(RuntimeError, match="broke down"):
        u_factor(lib, Vh, S, perm)
    Rx = Rx.copy()
    Rx[2, 50] = np.nan
    with pytest.raises(RuntimeError, match="broke down"):
        u_factor_rx(lib, Rx)


def test_indefinite_h_takes_kept_path(g, oracle_mod):
    """A negative eigenvalue among the dropped ones (indefinite H) must not go
    through the complement form H - B_c^T B_c (which keeps it); the auto rule
    takes the kept path and reproduces the oracle's perm and U."""
    rng = np.random.default_rng(17)
    n = 256
    Q = np.linalg.qr(rng.standard_normal((n, n)))[0]
    lam = np.concatenate([np.linspace(0.1, 1.0, 230), np.logspace(-5, -4, 25), [-1e-3]])
    H = (Q * lam) @ Q.T
    H = (H + H.T) / 2
    U, R_x, perm, S, k = g.truncated_spectral_factor(t(H), 1e-4, "energy")
    assert g.truncated_spectral_factor.last_path[0] == "kept"
    f = oracle_mod.process_hessian_alt(H, 1e-4, "energy")
    assert k == f.k
    assert np.array_equal(perm.cpu().numpy(), f.perm)
    assert rel(U.cpu().numpy(), f.U) < 1e-8
