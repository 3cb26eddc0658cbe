"""GPU checks of the band reduction's three panel factorisations
(gptq-svd_amd/csrc/pqr.hip, band.hip) against LAPACK on the same matrices:

* default: one compact-WY block per panel from CholeskyQR2 + Householder
  reconstruction (falls back per panel when the Gram matrix cannot certify Q);
* TG_PQR_FALLBACK=1: every panel through the in-kernel grid Householder path;
* TG_SB_TSQR=1: the TSQR tree of 256-row leaves (also the path past n = 65,536).

Inputs cover a Wishart matrix, a graded spectrum (1e-10 .. 1), a rank-deficient
X^T X (N < n: the late panels are numerically zero) and a block-diagonal
matrix (exactly zero panels).  Bars as tests/test_gpu_solver.py::test_eigh:
eigenvalues <= 1e-12 ||H||, residual <= 1e-10 ||H||, orthogonality <= 1e-10
(1e-8 for the graded spectrum's 1e-10-wide cluster).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _matrix(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "wishart":
        X = rng.standard_normal((3 * n // 2, n))
        return X.T @ X / X.shape[0]
    if kind == "lowrank":
        X = rng.standard_normal((3 * n // 4, n))
        return X.T @ X / X.shape[0]
    if kind == "graded":
        Q = np.linalg.qr(rng.standard_normal((n, n)))[0]
        return (Q * np.logspace(-10, 0, n)) @ Q.T
    if kind == "blockdiag":
        H = np.zeros((n, n))
        nb = n // 2
        X = rng.standard_normal((nb * 2, nb))
        H[:nb, :nb] = X.T @ X / X.shape[0]
        H[nb:, nb:] = np.diag(np.linspace(0.1, 3.0, n - nb))
        return H
    raise ValueError(kind)


@pytest.mark.parametrize("mode", ["default", "fallback", "tsqr"])
@pytest.mark.parametrize("kind,n", [("wishart", 700), ("lowrank", 1024), ("graded", 512),
                                    ("blockdiag", 600), ("wishart", 2100)])
def test_band_reduction_modes(mode, kind, n, monkeypatch):
    from gptq_svd_amd import _lib as lib
    if mode == "fallback":
        monkeypatch.setenv("TG_PQR_FALLBACK", "1")
    elif mode == "tsqr":
        monkeypatch.setenv("TG_SB_TSQR", "1")
    H = _matrix(kind, n, n + len(kind))
    A = torch.from_numpy(H).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    w = torch.empty(n, dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    count = min(n, 64)
    V = torch.empty((count, n), dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), 0, count, lib.ptr(V), n,
             lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    ref = np.linalg.eigvalsh(H)
    nrm = np.abs(ref).max()
    err = np.abs(w.cpu().numpy() - ref).max()
    assert err <= 1e-12 * nrm, (mode, kind, err / nrm)
    Vh = V.cpu().numpy()
    lam = w.cpu().numpy()[::-1][:count]
    resid = np.linalg.norm(Vh @ H - lam[:, None] * Vh, axis=1).max()
    assert resid <= 1e-10 * nrm, (mode, kind, resid / nrm)
    orth = np.abs(Vh @ Vh.T - np.eye(count)).max()
    assert orth <= (1e-8 if kind == "graded" else 1e-10), (mode, kind, orth)
