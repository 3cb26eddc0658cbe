"""GPU check of tg_eigh_vectors_range for a few dropped eigenpairs (the
complement path's request: count ~ 1-50 starting at k), on the two-stage
eigensolver, including a range ending at the last eigenvector.

Bars (as tests/test_gpu_solver.py::test_eigh): residual ||H v - lambda v|| <=
1e-10 ||H||, orthogonality <= 1e-10, and agreement with LAPACK's eigenvectors
up to sign where the eigenvalue gap is large.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("n,first,count", [(600, 0, 14), (2048, 1500, 14), (2048, 0, 48),
                                           (4100, 3058, 14), (4100, 4099, 1)])
def test_few_vectors(n, first, count):
    from gptq_svd_amd import _lib as lib
    rng = np.random.default_rng(n + first)
    X = rng.standard_normal((3 * n // 2, n))
    H = X.T @ X / X.shape[0]
    A = torch.from_numpy(H).to(DEV)
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), torch.device(DEV))
    w = torch.empty(n, dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    V = torch.empty((count, n), dtype=torch.float64, device=DEV)
    lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), first, count, lib.ptr(V), n,
             lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    Vh = V.cpu().numpy()
    lam_desc = w.cpu().numpy()[::-1]
    lam = lam_desc[first:first + count]
    nrm = np.abs(lam_desc).max()
    resid = np.linalg.norm(Vh @ H - lam[:, None] * Vh, axis=1).max()
    assert resid <= 1e-10 * nrm, resid
    orth = np.abs(Vh @ Vh.T - np.eye(count)).max()
    assert orth <= 1e-10, orth
    L, Q = np.linalg.eigh(H)
    Qd = Q[:, ::-1][:, first:first + count].T
    gaps = np.abs(np.diff(L[::-1]))
    for j in range(count):
        g = min(gaps[first + j - 1] if first + j > 0 else np.inf,
                gaps[first + j] if first + j < n - 1 else np.inf)
        if g > 1e-6 * nrm:
            assert abs(abs(Vh[j] @ Qd[j]) - 1.0) <= 1e-8
