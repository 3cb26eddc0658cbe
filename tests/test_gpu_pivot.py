"""GPU parity of the candidate-set pivot order (tg_pivoted_factor_complement
with nc = 0, i.e. greedy diagonal pivoting on H_k = H) against the numpy
restatement of dgeqp3's rule (tests/test_complement_math.pivoted_cholesky).

The cases are sized above the candidate count (1024) so the selection path
runs, and shaped to hit its edge cases:
  generic  random Gram matrix;
  ties     every column duplicated: exact ties on the Schur diagonal, broken by
           dgeqp3 position;
  groups   groups of 8 near-identical heavy columns: one pivot per group knocks
           its 7 siblings to the bottom, so candidates run out against the
           bound of the non-candidates and panels end early (re-selection);
  full     k = n, n not a multiple of the 64-row tiles: the compacted Schur
           complement shrinks to its last partial tiles.
Bars: perm identical; R_x relative Frobenius <= 1e-10.
"""
import numpy as np
import pytest
import torch

from test_complement_math import pivoted_cholesky

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(kind, rng):
    if kind == "generic":
        n, k = 1536, 1200
        X = rng.standard_normal((2000, n))
    elif kind == "ties":
        n, k = 1280, 500
        B = rng.standard_normal((900, n // 2))
        X = np.repeat(B, 2, axis=1)
    elif kind == "full":
        n, k = 1300, 1300
        X = rng.standard_normal((1700, n))
    else:  # groups
        ng, g, nsmall = 150, 8, 1000
        base = 10.0 * rng.standard_normal((1500, ng))
        heavy = np.repeat(base, g, axis=1) + 1e-3 * rng.standard_normal((1500, ng * g))
        small = rng.standard_normal((1500, nsmall))
        X = np.concatenate([heavy, small], axis=1)
        X = X[:, rng.permutation(X.shape[1])]
        n, k = X.shape[1], 450
    H = X.T @ X / X.shape[0]
    return H, k


@pytest.mark.parametrize("kind", ["generic", "ties", "groups", "full"])
def test_pivot_order_candidate_sets(kind):
    from gptq_svd_amd import _lib as lib
    rng = np.random.default_rng(7)
    H, k = _case(kind, rng)
    n = H.shape[0]
    Hd = torch.from_numpy(H).to(DEV)
    perm = torch.empty(n, dtype=torch.int64, device=DEV)
    Rx = torch.empty((k, n), dtype=torch.float64, device=DEV)
    ws = lib.workspace(lib.lib.tg_pivot_workspace_size(n, k), torch.device(DEV))
    lib.call("tg_pivoted_factor_complement", lib.stream(), lib.ptr(Hd), n, None, n, None, 0, n, k,
             lib.ptr(perm), lib.ptr(Rx), n, lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    order, Rx_ref = pivoted_cholesky(H, k)
    p = perm.cpu().numpy()
    assert np.array_equal(p[:k], order[:k]), f"first mismatch at {np.argmax(p[:k] != order[:k])}"
    assert np.array_equal(p, order), "dgeqp3 tail order differs"
    err = np.linalg.norm(Rx.cpu().numpy() - Rx_ref) / np.linalg.norm(Rx_ref)
    assert err <= 1e-10, err
