"""GPU: the column-sharded pieces of the complement-path U factor
(tg_urx_c / tg_urx_u11 / tg_urx_u12, gptq_svd_amd.dist.u_factor_rx_sharded)
reproduce tg_u_factor_rx's explicit form bit for bit when the m = n - k
columns are split over (simulated) ranks: every C = R11^-1 R12 and U12 =
V^-1 C column depends on its own input column only.  Shapes: even and odd
k / m (R12's rows and C's ld unaligned), splits into 3 and 8 blocks, one
block of a single column, and the world-size-1 call of the dist helper."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rx(n, k, seed):
    """R_x-like factor: the R of a k x n Gaussian matrix (positive diagonal),
    conditioned like a real R_x (a random triangle is exponentially worse)"""
    rng = np.random.default_rng(seed)
    R = np.linalg.qr(rng.standard_normal((k, n)), mode="r")
    R = np.sign(np.diag(R))[:, None] * R
    return torch.from_numpy(R).to(DEV)


@pytest.mark.parametrize("n,k,world", [(1536, 1100, 3), (1500, 1001, 8), (1200, 1000, 3)])
def test_column_blocks_match_one_call(n, k, world):
    from gptq_svd_amd import _lib as L
    from gptq_svd_amd.dist import UrxHip, shard_rows
    Rx = _rx(n, k, n + k)
    m = n - k
    assert m * 16 > k  # the explicit form (the small-m form is not sharded)
    ops = UrxHip()
    ref = ops.full(Rx, n, k)
    blocks = [shard_rows(m, world, r) for r in range(world)]
    C = torch.cat([ops.c_cols(Rx, n, k, c0, c1) for c0, c1 in blocks], dim=1)
    U = ops.u11(Rx, n, k, C)
    U[:, k:] = torch.cat([ops.u12(U, k, C[:, c0:c1]) for c0, c1 in blocks], dim=1)
    torch.cuda.synchronize()
    assert torch.equal(U, ref)
    # one column on its own
    c1 = ops.c_cols(Rx, n, k, m // 2, m // 2 + 1)
    assert torch.equal(c1[:, 0], C[:, m // 2])
    del L


def test_dist_helper_world_one():
    from gptq_svd_amd.dist import UrxHip, u_factor_rx_sharded
    n, k = 1536, 1100
    Rx = _rx(n, k, 5)
    assert torch.equal(u_factor_rx_sharded(Rx, n, k), UrxHip().full(Rx, n, k))
