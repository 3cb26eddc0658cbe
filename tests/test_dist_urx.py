"""CPU multi-process (gloo, world size 2 and 3) coverage of the column-sharded
complement-path U factor (gptq_svd_amd.dist.u_factor_rx_sharded; the
multi-GPU split of tg_u_factor_rx for config 5's n = 28,672 layers).

The per-process pieces run as a numpy stand-in of the library's explicit form
(C = R11^-1 R12 column by column, Z^T = R11 + R12 C^T, N = Z Z^T, the upper
Cholesky of J N J, U11 = V^-1, U12 = U11 C): the gathered U of every world
size equals the one-process U bit for bit, and U is the R factor of
QR(S^-1 R_x), S = R_x R_x^T (gptq_utils.py:118-124 through the identity in
csrc/factor.hip), to 1e-8.  The HIP pieces' column independence is
tests/test_gpu_urx_sharded.py."""
import os
import socket

import numpy as np
import pytest
import scipy.linalg as sl
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


class UrxNumpy:
    """numpy stand-in of dist.UrxHip (same arguments and shapes)."""

    def small_m(self, k, m):
        return False

    def full(self, Rx, n, k):
        raise AssertionError("the sharded path must not fall back here")

    def c_cols(self, Rx, n, k, c0, c1):
        R = Rx.numpy()
        out = np.empty((k, c1 - c0))
        for j in range(c0, c1):  # column by column: independent of the split
            out[:, j - c0] = sl.solve_triangular(R[:, :k], R[:, k + j])
        return torch.from_numpy(out)

    def u11(self, Rx, n, k, C):
        R = Rx.numpy()
        ZT = R[:, :k] + R[:, k:] @ C.numpy().T
        N = ZT.T @ ZT
        Rc = np.linalg.cholesky(N[::-1, ::-1]).T           # J N J = Rc^T Rc
        U = np.zeros((k, n))
        U[:, :k] = np.linalg.inv(Rc).T[::-1, ::-1]           # V^-1 = J Rc^-T J
        return torch.from_numpy(U)

    def u12(self, U, k, Cb):
        U11, Cn = U.numpy()[:, :k], Cb.numpy()
        out = np.empty((k, Cn.shape[1]))
        for j in range(Cn.shape[1]):
            out[:, j] = U11 @ Cn[:, j]
        return torch.from_numpy(out)


def _rx(n, k, seed):
    """R_x-like factor: the R of a k x n Gaussian matrix (positive diagonal),
    conditioned like a real R_x (a random triangle is exponentially worse)"""
    rng = np.random.default_rng(seed)
    R = np.linalg.qr(rng.standard_normal((k, n)), mode="r")
    R = np.sign(np.diag(R))[:, None] * R
    return R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, Rx, n, k, out):
    torch.set_num_threads(1)
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gptq_svd_amd.dist import u_factor_rx_sharded
    U = u_factor_rx_sharded(torch.from_numpy(Rx), n, k, ops=UrxNumpy())
    if rank == 0:
        out["U"] = U.numpy()
    else:
        out[f"U{rank}"] = U.numpy()
    dist.barrier()
    dist.destroy_process_group()


def _sharded(world, Rx, n, k):
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        mp.start_processes(_worker, args=(world, _free_port(), Rx, n, k, out), nprocs=world,
                           join=True, start_method="spawn")
        return dict(out)


@pytest.mark.parametrize("world,n,k", [(2, 96, 70), (3, 96, 70), (3, 40, 37)])
def test_sharded_u_bit_identical(world, n, k):
    """(3, 40, 37): m = 3 columns over 3 ranks, one each."""
    import sys
    sys.path.insert(0, ROOT)
    from gptq_svd_amd.dist import u_factor_rx_sharded
    Rx = _rx(n, k, n + k)
    ref = u_factor_rx_sharded(torch.from_numpy(Rx), n, k, ops=UrxNumpy()).numpy()
    got = _sharded(world, Rx, n, k)
    for r in range(world):
        U = got["U" if r == 0 else f"U{r}"]
        assert np.array_equal(U, ref), r  # every rank holds the same U
    # U is the R factor of QR(S^-1 R_x), S = R_x R_x^T (positive diagonal)
    A = np.linalg.solve(Rx @ Rx.T, Rx)
    Rq = np.linalg.qr(A, mode="r")
    Rq = np.sign(np.diag(Rq))[:, None] * Rq
    assert np.abs(ref - Rq).max() <= 1e-8 * np.abs(Rq).max()  # the U bar of test_gpu_solver


def test_column_shards_cover_once():
    from gptq_svd_amd.dist import shard_rows
    for m in (0, 1, 3, 7270):
        for world in (1, 2, 3, 8):
            cols = [shard_rows(m, world, r) for r in range(world)]
            assert cols[0][0] == 0 and cols[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(cols, cols[1:]))
