"""CPU multi-process (gloo, world_size 2) coverage of the multi-GPU path:
row sharding + gather is bit-identical to the single-process result, and the
packed-weight gather returns every rank's tensor in rank order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fn():
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as o

    def fn(Wl, U, perm, b, g, s, bs):
        Wq, _, codes = o.gptq_fwrd(Wl.numpy(), U.numpy(), perm.numpy(), b, g, s, bs, gemm="fma",
                                   impl="c", return_codes=True)
        return torch.from_numpy(Wq), torch.from_numpy(codes)
    return fn


def _worker(rank, world, port, W, U, perm, out):
    torch.set_num_threads(1)
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gptq_svd_amd.dist import gather_packed, quantize_rows_sharded
    Wq, codes = quantize_rows_sharded(W, U, perm, 4, 128, False, 256, fn=_oracle_fn())
    packed = gather_packed(torch.full((3, 5), rank, dtype=torch.int32))
    if rank == 0:
        out["Wq"] = Wq.numpy()
        out["codes"] = codes.numpy()
        out["packed"] = packed.numpy()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,m", [(2, 37), (3, 2)])
def test_row_sharded_matches_single(oracle_mod, world, m):
    """m < world included: a rank without rows still joins the gathers."""
    rng = np.random.default_rng(3)
    n, k = 512, 480
    W = (rng.standard_normal((m, n)) * 0.05).astype(np.float32)
    U = np.triu(rng.standard_normal((k, n)) * 0.02)
    U[np.arange(k), np.arange(k)] = 1.0 + np.abs(rng.standard_normal(k))
    U = U.astype(np.float32)
    perm = rng.permutation(n).astype(np.int64)
    ref, _, ref_codes = oracle_mod.gptq_fwrd(W, U, perm, 4, 128, False, 256, gemm="fma", impl="c",
                                             return_codes=True)
    manager = mp.Manager()
    out = manager.dict()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, torch.from_numpy(W), torch.from_numpy(U),
                            torch.from_numpy(perm), out), nprocs=world, join=True)
    assert np.array_equal(out["Wq"], ref)
    assert np.array_equal(out["codes"], ref_codes)
    packed = out["packed"]
    assert packed.shape == (world, 3, 5)
    assert all((packed[r] == r).all() for r in range(world))


def test_shard_rows_partition():
    from gptq_svd_amd.dist import shard_rows
    for m in (1, 7, 64, 4097):
        for world in (1, 2, 3, 8):
            ranges = [shard_rows(m, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
