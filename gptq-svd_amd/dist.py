"""Multi-GPU helpers (one process per GPU, torch.distributed over RCCL/xGMI).

The solver path shards two ways; neither needs a collective
inside the solve:

* independent layers / Hessians per rank (the synthetic 1/2/4/8-GPU bench):
  each rank solves its own problem, then ONE ``all_gather`` of the packed int32
  weights (``gather_packed``);
* row-sharded quantisation of one weight (``quantize_rows_sharded``): rows of
  W are independent given (U, perm, per-row scale/zero), so each rank
  quantises a contiguous row range and the dequantised rows / codes are
  gathered.  Results are identical to the single-GPU call, bit for bit.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def _world(pg):
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(pg), dist.get_rank(pg)


def shard_rows(m: int, world: int, rank: int) -> tuple[int, int]:
    """Balanced contiguous row range [r0, r1) of rank `rank`."""
    base, extra = divmod(m, world)
    r0 = rank * base + min(rank, extra)
    return r0, r0 + base + (1 if rank < extra else 0)


def _gloo(pg) -> bool:
    return dist.get_backend(pg) == "gloo"


def all_reduce_sum(t: torch.Tensor, pg=None) -> torch.Tensor:
    """SUM all-reduce; returns the result (device tensors go through the host
    under gloo, which has no device-side reduction here)."""
    world, _ = _world(pg)
    if world == 1:
        return t
    if t.is_cuda and _gloo(pg):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=pg)
        return h.to(t.device)
    t = t.contiguous()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
    return t


def gather_packed(t: torch.Tensor, pg=None) -> torch.Tensor:
    """all_gather of one equally-shaped tensor per rank -> (world, *shape)."""
    world, _ = _world(pg)
    if world == 1:
        return t.unsqueeze(0)
    t = t.contiguous()
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t, group=pg)
    return out.view((world,) + tuple(t.shape))


def all_gather_rows(t: torch.Tensor, m: int, pg=None) -> torch.Tensor:
    """Concatenate per-rank row shards (shapes from shard_rows) along dim 0."""
    world, _ = _world(pg)
    if world == 1:
        return t
    rows_max = max(shard_rows(m, world, r)[1] - shard_rows(m, world, r)[0] for r in range(world))
    dev = t.device
    if t.is_cuda and _gloo(pg):
        t = t.cpu()
    pad = torch.zeros((rows_max,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=pg)
    parts = []
    for r in range(world):
        r0, r1 = shard_rows(m, world, r)
        parts.append(bufs[r][: r1 - r0])
    return torch.cat(parts, dim=0).to(dev)


def quantize_rows_sharded(W: torch.Tensor, U: torch.Tensor, perm: torch.Tensor, w_bits: int,
                          group_size: int, sym: bool, block_size: int = 1024, pg=None,
                          fn: Optional[Callable] = None):
    """Row-sharded gptq_fwrd: returns (dequantised W, codes) gathered on every rank.

    `fn(W_rows, U, perm, w_bits, group_size, sym, block_size) -> (Wq_rows, codes_rows)`
    defaults to the HIP path (gptq_utils.gptq_fwrd on the local GPU)."""
    world, rank = _world(pg)
    m = W.shape[0]
    r0, r1 = shard_rows(m, world, rank)
    if fn is None:
        from .gptq_utils import Quantizer, gptq_fwrd

        def fn(Wl, U_, perm_, b, g, s, bs):
            q = Quantizer(b, g, s)
            Wq, _ = gptq_fwrd(Wl, U_, q, perm_, block_size=bs)
            return Wq, q.codes
    if r1 > r0:
        Wq, codes = fn(W[r0:r1], U, perm, w_bits, group_size, sym, block_size)
        # one dtype on every rank (an empty rank cannot ask fn): codes are < 2^8
        Wq, codes = Wq.to(W.dtype), codes.to(torch.uint8)
    else:
        # m < world: this rank owns no rows (the solver rejects m = 0) but
        # still joins both all_gathers, or the other ranks would block there
        n = W.shape[1]
        Wq = torch.empty((0, n), dtype=W.dtype, device=W.device)
        codes = torch.empty((0, n), dtype=torch.uint8, device=W.device)
    return all_gather_rows(Wq, m, pg), all_gather_rows(codes, m, pg)
