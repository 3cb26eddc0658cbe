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


def all_gather_cols(t: torch.Tensor, m: int, pg=None) -> torch.Tensor:
    """Concatenate per-rank column shards (widths from shard_rows(m, ...))
    along dim 1."""
    world, _ = _world(pg)
    if world == 1:
        return t
    return all_gather_rows(t.t().contiguous(), m, pg).t().contiguous()


class UrxHip:
    """The column-sharded pieces of the complement-path U factor on this
    process's GPU (include/truncgptq.h tg_urx_c / tg_urx_u11 / tg_urx_u12)."""

    def __init__(self):
        from . import _lib
        self.L = _lib

    def small_m(self, k: int, m: int) -> bool:
        import os
        e = os.environ.get("TG_URX_SMALLM")  # the library's switch (factor.hip urx_small_m)
        return e == "1" if e is not None else m * 16 <= k

    def _ws(self, n, k, dev):
        return self.L.workspace(self.L.lib.tg_ufactor_rx_workspace_size(n, k), dev)

    def full(self, Rx: torch.Tensor, n: int, k: int) -> torch.Tensor:
        L = self.L
        U = torch.empty((k, n), dtype=torch.float64, device=Rx.device)
        ws = self._ws(n, k, Rx.device)
        L.call("tg_u_factor_rx", L.stream(), L.ptr(Rx), Rx.stride(0), n, k, L.ptr(U), n, L.ptr(ws),
               ws.numel())
        return U

    def c_cols(self, Rx, n, k, c0, c1):
        L = self.L
        C = torch.empty((k, max(c1 - c0, 1)), dtype=torch.float64, device=Rx.device)
        ws = self._ws(n, k, Rx.device)
        L.call("tg_urx_c", L.stream(), L.ptr(Rx), Rx.stride(0), n, k, c0, c1, L.ptr(C),
               C.stride(0), L.ptr(ws), ws.numel())
        return C[:, : c1 - c0]

    def u11(self, Rx, n, k, C):
        L = self.L
        C = C.contiguous()
        U = torch.zeros((k, n), dtype=torch.float64, device=Rx.device)
        ws = self._ws(n, k, Rx.device)
        L.call("tg_urx_u11", L.stream(), L.ptr(Rx), Rx.stride(0), n, k, L.ptr(C),
               max(C.stride(0), 1), L.ptr(U), n, L.ptr(ws), ws.numel())
        return U

    def u12(self, U, k, Cb):
        L = self.L
        Cb = Cb.contiguous()
        w = Cb.shape[1]
        out = torch.empty((k, max(w, 1)), dtype=torch.float64, device=U.device)
        L.call("tg_urx_u12", L.stream(), L.ptr(U), U.stride(0), k, L.ptr(Cb), max(Cb.stride(0), 1),
               w, L.ptr(out), out.stride(0))
        return out[:, :w]


def u_factor_rx_sharded(Rx: torch.Tensor, n: int, k: int, pg=None, ops=None) -> torch.Tensor:
    """The complement-path U factor (tg_u_factor_rx, gptq_utils.py:118-124's
    QR) with its column-parallel work split over the ranks of `pg`: rank r
    forms C[:, cols_r] = R11^-1 R12[:, cols_r] (block back substitution), the
    ranks all-gather C, every rank forms U11 = V^-1 from it (one k x k
    Cholesky, replicated), rank r its U12 columns V^-1 C[:, cols_r], and the
    ranks all-gather U12.  Every C / U12 column depends on its own input
    column only, so U equals the one-process factor bit for bit
    (tests/test_gpu_urx_sharded.py on the HIP path, tests/test_dist_urx.py on
    gloo).  Collectives: two all-gathers of k x m doubles (1.2 GB each at
    Llama-3-70B down_proj width with k = 21,402).  The small-m form (m * 16 <=
    k: near-full-rank layers, where C is a sliver) and world size 1 run the
    one-process call.  `ops`: the per-process pieces (default: UrxHip)."""
    world, rank = _world(pg)
    ops = ops if ops is not None else UrxHip()
    m = n - k
    if m <= 0 or ops.small_m(k, m):
        return ops.full(Rx, n, k)
    c0, c1 = shard_rows(m, world, rank)
    C = all_gather_cols(ops.c_cols(Rx, n, k, c0, c1), m, pg)
    U = ops.u11(Rx, n, k, C)
    U[:, k:] = all_gather_cols(ops.u12(U, k, C[:, c0:c1]), m, pg)
    return U
