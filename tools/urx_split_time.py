"""Time the column-sharded U-factor pieces (tg_urx_c / tg_urx_u11 /
tg_urx_u12, gptq_svd_amd.dist) against the one-call tg_u_factor_rx at a
config-5 width, for DESIGN.md section 6's bound (development tool).

usage: python tools/urx_split_time.py [N] [K] [WORLD]
Prints the one-call time, each piece over all m = N - K columns, the two
column pieces over one rank's block (m / WORLD columns), and checks that
the pieces reproduce the one-call U bit for bit.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd.dist import UrxHip, shard_rows  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 28672
k = int(sys.argv[2]) if len(sys.argv) > 2 else 21504
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
Rx = torch.randn(k, n, dtype=torch.float64, device=dev, generator=g) / n ** 0.5
Rx = torch.triu(Rx)
Rx.diagonal().copy_(1.0 + torch.rand(k, dtype=torch.float64, device=dev, generator=g))
m = n - k
ops = UrxHip()
assert not ops.small_m(k, m), "the explicit form is the sharded one"


def timed(f, reps=2):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best, out = None, None
    for _ in range(reps):
        out = None
        torch.cuda.synchronize()
        ev[0].record()
        out = f()
        ev[1].record()
        torch.cuda.synchronize()
        t = ev[0].elapsed_time(ev[1])
        best = t if best is None else min(best, t)
    return best, out


t_full, ref = timed(lambda: ops.full(Rx, n, k))
print(f"n={n} k={k} m={m}: tg_u_factor_rx {t_full:.1f} ms", flush=True)
t_c, C = timed(lambda: ops.c_cols(Rx, n, k, 0, m))
print(f"  tg_urx_c   all {m} columns: {t_c:.1f} ms", flush=True)
t_11, U = timed(lambda: ops.u11(Rx, n, k, C))
print(f"  tg_urx_u11 (replicated):   {t_11:.1f} ms", flush=True)
t_12, U12 = timed(lambda: ops.u12(U, k, C))
print(f"  tg_urx_u12 all columns:    {t_12:.1f} ms", flush=True)
U[:, k:] = U12
del U12
print(f"  pieces == one call: {bool(torch.equal(U, ref))}", flush=True)
del ref
c0, c1 = shard_rows(m, world, 0)
t_cb, Cb = timed(lambda: ops.c_cols(Rx, n, k, c0, c1))
t_12b, _ = timed(lambda: ops.u12(U, k, Cb))
print(f"  one rank of {world} ({c1 - c0} columns): tg_urx_c {t_cb:.1f} ms, tg_urx_u12 {t_12b:.1f} ms",
      flush=True)
gather = 2 * k * m * 8 * (world - 1) / world
print(f"  per rank at world {world}: {t_cb + t_11 + t_12b:.1f} ms compute + two all-gathers of "
      f"{gather / 1e9:.2f} GB received per rank (vs {t_full:.1f} ms on one GPU)", flush=True)
