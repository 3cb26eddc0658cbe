"""Time tg_eigh_vectors_range for the last K eigenpairs (the complement
path's request) under environment variants, interleaved rep by rep in one
process (development tool):
    N=4096,12288 K=16,24,43 REPS=6 python tools/few_time.py TG_BT_SLABS=1 TG_BT_SLABS=0 TG_BT_MULTI=1
Prints the median and min ms per (n, k, variant) and the largest difference
of each variant's vectors from the first variant's.  FIRST=f: eigenpairs
f .. f + k - 1 (descending) instead of the last k (FIRST=3058 at n = 4096 is
the bench's complement request: the smallest nonzero eigenvalues of the
rank-3072 H)."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402
from gptq_svd_amd import _lib as lib  # noqa: E402


def main(variants):
    dev = torch.device("cuda")
    reps = int(os.environ.get("REPS", "6"))
    for n in [int(x) for x in os.environ.get("N", "4096").split(",")]:
        torch.manual_seed(0)
        acc = g.HessianAccumulator(n, dev)
        rows = 3 * n // 4
        for r0 in range(0, rows, 16384):
            acc.add_batch(torch.randn(min(16384, rows - r0), n, device=dev).half())
        A = acc.get_hessian().double()
        del acc
        ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), dev)
        w = torch.empty(n, dtype=torch.float64, device=dev)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        torch.cuda.synchronize()
        for k in [int(x) for x in os.environ.get("K", "16").split(",")]:
            V = torch.empty((k, n), dtype=torch.float64, device=dev)
            first = int(os.environ["FIRST"]) if "FIRST" in os.environ else n - k
            times = {v: [] for v in variants}
            outs = {}
            for r in range(reps + 1):
                for v in variants:
                    saved = {}
                    for kv in v.split(","):
                        key, val = kv.split("=")
                        saved[key] = os.environ.get(key)
                        os.environ[key] = val
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    lib.call("tg_eigh_vectors_range", lib.stream(), n, lib.ptr(w), first, k,
                             lib.ptr(V), n, lib.ptr(ws), ws.numel())
                    torch.cuda.synchronize()
                    if r:
                        times[v].append((time.perf_counter() - t0) * 1e3)
                    else:
                        outs[v] = V.cpu().numpy()
                    for key, val in saved.items():
                        if val is None:
                            os.environ.pop(key, None)
                        else:
                            os.environ[key] = val
            ref = outs[variants[0]]
            for v in variants:
                d = float(np.abs(np.abs(outs[v]) - np.abs(ref)).max())
                print(f"n={n} k={k} {v}: median {statistics.median(times[v]):.3f} ms, "
                      f"min {min(times[v]):.3f} ms, max|dV| {d:.2e}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["TG_BT_SLABS=1"])
