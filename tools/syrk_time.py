"""SYRK (A1) kernel timing: the 16-bit stream-K SYRK (tg_syrk_accum_ws) vs
the generic FP64 GEMM path (tg_syrk_accum), at the harness's batch
(32 x 2048 = 65,536 rows) for n = 4096 and 12,288.  Prints kernel TF/s
(flops of the lower 128-tiles) and the fraction of the FP64 MFMA peak."""
import sys
import time

import torch

sys.path.insert(0, ".")
import gptq_svd_amd.gptq_utils as g  # noqa: E402
from gptq_svd_amd import _lib  # noqa: E402

dev = "cuda:0"
for n in [int(a) for a in sys.argv[1:]] or [4096, 12288]:
    rows = 65536
    X = torch.randn(rows, n, device=dev).half()
    nt = -(-n // 128)
    flops = 2.0 * rows * (nt * (nt + 1) // 2) * 128 * 128
    acc = g.HessianAccumulator(n, dev)
    for name, fn in (("stream-K 16-bit", lambda: acc.add_batch(X)),
                     ("generic", lambda: _lib.call("tg_syrk_accum", _lib.stream(), _lib.ptr(X),
                                                   _lib.TG_F16, rows, n, n, _lib.ptr(acc.H), n))):
        fn()
        torch.cuda.synchronize()
        reps = 4
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"n={n} {name}: {dt * 1e3:.2f} ms/call, {flops / dt / 1e12:.1f} TF/s "
              f"({flops / dt / 1e12 / 78.6:.3f} of FP64 MFMA peak)", flush=True)
    del X, acc
    torch.cuda.empty_cache()

if __import__("os").environ.get("TG_SYRK_STAMPS"):
    # per-workgroup spread of one call (the library wrote {start, end, xcc} per
    # workgroup after the partial tiles; 100 MHz clock)
    import numpy as np
    for n in [int(a) for a in sys.argv[1:]] or [4096, 12288]:
        rows = 65536
        X = torch.randn(rows, n, device=dev).half()
        acc = g.HessianAccumulator(n, dev)
        acc.add_batch(X)
        acc.add_batch(X)
        torch.cuda.synchronize()
        G = (acc._ws.numel() // 8 - 64) // (4 * 128 * 128 + 3)  # G x 4 partial tiles
        off = (G * 4 * 128 * 128 + 64) * 8
        st = acc._ws[off:off + 24 * G].view(torch.int64).cpu().numpy().reshape(G, 3)
        t0 = st[:, 0].min()
        s, e, x = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, st[:, 2]
        d = e - s
        print(f"n={n}: G={G}, start spread {s.max():.1f} us, end min/median/max "
              f"{e.min():.0f}/{np.median(e):.0f}/{e.max():.0f} us, duration min/median/max "
              f"{d.min():.0f}/{np.median(d):.0f}/{d.max():.0f} us")
        print("  per XCD median duration (us):",
              [round(float(np.median(d[x == i])), 0) for i in range(8) if (x == i).any()])
        order = np.argsort(d)
        print("  slowest workgroups:", [(int(i), round(float(d[i])), int(x[i])) for i in order[-6:]])
