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
