"""SYRK (A1) kernel timing (development tool): the 16-bit stream-K SYRK
(tg_syrk_accum_ws) with X 16-bit in LDS (TG_SYRK_LDS64=0) and with X
converted to FP64 at staging (the default), at the harness's batch (32 x 2048 =
65,536 rows), n = 4096 and 12,288 by default.  Prints kernel TF/s (flops of
the lower 128-tiles), the fraction of the FP64 MFMA peak, and the largest
difference between the two kernels' H relative to max |H|.
    python tools/syrk_time.py [n ...]            (REPS=4, GENERIC=1 adds the
                                                  generic FP64 GEMM path;
                                                  TG_SYRK_NC = tail chunks)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402
from gptq_svd_amd import _lib  # noqa: E402

dev = "cuda:0"
reps = int(os.environ.get("REPS", "4"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for n in [int(a) for a in sys.argv[1:]] or [4096, 12288]:
    rows = int(os.environ.get("ROWS", "65536"))
    torch.manual_seed(0)
    X = torch.randn(rows, n, device=dev).half()
    nt = -(-n // 128)
    flops = 2.0 * rows * (nt * (nt + 1) // 2) * 128 * 128
    Hs = {}
    for mode in ("0", "1"):
        os.environ["TG_SYRK_LDS64"] = mode
        acc = g.HessianAccumulator(n, dev)
        acc.add_batch(X)
        Hs[mode] = acc.H.clone()
        dt = timed(lambda: acc.add_batch(X))
        name = "fp64 in LDS" if mode == "1" else "16-bit in LDS"
        print(f"n={n} {name}: {dt * 1e3:.2f} ms/call, {flops / dt / 1e12:.1f} TF/s "
              f"({flops / dt / 1e12 / 78.6:.3f} of FP64 MFMA peak)", flush=True)
        del acc
    os.environ.pop("TG_SYRK_LDS64")
    d = (Hs["0"] - Hs["1"]).abs().max().item() / Hs["0"].abs().max().item()
    print(f"n={n}: max |H16 - H64| / max |H| = {d:.2e}, symmetric: "
          f"{bool(torch.equal(Hs['1'], Hs['1'].T))}", flush=True)
    if os.environ.get("GENERIC"):
        H = torch.zeros(n, n, dtype=torch.float64, device=dev)
        dt = timed(lambda: _lib.call("tg_syrk_accum", _lib.stream(), _lib.ptr(X), _lib.TG_F16,
                                     rows, n, n, _lib.ptr(H), n))
        print(f"n={n} generic: {dt * 1e3:.2f} ms/call, {flops / dt / 1e12:.1f} TF/s", flush=True)
    del X, Hs
    torch.cuda.empty_cache()
