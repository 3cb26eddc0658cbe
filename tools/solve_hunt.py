"""Run-to-run reproducibility of whole solves at the bench and large widths
(development tool): process_hessian_alt on one synthetic H per width (the
bench's recipe: 3n/4 fp16 rows through HessianAccumulator) REPS times,
(perm, R_x, U) compared on the device with the first solve.  Prints the
number of differing solves per width.
    N=4096,12288 REPS=300,30 python tools/solve_hunt.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402

dev = torch.device("cuda")
ns = [int(x) for x in os.environ.get("N", "4096,12288").split(",")]
reps = [int(x) for x in os.environ.get("REPS", "300,30").split(",")]
for n, r in zip(ns, reps):
    torch.manual_seed(1)
    acc = g.HessianAccumulator(n, dev)
    rows = 3 * n // 4
    for r0 in range(0, rows, 16384):
        acc.add_batch(torch.randn(min(16384, rows - r0), n, device=dev).half())
    H = acc.get_hessian()
    del acc
    ref = None
    bad = 0
    t0 = time.time()
    for i in range(r):
        R, R_x, perm = g.process_hessian_alt(H, 1e-4, "energy")
        if ref is None:
            ref = (R.clone(), R_x.clone(), perm.clone())
            continue
        same = (R.shape == ref[0].shape and torch.equal(perm, ref[2]) and torch.equal(R, ref[0])
                and torch.equal(R_x, ref[1]))
        if not same:
            bad += 1
            print(f"  n={n} solve {i}: differs (k {R.shape[0]} vs {ref[0].shape[0]}, perm equal "
                  f"{R.shape == ref[0].shape and torch.equal(perm, ref[2])})", flush=True)
        if i % 50 == 0:
            print(f"  n={n} solve {i} ({time.time() - t0:.0f} s)", flush=True)
    print(f"n={n}: {bad} of {r - 1} solves differ ({time.time() - t0:.0f} s)", flush=True)
