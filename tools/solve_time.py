"""One synthetic layer of width n (H from ROWS x n fp16 rows, default 3n/4 as
the bench's large_n extras; ROWS=2 gives a full-rank H like a real layer's) through process_hessian_alt + quantize, REPS times
(development tool: run plain or under rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402

n = int(os.environ.get("N", "12288"))
reps = int(os.environ.get("REPS", "2"))
rows = int(float(os.environ.get("ROWS", "0.75")) * n)  # calibration rows (x n)
dev = torch.device("cuda")
torch.manual_seed(1)
acc = g.HessianAccumulator(n, dev)
xf32 = os.environ.get("XF32") == "1"  # fp32 rows: the generic (not the 16-bit) SYRK
for r0 in range(0, rows, 16384):
    x = torch.randn(min(16384, rows - r0), n, device=dev).half()
    acc.add_batch(x.float() if xf32 else x)
H = acc.get_hessian()
del acc
W = torch.randn(4096, n, device=dev)
for r in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    R, R_x, perm = g.process_hessian_alt(H, 1e-4, "energy")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    q = g.Quantizer(4, 128, False)
    g.gptq_fwrd(W, R, q, perm, block_size=1024)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n} k={R.shape[0]}: factor {1e3 * (t1 - t0):.1f} ms, quantize {1e3 * (t2 - t1):.1f} ms",
          flush=True)
