"""Time gptq_fwrd (quantize + propagate) on one synthetic layer of width n
(development tool; the library from TRUNCGPTQ_LIB): the factor from
process_hessian_alt once, then REPS timed gptq_fwrd calls; prints the median
ms and a checksum of the codes-derived weights."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402

n = int(os.environ.get("N", "4096"))
reps = int(os.environ.get("REPS", "10"))
dev = torch.device("cuda")
torch.manual_seed(1)
acc = g.HessianAccumulator(n, dev)
acc.add_batch(torch.randn(3 * n // 4, n, device=dev).half())
H = acc.get_hessian()
W = torch.randn(n, n, device=dev)
U, R_x, perm = g.process_hessian_alt(H, 1e-4, "energy")
q = g.Quantizer(4, 128, False)
ts = []
for r in range(reps + 1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Wq, _ = g.gptq_fwrd(W, U, q, perm, block_size=1024)
    torch.cuda.synchronize()
    if r:
        ts.append((time.perf_counter() - t0) * 1e3)
print(f"n={n} gptq_fwrd median {statistics.median(ts):.3f} ms min {min(ts):.3f} ms "
      f"checksum {float(Wq.double().sum()):.10e}")
