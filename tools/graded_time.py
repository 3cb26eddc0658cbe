"""Phases of one solve on a graded-spectrum Hessian (development tool).

H = Q diag(lam) Q^T with lam geometric from 1 down to LO (default 1e-10) and
Q a random orthogonal matrix (torch QR on the device: tool only, not the
solver path).  The tiny eigenvalues form one cluster at the 1e-6 ||T||
clustering tolerance of the inverse iteration, so this times the block
Gram-Schmidt fallback at production widths.  Prints the
rank, the spectral path and bench.phases' per-stage milliseconds (both of
two calls; the second is warm).
    N=8192 python tools/graded_time.py"""
import os
import sys
import time
from types import SimpleNamespace

import torch

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(here))
import bench  # noqa: E402
import gptq_svd_amd.gptq_utils as g  # noqa: E402

n = int(os.environ.get("N", "8192"))
lo = float(os.environ.get("LO", "1e-10"))
dev = torch.device("cuda")
torch.manual_seed(3)
t0 = time.perf_counter()
Q, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=dev))
lam = torch.logspace(0.0, torch.log10(torch.tensor(lo)).item(), n, dtype=torch.float64, device=dev)
H = (Q * lam) @ Q.T
H = 0.5 * (H + H.T)
del Q
torch.cuda.synchronize()
print(f"n={n}: H built in {time.perf_counter() - t0:.1f} s", flush=True)
W = torch.randn(4096, n, device=dev)
args = SimpleNamespace(eps=1e-4, bits=4, group=128, sym=False, block=1024)
for r in range(2):
    ph, k = bench.phases(g, H, W, args)
    print(f"n={n} k={k} path={bench.phases.path} solve {sum(ph.values()):.1f} ms "
          f"phases {ph}", flush=True)
