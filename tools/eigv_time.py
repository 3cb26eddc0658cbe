"""Time tg_eigh_values on the bench's synthetic Hessian (development tool).
Prints ms per call (min / median of REPS) and writes the eigenvalues to
argv[1] (.npy) for cross-variant comparison."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402
from gptq_svd_amd import _lib as lib  # noqa: E402

n = int(os.environ.get("N", "4096"))
reps = int(os.environ.get("REPS", "6"))
dev = torch.device("cuda")
torch.manual_seed(0)
X = torch.randn(3072, n, device=dev).half()
acc = g.HessianAccumulator(n, dev)
acc.add_batch(X)
H = acc.get_hessian()
ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), dev)
w = torch.empty(n, dtype=torch.float64, device=dev)
ts = []
for r in range(reps + 1):
    A = H.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    if r:
        ts.append(1e3 * (time.perf_counter() - t0))
wc = w.cpu().numpy()
ref = np.linalg.eigvalsh(H.cpu().numpy())
err = float(np.abs(wc - ref).max() / np.abs(ref).max())
if len(sys.argv) > 1:
    np.save(sys.argv[1], wc)
print(f"{os.path.basename(lib.LIB_PATH)}: eigh_values min {min(ts):.2f} med {np.median(ts):.2f} ms"
      f" max|w - w_lapack|/|w|max = {err:.2e}",
      flush=True)
