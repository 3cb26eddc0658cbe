"""Time the eigensolver stages on the GPU (development tool)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda")
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.standard_normal((3 * n // 4, n))).to(dev)
H = (X.T @ X) / X.shape[0]
ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), dev)
w = torch.empty(n, dtype=torch.float64, device=dev)
k = 3 * n // 4 - 16
Vh = torch.empty((k, n), dtype=torch.float64, device=dev)
ref = None
for mode in ("0", "1", "0", "1"):
    os.environ["TG_EIGH_TWOSTAGE"] = mode
    A = H.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    lib.call("tg_eigh_vectors", lib.stream(), n, lib.ptr(w), k, lib.ptr(Vh), n, lib.ptr(ws),
             ws.numel())
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wc = w.cpu().numpy()
    if ref is None:
        ref = wc.copy()
    lam = torch.flip(w, [0])[:k]
    res = torch.linalg.norm(Vh @ H - lam[:, None] * Vh, dim=1).max().item()
    print(f"two_stage={mode} values {1e3*(t1-t0):.1f} ms vectors {1e3*(t2-t1):.1f} ms "
          f"|w-w0| {np.abs(wc-ref).max():.2e} resid {res:.2e}", flush=True)
