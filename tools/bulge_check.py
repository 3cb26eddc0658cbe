"""Band -> tridiagonal stage alone (tg_band_tridiag) on a random band matrix:
eigenvalues of the tridiagonal vs LAPACK on the band (development tool; the
same check as tests/test_gpu_solver.py::test_band_tridiag).
    N=4096 REPS=3 python tools/bulge_check.py"""
import os
import sys
import time

import numpy as np
import scipy.linalg as sl
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

n = int(os.environ.get("N", "4096"))
reps = int(os.environ.get("REPS", "3"))
rng = np.random.default_rng(1)
b = 32
A = np.zeros((n, n))
for dgl in range(b + 1):
    v = rng.standard_normal(n - dgl)
    A[np.arange(dgl, n), np.arange(n - dgl)] = v
    A[np.arange(n - dgl), np.arange(dgl, n)] = v
ref = sl.eigvalsh(A)
dev = torch.device("cuda")
Ad = torch.from_numpy(A).to(dev)
ws = lib.workspace(lib.lib.tg_band_tridiag_workspace_size(n), dev)
d = torch.empty(n, dtype=torch.float64, device=dev)
e = torch.empty(n, dtype=torch.float64, device=dev)
ts = []
for r in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lib.call("tg_band_tridiag", lib.stream(), lib.ptr(Ad), n, n, lib.ptr(d), lib.ptr(e),
             lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    ts.append(1e3 * (time.perf_counter() - t0))
    dh, eh = d.cpu().numpy(), e.cpu().numpy()
    ok = np.isfinite(dh).all() and np.isfinite(eh[:n - 1]).all()
    w = sl.eigvalsh_tridiagonal(dh, eh[:n - 1]) if ok else np.full(n, np.nan)
    err = float(np.abs(w - ref).max() / np.abs(ref).max())
    print(f"{os.path.basename(lib.LIB_PATH)} n={n} rep {r}: {ts[-1]:.2f} ms  "
          f"max|w - w_lapack|/|w|max = {err:.2e}", flush=True)
