"""Run-to-run determinism of tg_eigh_values (development tool): the golden
Hessians NAMES (default s_n384_w3s_cliff_e7, p_n1024_w3s_e4) REPS times each,
the workspace zeroed on every other run; prints the number of distinct
eigenvalue vectors and, on a difference, the largest relative deviation."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gptq_svd_amd import _lib as lib  # noqa: E402

dev = torch.device("cuda")
for name in os.environ.get("NAMES", "s_n384_w3s_cliff_e7,p_n1024_w3s_e4").split(","):
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    if "H" in d:
        H = torch.from_numpy(d["H"]).to(dev)
    else:
        X = torch.from_numpy(d["X"]).double()
        H = (X.T @ X / X.shape[0]).to(dev)
    n = H.shape[0]
    ws = lib.workspace(lib.lib.tg_eigh_workspace_size(n), dev)
    seen, first = {}, None
    for r in range(int(os.environ.get("REPS", "300"))):
        if r % 2:
            ws.zero_()
        A = H.clone()
        w = torch.empty(n, dtype=torch.float64, device=dev)
        lib.call("tg_eigh_values", lib.stream(), lib.ptr(A), n, n, lib.ptr(w), lib.ptr(ws),
                 ws.numel())
        key = hashlib.sha1(w.cpu().numpy().tobytes()).hexdigest()[:12]
        seen[key] = seen.get(key, 0) + 1
        if first is None:
            first = w.clone()
        elif key not in list(seen)[:1]:
            dev_rel = ((w - first).abs().max() / first.abs().max()).item()
            print(f"{name} rep {r}: eigenvalues differ, max rel {dev_rel:.2e}", flush=True)
    print(f"{name} (n = {n}): {len(seen)} distinct over {sum(seen.values())} runs {seen}", flush=True)
