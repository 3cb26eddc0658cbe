"""Residual/orthogonality of the GPU eigensolver on the test problems (development tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from test_gpu_solver import eig_problem, run_eigh  # noqa: E402
from gptq_svd_amd import _lib as lib  # noqa: E402

for kind, n in [("clustered", 256), ("clustered", 544), ("wishart", 300), ("graded", 300)]:
    H = eig_problem(kind, n, n)
    for mode in ("0", "1"):
        os.environ["TG_EIGH_TWOSTAGE"] = mode
        w, Vh = run_eigh(lib, H, n)
        L = np.linalg.eigvalsh(H)
        lam = w[::-1]
        res = np.linalg.norm(Vh @ H - lam[:, None] * Vh, axis=1)
        orth = np.abs(Vh @ Vh.T - np.eye(n)).max()
        print(f"{kind} {n} two_stage={mode}: eig {np.abs(w - L).max():.2e} resid max {res.max():.2e} "
              f"at {res.argmax()} (lam {lam[res.argmax()]:.6f}) orth {orth:.2e}", flush=True)
