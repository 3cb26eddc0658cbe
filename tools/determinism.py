"""Run-to-run determinism of the solver (development tool): the golden
Hessian p_n1024_w3s_e4 (or NAME) through truncated_spectral_factor on both
spectral paths REPS times in one process, with other solves (n = 4096,
2048) interleaved so the workspace holds different data each time; prints
how many distinct (perm, S, U) results each path produced and, on a
difference, which outputs differ."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gptq_svd_amd.gptq_utils as g  # noqa: E402

dev = torch.device("cuda")
name = os.environ.get("NAME", "p_n1024_w3s_e4")
d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
if "H" in d:
    H = torch.from_numpy(d["H"]).to(dev)
else:
    X = torch.from_numpy(d["X"]).double()
    H = (X.T @ X / X.shape[0]).to(dev)
others = []
for n in (4096, 2048):
    torch.manual_seed(n)
    acc = g.HessianAccumulator(n, dev)
    acc.add_batch(torch.randn(3 * n // 4, n, device=dev).half())
    others.append(acc.get_hessian())


def h(t):
    return hashlib.sha1(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


reps = int(os.environ.get("REPS", "20"))
for path in ("kept", "complement"):
    os.environ["TG_SPECTRAL_PATH"] = path
    seen = {}
    first = None
    for r in range(reps):
        U, R_x, perm, S, k = g.truncated_spectral_factor(H, float(d["eps"]), str(d["method"]))
        key = (h(perm), h(S), h(U), h(R_x))
        seen[key] = seen.get(key, 0) + 1
        if first is None:
            first = key
            ref = (perm.clone(), S.clone(), U.clone())
        elif key != first:
            diff = [nm for nm, a, b in zip(("perm", "S", "U", "R_x"), key, first) if a != b]
            print(f"{path} rep {r}: differs in {diff}; perm equal to golden: "
                  f"{np.array_equal(perm.cpu().numpy(), d['perm'])}", flush=True)
        g.process_hessian_alt(others[r % 2], 1e-4, "energy")
    print(f"{path}: {len(seen)} distinct results over {reps} reps "
          f"(perm equal to golden on the first: {np.array_equal(ref[0].cpu().numpy(), d['perm'])})",
          flush=True)
