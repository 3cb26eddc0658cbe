"""Run-to-run reproducibility under a mixed load (development tool): small
golden solves (truncated_spectral_factor on every (path, refine) pair, as
tests/test_gpu_conditioning.py runs them) interleaved with large eigh /
solver calls that change cache, clock and allocator state between them, for
SECONDS of wall time.  Prints every result that differs from the first one of
its case and the number of distinct results per case."""
import hashlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gptq_svd_amd import _lib  # noqa: E402
import gptq_svd_amd.gptq_utils as g  # noqa: E402

dev = torch.device("cuda")
rng = np.random.default_rng(0)


def load(name):
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    if "H" in d:
        H = torch.from_numpy(d["H"]).to(dev)
    else:
        X = torch.from_numpy(d["X"]).double()
        H = (X.T @ X / X.shape[0]).to(dev)
    eps = float(d["eps"]) if "eps" in d else 1e-4
    return H, eps, str(d["method"]) if "method" in d else "energy"


names = os.environ.get("NAMES", "s_n384_w3s_cliff_e7,s_n512_w4a_graded_e7,p_n1024_w3s_e4").split(",")
cases = [(nm, p, r) for nm in names for p in ("auto", "kept", "complement") for r in ("auto", "0", "1")]
data = {nm: load(nm) for nm in names}
big = []
for n in (2048, 4096):
    X = torch.randn(2 * n, n, dtype=torch.float64, device=dev)
    big.append((X.T @ X) / (2 * n))
seen = {c: {} for c in cases}
first = {}
t_end = time.time() + float(os.environ.get("SECONDS", "300"))
it = 0
while time.time() < t_end:
    c = cases[rng.integers(len(cases))]
    nm, path, refine = c
    os.environ["TG_SPECTRAL_PATH"] = path
    if refine == "auto":
        os.environ.pop("TG_U_REFINE", None)
    else:
        os.environ["TG_U_REFINE"] = refine
    H, eps, method = data[nm]
    U, R_x, perm, S, k = g.truncated_spectral_factor(H.clone(), eps, method)
    h = hashlib.sha1()
    for a in (perm, S, U, R_x):
        h.update(a.cpu().numpy().tobytes())
    key = h.hexdigest()[:12]
    Sn = S.cpu().numpy()
    if c not in first:
        first[c] = (perm.cpu().numpy(), Sn)
    elif key not in seen[c]:
        dS = float(np.linalg.norm(Sn - first[c][1]) / np.linalg.norm(first[c][1]))
        print(f"iter {it} {c}: new result, perm equal {np.array_equal(perm.cpu().numpy(), first[c][0])}, "
              f"rel dS {dS:.2e}, max-dev index {int(np.argmax(np.abs(Sn - first[c][1])))}", flush=True)
    seen[c][key] = seen[c].get(key, 0) + 1
    # perturbation between small solves
    sel = rng.integers(4)
    if sel == 0:
        os.environ.pop("TG_SPECTRAL_PATH", None)
        os.environ.pop("TG_U_REFINE", None)
        Hb = big[rng.integers(len(big))]
        g.truncated_spectral_factor(Hb.clone(), 1e-4, "energy")
    elif sel == 1:
        a = torch.randn(8192, 8192, device=dev)
        (a @ a).sum().item()
    it += 1
    if it % 50 == 0:
        print(f"iter {it}", flush=True)
bad = sum(len(v) > 1 for v in seen.values())
for c, v in seen.items():
    print(c, len(v), "distinct over", sum(v.values()), "runs")
print("HUNT", "DIFF" if bad else "SAME", f"{it} iterations")
