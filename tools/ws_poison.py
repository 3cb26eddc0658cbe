"""Uninitialised-workspace check (development tool): runs
gptq_utils.truncated_spectral_factor on golden Hessians with every caller
workspace pre-filled with a different byte pattern per run (zeros, 0xFF =
NaN, random bytes, 0x7F), REPS runs per (golden, spectral path); prints the
number of distinct (perm, S, U, R_x) results.  A kernel that reads a
workspace word before writing it shows up as more than one result."""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gptq_svd_amd import _lib  # noqa: E402
import gptq_svd_amd.gptq_utils as g  # noqa: E402

dev = torch.device("cuda")
state = {"r": 0}
gen = torch.Generator(device=dev)


def poisoned(nbytes, device):
    t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
    r = state["r"] % 4
    if r == 0:
        t.zero_()
    elif r == 1:
        t.fill_(0xFF)
    elif r == 2:
        gen.manual_seed(state["r"])
        t.random_(0, 256, generator=gen)
    else:
        t.fill_(0x7F)
    return t


_lib.workspace = poisoned
g.workspace = poisoned

names = os.environ.get("NAMES", "s_n384_w3s_cliff_e7,p_n1024_w3s_e4").split(",")
paths = os.environ.get("PATHS", "kept,auto").split(",")
reps = int(os.environ.get("REPS", "40"))
bad = 0
for name in names:
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    if "H" in d:
        H = torch.from_numpy(d["H"]).to(dev)
    else:
        X = torch.from_numpy(d["X"]).double()
        H = (X.T @ X / X.shape[0]).to(dev)
    eps = float(d["eps"]) if "eps" in d else 1e-4
    method = str(d["method"]) if "method" in d else "energy"
    for path in paths:
        os.environ["TG_SPECTRAL_PATH"] = path
        seen, first = {}, None
        for r in range(reps):
            state["r"] = r
            U, R_x, perm, S, k = g.truncated_spectral_factor(H.clone(), eps, method)
            h = hashlib.sha1()
            for a in (perm, S, U, R_x):
                h.update(a.cpu().numpy().tobytes())
            key = h.hexdigest()[:12]
            if first is None:
                first = (perm.cpu().numpy(), S.cpu().numpy())
            elif key not in seen:
                dS = float(np.abs(S.cpu().numpy() - first[1]).max() / np.abs(first[1]).max())
                print(f"{name} {path} rep {r} (pattern {r % 4}): new result, perm equal "
                      f"{np.array_equal(perm.cpu().numpy(), first[0])}, max rel dS {dS:.2e}",
                      flush=True)
            seen[key] = seen.get(key, 0) + 1
        bad += len(seen) > 1
        print(f"{name} (n = {H.shape[0]}) {path}: {len(seen)} distinct over {reps} runs {seen}",
              flush=True)
print("POISON", "FAIL" if bad else "OK")
