"""Stage attribution for tools/flake_hunt.py (development tool): the
truncated_spectral_factor pipeline restated call by call, each stage's output
hashed -- A after tg_eigh_values (the band form sy2sb leaves), the
eigenvalues, (d, e) of a separate tg_band_tridiag of that band, the
eigenvectors, (perm, R_x), U -- under the same mixed load.  On a difference
prints the first stage that differs and the perturbation that preceded it."""
import hashlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gptq_svd_amd import _lib  # noqa: E402
from gptq_svd_amd._lib import call, ptr, stream, workspace  # noqa: E402
import gptq_svd_amd.gptq_utils as g  # noqa: E402

dev = torch.device("cuda")
rng = np.random.default_rng(int(os.environ.get("SEED", "0")))


def hsh(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()[:10]


def load(name):
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    if "H" in d:
        H = torch.from_numpy(d["H"]).to(dev)
    else:
        X = torch.from_numpy(d["X"]).double()
        H = (X.T @ X / X.shape[0]).to(dev)
    return H, float(d["eps"]), str(d["method"])


def pipeline(H, eps, method, path):
    n = H.shape[0]
    out = []
    A = H.clone()
    ws = workspace(_lib.lib.tg_eigh_workspace_size(n), dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    call("tg_eigh_values", stream(), ptr(A), n, n, ptr(w), ptr(ws), ws.numel())
    out.append(("band", hsh(A)))
    out.append(("eig", hsh(w)))
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.empty(n, dtype=torch.float64, device=dev)
    bws = workspace(_lib.lib.tg_band_tridiag_workspace_size(n), dev)
    call("tg_band_tridiag", stream(), ptr(A), n, n, ptr(d), ptr(e), ptr(bws), bws.numel())
    out.append(("tridiag", hsh(d, e[:n - 1])))
    S = torch.empty(n, dtype=torch.float64, device=dev)
    kdev = torch.empty(1, dtype=torch.int32, device=dev)
    call("tg_truncation_rank", stream(), ptr(w), n, float(eps), _lib.RULES.get(method, 0), ptr(S),
         ptr(kdev))
    wk = torch.cat((w, kdev.to(torch.float64))).cpu().numpy()
    k = int(wk[n])
    sp = g._complement_count(wk[:n], k)
    nc = sp.nc
    if path == "auto":
        path = g.spectral_path(n, k, sp)
    perm = torch.empty(n, dtype=torch.int64, device=dev)
    R_x = torch.empty((k, n), dtype=torch.float64, device=dev)
    U = torch.empty((k, n), dtype=torch.float64, device=dev)
    if path == "kept":
        Vh = torch.empty((k, n), dtype=torch.float64, device=dev)
        call("tg_eigh_vectors", stream(), n, ptr(w), k, ptr(Vh), n, ptr(ws), ws.numel())
        out.append(("vec", hsh(Vh)))
        pws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
        call("tg_pivoted_factor", stream(), ptr(Vh), n, ptr(S), n, k, ptr(perm), ptr(R_x), n,
             ptr(pws), pws.numel())
        out.append(("pivot", hsh(perm, R_x)))
        uws = workspace(_lib.lib.tg_ufactor_workspace_size(n, k), dev)
        call("tg_u_factor", stream(), ptr(Vh), n, ptr(S), ptr(perm), n, k, ptr(U), n, ptr(uws),
             uws.numel())
    else:
        Vc = torch.empty((max(nc, 1), n), dtype=torch.float64, device=dev)
        if nc:
            call("tg_eigh_vectors_range", stream(), n, ptr(w), k, nc, ptr(Vc), n, ptr(ws),
                 ws.numel())
        out.append(("vec", hsh(Vc)))
        pws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
        Hd = H.contiguous()
        call("tg_pivoted_factor_complement", stream(), ptr(Hd), n, ptr(Vc), n,
             ptr(S[k:]) if nc else None, nc, n, k, ptr(perm), ptr(R_x), n, ptr(pws), pws.numel())
        out.append(("pivot", hsh(perm, R_x)))
        uws = workspace(_lib.lib.tg_ufactor_rx_workspace_size(n, k), dev)
        call("tg_u_factor_rx", stream(), ptr(R_x), n, n, k, ptr(U), n, ptr(uws), uws.numel())
    out.append(("U", hsh(U)))
    return path, out, w.cpu().numpy()


names = os.environ.get("NAMES", "s_n384_w3s_cliff_e7,s_n512_w4a_graded_e7,p_n1024_w3s_e4").split(",")
cases = [(nm, p, r) for nm in names for p in ("kept", "complement") for r in ("auto", "0", "1")]
data = {nm: load(nm) for nm in names}
big = []
for n in (2048, 4096):
    X = torch.randn(2 * n, n, dtype=torch.float64, device=dev)
    big.append((X.T @ X) / (2 * n))
ref = {}
stage_diff = {}
t_end = time.time() + float(os.environ.get("SECONDS", "300"))
it, prev = 0, "none"
while time.time() < t_end:
    c = cases[rng.integers(len(cases))]
    nm, path, refine = c
    if refine == "auto":
        os.environ.pop("TG_U_REFINE", None)
    else:
        os.environ["TG_U_REFINE"] = refine
    H, eps, method = data[nm]
    taken, out, w = pipeline(H, eps, method, path)
    if c not in ref:
        ref[c] = (out, w)
    else:
        r_out, r_w = ref[c]
        for (stg, hv), (_, hr) in zip(out, r_out):
            if hv != hr:
                dw = float(np.abs(w - r_w).max() / np.abs(r_w).max())
                print(f"iter {it} {c}: first differing stage {stg} (after {prev}); "
                      f"max rel dw {dw:.2e} at {int(np.argmax(np.abs(w - r_w)))}", flush=True)
                stage_diff[stg] = stage_diff.get(stg, 0) + 1
                break
    sel = rng.integers(4)
    os.environ.pop("TG_U_REFINE", None)
    if sel == 0:
        Hb = big[rng.integers(len(big))]
        g.truncated_spectral_factor(Hb.clone(), 1e-4, "energy")
        prev = "big solve"
    elif sel == 1:
        a = torch.randn(8192, 8192, device=dev)
        (a @ a).sum().item()
        prev = "matmul"
    else:
        prev = "none"
    it += 1
    if it % 100 == 0:
        print(f"iter {it}", flush=True)
print("STAGES", stage_diff, f"{it} iterations")
