"""Generate golden vectors by running the REFERENCE solver in this container.

Runs only where /root/reference exists (the build container).  It imports the
reference's own ``gptq_utils`` with an in-process ``jax`` shim (SURVEY.md §4.3:
``jax.scipy.linalg.qr(pivoting=True)`` -> ``scipy.linalg.qr(pivoting=True)``,
i.e. LAPACK dgeqp3, the algorithm MAGMA runs for the reference) and Triton's
CPU interpreter (``TRITON_INTERPRET=1``) for ``gptq_block_kernel``.

Outputs small ``.npz`` fixtures (inputs + reference outputs) next to this
file.  Nothing from the reference is copied: only data it produced.

    python tests/golden/make_golden.py
"""
import os
import sys
import types

os.environ.setdefault("TRITON_INTERPRET", "1")
import datasets  # noqa: F401  (import before the shim: SURVEY.md §4.3)
import transformers  # noqa: F401
import numpy as np
import scipy.linalg
import torch

REF = "/root/reference/src/TruncGPTQ"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from synth import make_x  # noqa: E402  (shared with the tests)


def install_shim():
    jax = types.ModuleType("jax")
    jax.__path__ = []
    jax.config = types.SimpleNamespace(update=lambda *a, **k: None)
    jax.clear_caches = lambda: None
    dl = types.ModuleType("jax.dlpack")
    dl.from_dlpack = lambda t: t.detach().cpu().numpy()
    sp = types.ModuleType("jax.scipy")
    spl = types.ModuleType("jax.scipy.linalg")

    def qr(a, pivoting=False, mode="full"):
        q, r, p = scipy.linalg.qr(np.asarray(a), pivoting=True, mode=mode)
        return q, r, p.astype(np.int32)

    spl.qr = qr
    sp.linalg = spl
    jax.scipy = sp
    jax.dlpack = dl
    sys.modules.update({"jax": jax, "jax.dlpack": dl, "jax.scipy": sp, "jax.scipy.linalg": spl})
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.empty_cache = lambda *a, **k: None
    sys.path.insert(0, REF)
    import gptq_utils  # noqa: E402
    return gptq_utils


# name, n, m, N, xkind, bits, group, sym, eps, method, block_size
PIPELINE = [
    ("p_n256_w4a_e4", 256, 64, 384, "gaussian", 4, 128, False, 1e-4, "energy", 1024),
    ("p_n256_w3s_e2", 256, 96, 192, "gaussian", 3, 128, True, 1e-2, "energy", 1024),
    ("p_n512_w4s_mt", 512, 128, 384, "ar1", 4, 128, True, 1e-2, "mean_trimmed", 1024),
    ("p_n512_w2a_e6_gall", 512, 64, 768, "lognormal", 2, -1, False, 1e-6, "energy", 1024),
    ("p_n512_w4a_e4_b128", 512, 128, 640, "gaussian", 4, 128, False, 1e-4, "energy", 128),
    ("p_n384_w8a_e5_b128", 384, 80, 256, "ar1", 8, 128, False, 1e-5, "energy", 128),
    ("p_n1024_w3s_e4", 1024, 64, 1536, "gaussian", 3, 128, True, 1e-4, "energy", 1024),
    ("p_n1024_w4a_e4_b256", 1024, 64, 768, "gaussian", 4, 128, False, 1e-4, "energy", 256),
]

# Hessians given by their spectrum, H = Q diag(lam) Q^T (Q Haar, float64):
# graded / cliff spectra at energy eps 1e-7, where the smallest kept
# eigenvalue is ~1e-7 lam_max and a Gram-matrix (CholeskyQR) U factor loses
# ~cond^2 eps.  name, n, m, spectrum, bits, group, sym, eps, method, block_size
SPECTRA = [
    ("s_n512_w4a_graded_e7", 512, 64, "graded14", 4, 128, False, 1e-7, "energy", 1024),
    ("s_n384_w3s_cliff_e7", 384, 48, "cliff", 3, 128, True, 1e-7, "energy", 1024),
]


def spectrum(kind, n, gen):
    if kind == "graded14":   # 1 .. 1e-14, geometric
        return torch.logspace(0, -14, n, dtype=torch.float64)
    if kind == "cliff":      # half geometric 1 .. 1e-3, half ~1e-7
        h = n // 2
        lo = 1e-7 * (1.0 + 0.5 * torch.rand(n - h, generator=gen, dtype=torch.float64))
        return torch.cat([torch.logspace(0, -3, h, dtype=torch.float64), lo])
    raise ValueError(kind)


def gen_spectrum(g, spec, seed):
    name, n, m, kind, bits, group, sym, eps, method, bs = spec
    gen = torch.Generator().manual_seed(seed)
    Qm = torch.linalg.qr(torch.randn(n, n, generator=gen, dtype=torch.float64))[0]
    lam = spectrum(kind, n, gen)
    H = (Qm * lam) @ Qm.T
    H = (H + H.T) / 2
    R, R_x, perm = g.process_hessian_alt(H, threshold=eps, threshold_method=method)
    W = torch.randn(m, n, generator=gen) * 0.05
    q = g.Quantizer(w_bits=bits, group_size=group, sym=sym)
    final_W, k = g.gptq_fwrd(W.clone(), R, q, perm, block_size=bs, use_triton=True, R_x=R_x)
    L, _ = torch.linalg.eigh(H)
    S = torch.sqrt(L.clamp(min=1e-12)).flip(0)
    scale, zero = q.scale.squeeze(-1), q.zero.squeeze(-1)
    return name, dict(
        H=H.numpy(), S=S.numpy(), k=np.int64(k), perm=perm.numpy().astype(np.int64),
        U=R.numpy(), Rx=R_x.numpy(), W=W.numpy(), final_W=final_W.numpy(),
        scale=scale.numpy(), zero=zero.numpy(), bits=np.int64(bits), group=np.int64(group),
        sym=np.bool_(sym), eps=np.float64(eps), method=np.str_(method),
        block_size=np.int64(bs))


# block-kernel fixtures: name, m, B, bits, sym
BLOCKS = [
    ("b_m64_B64_w4a", 64, 64, 4, False),
    ("b_m70_B100_w3s", 70, 100, 3, True),
    ("b_m130_B1024_w4a", 130, 1024, 4, False),
    ("b_m33_B16_w2a", 33, 16, 2, False),
]


def gen_pipeline(g, spec, seed):
    name, n, m, N, xkind, bits, group, sym, eps, method, bs = spec
    gen = torch.Generator().manual_seed(seed)
    X = make_x(xkind, N, n, gen)
    acc = g.HessianAccumulator(n, "cpu")
    # two batches, like several hook calls (quantize.py:139-148)
    h = N // 2
    acc.add_batch(X[:h].reshape(1, h, n))
    acc.add_batch(X[h:])
    H = acc.get_hessian()
    R, R_x, perm = g.process_hessian_alt(H, threshold=eps, threshold_method=method)
    W = torch.randn(m, n, generator=gen) * 0.05
    q = g.Quantizer(w_bits=bits, group_size=group, sym=sym)
    final_W, k = g.gptq_fwrd(W.clone(), R, q, perm, block_size=bs, use_triton=True, R_x=R_x)
    # eigenvalues as the reference computes them (gptq_utils.py:93-94)
    L, _ = torch.linalg.eigh(H.double())
    S = torch.sqrt(L.clamp(min=1e-12)).flip(0)
    scale, zero = q.scale.squeeze(-1), q.zero.squeeze(-1)
    out = dict(
        X=X.numpy(), S=S.numpy(), k=np.int64(k), perm=perm.numpy().astype(np.int64),
        W=W.numpy(), final_W=final_W.numpy(), scale=scale.numpy(), zero=zero.numpy(),
        bits=np.int64(bits), group=np.int64(group), sym=np.bool_(sym), eps=np.float64(eps),
        method=np.str_(method), block_size=np.int64(bs), N=np.int64(N),
    )
    U = R.numpy()
    Rx = R_x.numpy()
    if n >= 1024:  # keep fixtures small: H is X^T X / N (recomputable from X), f32 U is
        out["U32"] = U.astype(np.float32)  # plenty for the 1e-3 bar, R_x only feeds the log metric
    else:
        out["H"] = H.numpy()
        out["U"] = U
        out["Rx"] = Rx
    return name, out


# GPTQ comparator (process_hessian + gptq_fwrd(use_triton=False)):
# name, n, m, N, xkind, bits, group, sym, actorder, block_size, H override
GPTQ = [
    ("g_n256_w4a", 256, 64, 384, "gaussian", 4, 128, False, False, 256, None),
    ("g_n384_w3s_act", 384, 48, 512, "ar1", 3, 128, True, True, 512, None),
    ("g_n256_w4a_lowrank", 256, 40, 96, "lognormal", 4, -1, False, False, 256, None),
    ("g_n512_w4a_b128", 512, 64, 640, "gaussian", 4, 128, False, True, 128, None),
    ("g_n128_w4a_indef", 128, 32, 0, "indef", 4, 128, False, False, 128, "indef"),
]


# OPT-125M shapes (BASELINE config 1: q/k/v/out_proj and fc1 read d = 768,
# fc2 reads 3072; 4-bit asym g128).  The inputs are regenerated from the seed
# by the test (gaussian X only: pure RNG, no BLAS), so the fixture holds only
# outputs: rank, perm, eigenvalues, U through 4 probe vectors, codes.
# name, n, m, N, bits, group, sym, eps, method, block_size
OPT = [
    ("o_opt_qkv_n768_m768", 768, 768, 1536, 4, 128, False, 1e-4, "energy", 1024),
    ("o_opt_fc1_n768_m3072", 768, 3072, 1536, 4, 128, False, 1e-4, "energy", 1024),
    ("o_opt_fc2_n3072_m768", 3072, 768, 4608, 4, 128, False, 1e-4, "energy", 1024),
]


def opt_probes(n, seed):
    return torch.randn(n, 4, generator=torch.Generator().manual_seed(seed + 99),
                       dtype=torch.float64)


def gen_opt(g, spec, seed):
    import logging
    name, n, m, N, bits, group, sym, eps, method, bs = spec
    gen = torch.Generator().manual_seed(seed)
    X = make_x("gaussian", N, n, gen)
    W = torch.randn(m, n, generator=gen) * 0.05
    acc = g.HessianAccumulator(n, "cpu")
    acc.add_batch(X)
    H = acc.get_hessian()
    R, R_x, perm = g.process_hessian_alt(H, threshold=eps, threshold_method=method)
    q = g.Quantizer(w_bits=bits, group_size=group, sym=sym)
    lines = []
    h = logging.Handler()
    h.emit = lambda r: lines.append(r.getMessage())
    logging.getLogger().addHandler(h)
    logging.getLogger().setLevel(logging.INFO)
    final_W, k = g.gptq_fwrd(W.clone(), R, q, perm, block_size=bs, use_triton=True, R_x=R_x)
    logging.getLogger().removeHandler(h)
    L, _ = torch.linalg.eigh(H.double())
    S = torch.sqrt(L.clamp(min=1e-12)).flip(0)
    s_, z_ = q.get_expanded_params(m, n)
    codes = torch.round(final_W / s_ + z_)       # exact: final_W = (q - z) s
    assert torch.equal((codes - z_) * s_, final_W)
    metric = [ln for ln in lines if "Relative prediction error" in ln][-1]
    return name, dict(
        seed=np.int64(seed), N=np.int64(N), n=np.int64(n), m=np.int64(m), k=np.int64(k),
        perm=perm.numpy().astype(np.int32), S=S.numpy(),
        Uprobe=(R @ opt_probes(n, seed)).numpy(), Unorm=np.float64(torch.linalg.norm(R)),
        codes=codes.numpy().astype(np.uint8), scale=q.scale.squeeze(-1).numpy(),
        zero=q.zero.squeeze(-1).numpy(), bits=np.int64(bits), group=np.int64(group),
        sym=np.bool_(sym), eps=np.float64(eps), method=np.str_(method), block_size=np.int64(bs),
        metric_line=np.str_(metric))


def gen_gptq(g, spec, seed):
    name, n, m, N, xkind, bits, group, sym, actorder, bs, hov = spec
    gen = torch.Generator().manual_seed(seed)
    if hov == "indef":
        # symmetric with one negative eigenvalue (-5% of the mean diagonal):
        # rung 1e-2 fails, 1e-1 succeeds (the damping ladder, :148-160)
        Qm = torch.linalg.qr(torch.randn(n, n, generator=gen, dtype=torch.float64))[0]
        ev = torch.rand(n, generator=gen, dtype=torch.float64) + 0.5
        ev[0] = -0.05 * float(ev.mean())
        H = (Qm * ev) @ Qm.T
        H = (H + H.T) / 2
        X = None
    else:
        X = make_x(xkind, N, n, gen)
        acc = g.HessianAccumulator(n, "cpu")
        acc.add_batch(X)
        H = acc.get_hessian()
    Hinv_chol, perm = g.process_hessian(H, actorder=actorder, damp_percent=0.01)
    W = torch.randn(m, n, generator=gen) * 0.05
    q = g.Quantizer(w_bits=bits, group_size=group, sym=sym)
    final_W, k = g.gptq_fwrd(W.clone(), Hinv_chol, q, perm, block_size=bs, use_triton=False)
    scale, zero = q.scale.squeeze(-1), q.zero.squeeze(-1)
    out = dict(H=H.numpy(), Hinv_chol=Hinv_chol.numpy(), perm=perm.numpy().astype(np.int64),
               W=W.numpy(), final_W=final_W.numpy(), scale=scale.numpy(), zero=zero.numpy(),
               bits=np.int64(bits), group=np.int64(group), sym=np.bool_(sym),
               actorder=np.bool_(actorder), block_size=np.int64(bs), k=np.int64(k))
    return name, out


def gen_block(g, spec, seed):
    name, m, B, bits, sym = spec
    gen = torch.Generator().manual_seed(seed)
    w = torch.randn(m, B, generator=gen) * 0.1
    q = g.Quantizer(w_bits=bits, group_size=-1, sym=sym)
    q.find_params(w)
    s, z = q.get_expanded_params(m, B)
    A = torch.randn(B, B, generator=gen, dtype=torch.float64)
    R = torch.linalg.qr(A @ A.T / B + torch.eye(B, dtype=torch.float64))[1]
    R = (R * torch.sign(torch.diagonal(R)).unsqueeze(1)).float()
    qv, e = g.triton_process_block(w.clone(), s.clone(), z.clone(), R.clone(), q)
    return name, dict(w=w.numpy(), s=s.numpy(), z=z.numpy(), R=R.numpy(), q=qv.numpy(),
                      e=e.numpy(), minq=np.int64(q.min_q), maxq=np.int64(q.max_q))


def main():
    g = install_shim()
    only = set(sys.argv[1:])
    for i, spec in enumerate(BLOCKS):
        if only and spec[0] not in only:
            continue
        name, d = gen_block(g, spec, 1000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)
    for i, spec in enumerate(PIPELINE):
        if only and spec[0] not in only:
            continue
        name, d = gen_pipeline(g, spec, 2000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, "k =", int(d["k"]))
    for i, spec in enumerate(GPTQ):
        if only and spec[0] not in only:
            continue
        name, d = gen_gptq(g, spec, 3000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)
    for i, spec in enumerate(OPT):
        if only and spec[0] not in only:
            continue
        name, d = gen_opt(g, spec, 5000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, "k =", int(d["k"]), str(d["metric_line"]))
    for i, spec in enumerate(SPECTRA):
        if only and spec[0] not in only:
            continue
        name, d = gen_spectrum(g, spec, 4000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, "k =", int(d["k"]))


if __name__ == "__main__":
    main()
