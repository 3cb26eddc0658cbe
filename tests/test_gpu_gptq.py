"""GPU parity of the GPTQ-comparator path (§8(f) rank 3): process_hessian
(gptq_utils.py:129-165) and gptq_fwrd(use_triton=False) (:516-534, :544),
through the C ABI (tg_hinv_chol, tg_gptq_quantize_loop).

Bars: factor within 1e-9 relative Frobenius of the reference's (it is
computed as J (chol(J H J))^-T J instead of cholesky -> cholesky_inverse ->
cholesky: same matrix, other rounding); perm identical; the damping rung
identical; quantised weights bit-exact given the reference's factor;
end to end (own factor) at most 1e-3 of the weights differ (a 1e-12 change
of the factor flips a code only at an exact rounding tie).
"""
import logging

import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def g():
    import gptq_svd_amd.gptq_utils as g
    return g


def t(a, dtype=None):
    x = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return x if dtype is None else x.to(dtype)


def rel_fro(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("name", golden_names("g_"))
def test_process_hessian_golden(g, name, caplog):
    d = load_golden(name)
    with caplog.at_level(logging.INFO):
        R, perm = g.process_hessian(t(d["H"]), actorder=bool(d["actorder"]), damp_percent=0.01)
    R = R.cpu().numpy()
    assert np.array_equal(perm.cpu().numpy(), d["perm"])
    assert rel_fro(R, d["Hinv_chol"]) <= 1e-9
    assert np.all(np.tril(R, -1) == 0.0) and np.all(np.diag(R) > 0)
    damped = "required high damping" in caplog.text
    assert damped == name.endswith("indef")


@pytest.mark.parametrize("name", golden_names("g_"))
def test_gptq_fwrd_loop_golden(g, name):
    d = load_golden(name)
    q = g.Quantizer(int(d["bits"]), int(d["group"]), bool(d["sym"]))
    Wq, k = g.gptq_fwrd(t(d["W"]), t(d["Hinv_chol"]), q, t(d["perm"]),
                        block_size=int(d["block_size"]), use_triton=False)
    Wq = Wq.cpu().numpy()
    assert k == int(d["k"])
    assert np.array_equal(Wq.view(np.uint32), d["final_W"].view(np.uint32)), \
        f"{np.mean(Wq != d['final_W'])} of weights differ"


@pytest.mark.parametrize("name", golden_names("g_"))
def test_gptq_end_to_end(g, name):
    d = load_golden(name)
    R, perm = g.process_hessian(t(d["H"]), actorder=bool(d["actorder"]))
    q = g.Quantizer(int(d["bits"]), int(d["group"]), bool(d["sym"]))
    Wq, _ = g.gptq_fwrd(t(d["W"]), R, q, perm, block_size=int(d["block_size"]),
                        use_triton=False)
    assert np.mean(Wq.cpu().numpy() != d["final_W"]) <= 1e-3


@pytest.mark.parametrize("m,n,bits,group,sym,block", [
    (100, 640, 4, 128, False, 256),
    (64, 2048, 3, 128, True, 1024),
    (48, 384, 8, -1, False, 100),
])
def test_gptq_loop_random_exact(g, oracle_mod, m, n, bits, group, sym, block):
    """Bit-exact against the C oracle's loop on random factors (multi-block,
    ragged rows, odd block width)."""
    rng = np.random.default_rng(m + n)
    X = rng.standard_normal((n + 64, n))
    H = X.T @ X / X.shape[0]
    R, perm, _ = oracle_mod.process_hessian(H, actorder=True)
    W = (rng.standard_normal((m, n)) * 0.05).astype(np.float32)
    q = g.Quantizer(bits, group, sym)
    Wq, _ = g.gptq_fwrd(t(W), t(R), q, t(perm), block_size=block, use_triton=False)
    ref, _ = oracle_mod.gptq_fwrd(W, R, perm, bits, group, sym, block, impl="c",
                                  use_triton=False, nthreads=16)
    Wq = Wq.cpu().numpy()
    assert np.array_equal(Wq.view(np.uint32), ref.view(np.uint32)), \
        f"{np.mean(Wq != ref)} of weights differ"


def test_process_hessian_identity_fallback(g, caplog):
    """Every rung fails (negative definite H): identity, with the warning --
    the reference's intent; as written it raises NameError (:147 vs :162)."""
    H = -torch.eye(64, dtype=torch.float64, device=DEV)
    with caplog.at_level(logging.WARNING):
        R, perm = g.process_hessian(H)
    assert torch.equal(R.cpu(), torch.eye(64, dtype=torch.float64))
    assert "Identity fallback" in caplog.text


@pytest.mark.parametrize("n", [64, 200, 1000, 4096])
def test_hinv_chol_sizes(g, n):
    """Factor property at sizes off the 64 grid and at the harness size:
    R^T R (H + damp I) = I."""
    torch.manual_seed(n)
    X = torch.randn(n + 32, n, dtype=torch.float64, device=DEV)
    H = X.T @ X / X.shape[0]
    R, _ = g.process_hessian(H, damp_percent=0.01)
    Hd = H + 0.01 * torch.diagonal(H).mean() * torch.eye(n, dtype=torch.float64, device=DEV)
    E = R.T @ R @ Hd - torch.eye(n, dtype=torch.float64, device=DEV)
    assert float(E.abs().max()) <= 1e-9


@pytest.mark.parametrize("n,actorder", [(300, False), (1100, True)])
def test_hinv_chol_reads_lower_triangle(g, n, actorder):
    """The reference's torch.linalg.cholesky(H_damped) (gptq_utils.py:152)
    reads only the lower triangle of H_p = H[perm][:, perm].  An H that is not
    bit-symmetric (an FP64 accumulation in another order leaves one) must give
    the factor of H_p's lower triangle: bit-identical to the factor of that
    triangle mirrored, and different from that of the upper one mirrored.
    With ActOrder the permutation depends on the diagonal only, so it is the
    same for all three inputs."""
    torch.manual_seed(n)
    X = torch.randn(n + 64, n, dtype=torch.float64, device=DEV)
    H = X.T @ X / X.shape[0]
    E = torch.randn(n, n, dtype=torch.float64, device=DEV) * 1e-9 * H.abs().max()
    Ha = H + torch.triu(E, 1)                                 # not bit-symmetric
    p = (torch.argsort(torch.diagonal(Ha), descending=True) if actorder
         else torch.arange(n, device=DEV))
    inv = torch.argsort(p)
    Hp = Ha[p][:, p]
    lower = (torch.tril(Hp) + torch.tril(Hp, -1).T)[inv][:, inv]
    upper = (torch.triu(Hp) + torch.triu(Hp, 1).T)[inv][:, inv]
    Ra, pa = g.process_hessian(Ha, actorder=actorder)
    Rl, pl = g.process_hessian(lower, actorder=actorder)
    Ru, _ = g.process_hessian(upper, actorder=actorder)
    assert torch.equal(pa, p) and torch.equal(pl, p)
    assert torch.equal(Ra, Rl)
    assert not torch.equal(Ra, Ru)
