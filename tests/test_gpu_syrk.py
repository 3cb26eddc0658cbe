"""A1 Hessian accumulation on the 16-bit SYRK (syrk.hip, tg_syrk_accum_ws)
against the FP64 oracle (gptq_utils.py:218-223: x cast to float64, H += x^T x).

The products of 16-bit inputs are exact in FP64, so the only difference to
the oracle is the FP64 summation order: rel. Frobenius <= 1e-14.  Cases: the
bench / real-model widths, widths that are not a multiple of the 128 tile,
row counts that are not a multiple of the 32-row slab, one row, a stream-K
split with many partial tiles (rows >> tiles), bf16, repeated accumulation,
and the fallbacks (n % 8 != 0, a strided view).  Both kernels: X converted to
FP64 at staging (default) and X 16-bit in LDS (TG_SYRK_LDS64=0)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(params=["lds16", "lds64"])
def kernel(request, monkeypatch):
    monkeypatch.setenv("TG_SYRK_LDS64", "1" if request.param == "lds64" else "0")
    return request.param


@pytest.fixture(scope="module")
def g():
    import gptq_svd_amd.gptq_utils as g
    return g


def ref_h(xs):
    H = None
    for x in xs:
        x64 = x.double().numpy()
        H = x64.T @ x64 if H is None else H + x64.T @ x64
    return H


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("n,rows,dtype", [
    (256, 384, torch.float16), (4096, 3072, torch.float16), (1000, 65, torch.bfloat16),
    (1032, 1, torch.float16), (128, 100_000, torch.float16), (2056, 2085, torch.bfloat16),
    (768, 4096, torch.float16)])
def test_syrk16_matches_fp64(g, kernel, n, rows, dtype):
    gen = torch.Generator().manual_seed(n + rows)
    X = (torch.randn(rows, n, generator=gen) * 3).to(dtype)
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(X.to(DEV))
    H = acc.H.cpu().numpy()
    R = ref_h([X])
    assert rel(H, R) <= 1e-14, rel(H, R)
    assert np.array_equal(H, H.T), "both triangles must be written, mirrored exactly"


def test_syrk16_repeated_and_deterministic(g, kernel):
    n = 1536
    gen = torch.Generator().manual_seed(3)
    xs = [torch.randn(777, n, generator=gen).half() for _ in range(3)]
    hs = []
    for _ in range(2):
        acc = g.HessianAccumulator(n, DEV)
        for x in xs:
            acc.add_batch(x.to(DEV).reshape(7, 111, n))  # 3-d batches like the hooks
        hs.append(acc.get_hessian().cpu().numpy())
        assert acc.n_samples == 3 * 777
    assert np.array_equal(hs[0], hs[1]), "same inputs, same device: bit-identical H"
    R = ref_h(xs) / (3 * 777)
    assert rel(hs[0], R) <= 1e-14


def test_syrk16_vs_generic_kernel(g, kernel):
    """The workspace path and the generic FP64 GEMM path agree to rounding."""
    from gptq_svd_amd import _lib
    n, rows = 2048, 4099
    X = torch.randn(rows, n, generator=torch.Generator().manual_seed(9)).half().to(DEV)
    H1 = torch.zeros(n, n, dtype=torch.float64, device=DEV)
    _lib.call("tg_syrk_accum", _lib.stream(), _lib.ptr(X), _lib.TG_F16, rows, n, n,
              _lib.ptr(H1), n)
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(X)
    assert rel(acc.H.cpu().numpy(), H1.cpu().numpy()) <= 1e-14


@pytest.mark.parametrize("case", ["n_not_mult_8", "strided_view", "float32"])
def test_syrk_fallbacks(g, case):
    gen = torch.Generator().manual_seed(11)
    if case == "n_not_mult_8":
        X = torch.randn(300, 100, generator=gen).half()
        Xd = X.to(DEV)
    elif case == "strided_view":
        big = torch.randn(300, 250, generator=gen).half()
        X = big[:, :248]
        Xd = big.to(DEV)[:, :248]  # ld 250 (not a multiple of 8), n 248
    else:
        X = torch.randn(300, 256, generator=gen)
        Xd = X.to(DEV)
    acc = g.HessianAccumulator(X.shape[1], DEV)
    acc.add_batch(Xd)
    assert rel(acc.H.cpu().numpy(), ref_h([X])) <= 1e-14


@pytest.mark.parametrize("nc", ["1", "3", "8"])
def test_syrk_tail_chunks(g, nc, monkeypatch):
    """TG_SYRK_NC (tail tiles cut into 1 / 3 / 8 chunks of K, partial tiles
    summed by the fix-up in chunk order): same H to rounding, deterministic."""
    monkeypatch.setenv("TG_SYRK_NC", nc)
    n, rows = 2048, 3000
    X = torch.randn(rows, n, generator=torch.Generator().manual_seed(12)).half()
    hs = []
    for _ in range(2):
        acc = g.HessianAccumulator(n, DEV)
        acc.add_batch(X.to(DEV))
        hs.append(acc.H.cpu().numpy())
    assert np.array_equal(hs[0], hs[1])
    assert rel(hs[0], ref_h([X])) <= 1e-14
