"""The FP64 MFMA GEMM behind tg_dgemm (gemm64.hip) against torch float64 on
the GPU: the 8-wave 128-tile kernel (default for large tiles), the 4-wave
one and the 64-tile one, every transpose combination, beta 0 / 1, ragged
edges, operands that are not 16-byte aligned (8-byte load path), and the
mirrored SYRK form (dsyrk_tn through tg_u_factor_rx's N = Z Z^T is covered by
the solver tests).  FP64 products and sums: rel. Frobenius <= 1e-13."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def lib():
    from gptq_svd_amd import _lib
    return _lib


def run(lib, ta, tb, M, N, K, beta, off=0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    Ab = torch.randn(((K, M) if ta else (M, K))[0] * ((K, M) if ta else (M, K))[1] + off,
                     dtype=torch.float64, device=DEV, generator=g)
    A = Ab[off:].view((K, M) if ta else (M, K))
    B = torch.randn((N, K) if tb else (K, N), dtype=torch.float64, device=DEV, generator=g)
    C = torch.randn(M, N, dtype=torch.float64, device=DEV, generator=g)
    ref = 0.7 * ((A.T if ta else A) @ (B.T if tb else B)) + beta * C
    lib.call("tg_dgemm", lib.stream(), ta, tb, M, N, K, 0.7, lib.ptr(A), A.shape[1], lib.ptr(B),
             B.shape[1], beta, lib.ptr(C), N)
    return (torch.linalg.norm(C - ref) / torch.linalg.norm(ref)).item()


@pytest.mark.parametrize("impl", ["own8", "own8-2d", "own"])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,beta,off", [(2816, 2816, 777, 0.0, 0), (2811, 2819, 301, 1.0, 0),
                                            (2816, 2813, 129, 1.0, 1), (4096, 4096, 64, 1.0, 0)])
def test_dgemm_large_tiles(lib, monkeypatch, impl, ta, tb, M, N, K, beta, off):
    monkeypatch.setenv("TG_GEMM_IMPL", impl.split("-")[0])
    monkeypatch.setenv("TG_GEMM_SWZ", "0" if impl.endswith("-2d") else "1")
    assert run(lib, ta, tb, M, N, K, beta, off) <= 1e-13


@pytest.mark.parametrize("M,N,K", [(100, 300, 50), (1000, 17, 333), (3058, 3058, 1038)])
def test_dgemm_small_tiles(lib, M, N, K):
    assert run(lib, 0, 1, M, N, K, 1.0) <= 1e-13
