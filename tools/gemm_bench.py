"""FP64 GEMM shapes of the solver: tg_dgemm (8-wave, 8-wave without the XCD tile order,
4-wave) vs torch (hipBLASLt / Tensile) (development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

dev = torch.device("cuda")
cases = [  # (name, ta, tb, M, N, K, beta)
    ("NN 4096^3", 0, 0, 4096, 4096, 4096, 0.0),
    ("NN 12288^2 K12288", 0, 0, 12288, 12288, 12288, 0.0),
    ("TN trail 12k K64", 1, 0, 12160, 12160, 64, 1.0),
    ("TN trail 12k K256", 1, 0, 12032, 12032, 256, 1.0),
    ("TN G=A^T A", 1, 0, 3058, 4096, 3058, 0.0),
    ("TN trail K64", 1, 0, 2994, 4032, 64, 1.0),
    ("TN trail K32", 1, 0, 2994, 4032, 32, 1.0),
    ("TN syrk-like K32", 1, 0, 4096, 4096, 32, 1.0),
    ("NN U12 64", 0, 0, 64, 4032, 64, 0.0),
    ("NN k k k", 0, 0, 3058, 3058, 3058, 0.0),
    ("TN k n k", 1, 0, 3058, 4096, 3058, 0.0),
    ("NN k n k", 0, 0, 3058, 4096, 3058, 0.0),
    ("NT k k m", 0, 1, 3058, 3058, 1038, 1.0),
]
for name, ta, tb, M, N, K, beta in cases:
    A = torch.randn((K, M) if ta else (M, K), dtype=torch.float64, device=dev)
    B = torch.randn((N, K) if tb else (K, N), dtype=torch.float64, device=dev)
    C = torch.randn(M, N, dtype=torch.float64, device=dev)
    def ours():
        lib.call("tg_dgemm", lib.stream(), ta, tb, M, N, K, 1.0, lib.ptr(A), A.shape[1], lib.ptr(B),
                 B.shape[1], beta, lib.ptr(C), N)
    opA = A.T if ta else A
    opB = B.T if tb else B
    def ref():
        torch.addmm(C, opA, opB, beta=beta, out=C) if beta else torch.mm(opA, opB, out=C)
    for fn, lab in ((ours, "own8"), (ours, "own8-2d"), (ours, "own"), (ref, "torch")):
        os.environ["TG_GEMM_IMPL"] = lab.split("-")[0]
        os.environ["TG_GEMM_SWZ"] = "0" if lab.endswith("-2d") else "1"
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name:18s} {lab:6s} {ms*1e3:9.1f} us  {2*M*N*K/ms/1e9:7.2f} TF/s", flush=True)
