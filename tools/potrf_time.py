"""Per-kernel timing of the blocked Cholesky pieces (development tool; run
under rocprofv3 --kernel-trace): tg_hinv_chol at n = 64 and n = 1024."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

from gptq_svd_amd import _lib as lib  # noqa: E402

dev = torch.device("cuda")
for n, reps in ((64, 50), (1024, 5)):
    X = torch.randn(2 * n, n, dtype=torch.float64, device=dev)
    H = X.T @ X / (2 * n)
    R = torch.empty(n, n, dtype=torch.float64, device=dev)
    ws = lib.workspace(lib.lib.tg_hinv_chol_workspace_size(n), dev)
    used = ctypes.c_int()
    for _ in range(reps):
        lib.call("tg_hinv_chol", lib.stream(), lib.ptr(H), n, n, None, 0.0, 1, lib.ptr(R), n,
                 ctypes.byref(used), lib.ptr(ws), ws.numel())
    torch.cuda.synchronize()
    print(n, "ok", used.value)
