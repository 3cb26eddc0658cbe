"""Time tg_u_factor_rx at the bench size (development tool; run plain or
under rocprofv3 --kernel-trace and read the last call's timeline with
tools/timeline.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3058
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
# R_x: upper trapezoidal with a dominant positive diagonal (well conditioned)
Rx = torch.randn(k, n, dtype=torch.float64, device=dev, generator=g) / n ** 0.5
Rx = torch.triu(Rx)
Rx.diagonal().copy_(1.0 + torch.rand(k, dtype=torch.float64, device=dev, generator=g))
U = torch.empty(k, n, dtype=torch.float64, device=dev)
ws = lib.workspace(lib.lib.tg_ufactor_rx_workspace_size(n, k), dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for r in range(reps):
    ev[0].record()
    lib.call("tg_u_factor_rx", lib.stream(), lib.ptr(Rx), n, n, k, lib.ptr(U), n, lib.ptr(ws),
             ws.numel())
    ev[1].record()
    torch.cuda.synchronize()
    print(f"u_factor_rx n={n} k={k}: {ev[0].elapsed_time(ev[1]):.3f} ms", flush=True)
if n > 8192:  # the dense check below needs several n^2 temporaries
    sys.exit(0)
del ws
torch.cuda.empty_cache()
# check: U^T U == A^T A, A = (Rx Rx^T)^-1 Rx
S = Rx @ Rx.T
A = torch.linalg.solve(S, Rx)
err = (torch.linalg.norm(U.T @ U - A.T @ A) / torch.linalg.norm(A.T @ A)).item()
print(f"rel err U^T U vs A^T A: {err:.2e}  triu ok: {bool((torch.tril(U, -1) == 0).all())}")
