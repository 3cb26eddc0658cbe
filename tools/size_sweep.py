"""Solver phases and size-independent checks at real-model widths.

usage: python tools/size_sweep.py N [N ...]   (GPU; one line of JSON per size)

For each n: X = randn(3n/4, n) fp16 -> H = X^T X / rows (rank 3n/4, like the
bench's synthetic layer), W = randn(n, n).  Prints per-phase wall ms (bench.py's
phases()) and the checks the full-size parity test uses:
  * ||P^T H P - R_x^T R_x||_F == sqrt(sum_{i>k} S_i^4)   (H - H_k = V_r L_r V_r^T)
  * U R_x^T orthogonal                                  (A S^T = I_k)
  * |diag R_x| non-increasing                           (column pivoting)
"""
import json
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import gptq_svd_amd.gptq_utils as g
    dev = torch.device("cuda:0")
    for n in map(int, sys.argv[1:]):
        torch.manual_seed(0)
        rows = 3 * n // 4
        X = torch.randn(rows, n).half().to(dev)
        acc = g.HessianAccumulator(n, dev)
        acc.add_batch(X)
        H = acc.get_hessian()
        W = torch.randn(n, n, device=dev)
        args = SimpleNamespace(eps=1e-4, bits=4, group=128, sym=False, block=1024)
        bench.phases(g, H, W, args)          # warm (module load, allocator)
        ph, k = bench.phases(g, H, W, args)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        U, R_x, perm, S, k = g.truncated_spectral_factor(H, 1e-4, "energy")
        torch.cuda.synchronize()
        t_fact = time.perf_counter() - t0
        Hp = H[perm][:, perm]
        d1 = torch.linalg.norm(Hp - R_x.T @ R_x).item()
        d1_exp = torch.sqrt(torch.sum(S[k:] ** 4)).item()
        M = U @ R_x.T
        orth = (M.T @ M - torch.eye(k, device=dev, dtype=M.dtype)).abs().max().item()
        dg = R_x.diagonal().abs()
        mono = bool((dg[1:] <= dg[:-1] * (1 + 1e-12)).all().item())
        isperm = bool(torch.equal(torch.sort(perm).values, torch.arange(n, device=dev)))
        print(json.dumps(dict(n=n, k=k, path=bench.phases.path, phases_ms=ph, total_ms=round(sum(ph.values()), 1),
                              factor_s=round(t_fact, 3), hk_resid=d1, hk_resid_expected=d1_exp,
                              hnorm=torch.linalg.norm(H).item(), urx_orth=orth,
                              rx_diag_monotone=mono, perm_valid=isperm)), flush=True)
        del U, R_x, perm, S, H, Hp, M, X, W, acc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
