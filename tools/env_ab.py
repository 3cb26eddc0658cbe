"""A/B of environment switches on the factorisation time (development tool):
    N=4096 REPS=8 python tools/env_ab.py TG_SCHUR_MIRROR=0 TG_SCHUR_MIRROR=1
Each variant runs process_hessian_alt on the same synthetic H (3n/4 fp16
rows; ROWS=2 for full rank) in one process, variants interleaved rep by rep;
prints the median and min factor ms per variant."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gptq_svd_amd.gptq_utils as g  # noqa: E402


def main(variants):
    ns = [int(x) for x in os.environ.get("N", "4096").split(",")]
    reps = int(os.environ.get("REPS", "8"))
    dev = torch.device("cuda")
    for n in ns:
        rows = int(float(os.environ.get("ROWS", "0.75")) * n)
        torch.manual_seed(1)
        acc = g.HessianAccumulator(n, dev)
        for r0 in range(0, rows, 16384):
            acc.add_batch(torch.randn(min(16384, rows - r0), n, device=dev).half())
        H = acc.get_hessian()
        del acc
        times = {v: [] for v in variants}
        for r in range(reps + 1):
            for v in variants:
                saved = {}
                for kv in v.split(","):
                    k, val = kv.split("=")
                    saved[k] = os.environ.get(k)
                    os.environ[k] = val
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.process_hessian_alt(H, 1e-4, "energy")
                torch.cuda.synchronize()
                if r > 0:  # first round warms every variant up
                    times[v].append(1e3 * (time.perf_counter() - t0))
                for k, old in saved.items():
                    if old is None:
                        del os.environ[k]
                    else:
                        os.environ[k] = old
        for v in variants:
            t = times[v]
            print(f"n={n} {v}: median {statistics.median(t):.2f} ms, min {min(t):.2f} ms", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
