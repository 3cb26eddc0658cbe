"""A/B of library builds (TRUNCGPTQ_LIB) on process_hessian_alt (development
tool): each build runs in its own process on the same seeded H (N = 4096,12288
by default, ROWS x n fp16 rows, default 3n/4), REPS timed solves; prints the
median / min and a hash of (perm, R_x, U) so builds that must be bit-identical
can be compared.
    N=12288 python tools/lib_ab.py gptq-svd_amd/variants/lib_band_v*.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import hashlib, os, statistics, sys, time, torch
sys.path.insert(0, ROOT)
import gptq_svd_amd.gptq_utils as g
from gptq_svd_amd import _lib
dev = torch.device("cuda")
for n in [int(x) for x in os.environ.get("N", "4096,12288").split(",")]:
    rows = int(float(os.environ.get("ROWS", "0.75")) * n)
    torch.manual_seed(1)
    acc = g.HessianAccumulator(n, dev)
    for r0 in range(0, rows, 16384):
        acc.add_batch(torch.randn(min(16384, rows - r0), n, device=dev).half())
    H = acc.get_hessian()
    del acc
    ts = []
    for r in range(int(os.environ.get("REPS", "4")) + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        R, R_x, perm = g.process_hessian_alt(H, 1e-4, "energy")
        torch.cuda.synchronize()
        if r:
            ts.append(1e3 * (time.perf_counter() - t0))
    h = hashlib.sha1()
    for t in (perm, R_x, R):
        h.update(t.contiguous().cpu().numpy().tobytes())
    print(f"{os.path.basename(_lib.LIB_PATH)} n={n}: median {statistics.median(ts):.2f} ms, "
          f"min {min(ts):.2f} ms, hash {h.hexdigest()[:16]}", flush=True)
'''


def main(libs):
    for lib in libs:
        env = dict(os.environ, TRUNCGPTQ_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env,
                           timeout=600)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main(sys.argv[1:])
