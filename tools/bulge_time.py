"""Time the band -> tridiagonal stage (tg_band_tridiag) for the step and
dataflow kernels on one or more library builds, and check that every build's
dataflow output equals the step kernel's bit for bit (development tool).
    python tools/bulge_time.py [lib.so ...]        (N=4096,12288 REPS=5)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, numpy as np, torch
sys.path.insert(0, ROOT)
from gptq_svd_amd import _lib as lib
dev = torch.device("cuda")
B, LDB = 32, 64
for n in [int(x) for x in os.environ.get("N", "4096,12288").split(",")]:
    rng = np.random.default_rng(1)
    A = np.zeros((n, n))
    for dg in range(B + 1):
        v = rng.standard_normal(n - dg)
        A[np.arange(dg, n), np.arange(n - dg)] = v
        A[np.arange(n - dg), np.arange(dg, n)] = v
    Ad = torch.from_numpy(A).to(dev)
    ws = lib.workspace(lib.lib.tg_band_tridiag_workspace_size(n), dev)
    out = {}
    for df in ("0", "1"):
        os.environ["TG_BULGE_DF"] = df
        d = torch.empty(n, dtype=torch.float64, device=dev)
        e = torch.empty(n, dtype=torch.float64, device=dev)
        ts = []
        for r in range(int(os.environ.get("REPS", "5"))):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lib.call("tg_band_tridiag", lib.stream(), lib.ptr(Ad), n, n, lib.ptr(d), lib.ptr(e),
                     lib.ptr(ws), ws.numel())
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        off = n * LDB * 8
        nsw, smax = n - 2, (n - 3) // B + 1
        v2 = ws[off: off + nsw * smax * B * 8].clone()
        out[df] = (d.clone(), e.clone(), v2, ts)
    same = all(torch.equal(out["0"][i], out["1"][i]) for i in range(2))
    print(f"{os.path.basename(lib.LIB_PATH)} n={n}: step {min(out['0'][3]):.2f} ms, "
          f"dataflow {min(out['1'][3]):.2f} ms (all {[round(t, 2) for t in out['1'][3]]}), "
          f"d/e bit-identical: {same}", flush=True)
'''


def main(libs):
    for lib in libs or [""]:
        env = dict(os.environ)
        if lib:
            env["TRUNCGPTQ_LIB"] = lib
        r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], env=env,
                           timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main(sys.argv[1:])
