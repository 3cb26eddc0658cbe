"""Run tools/eigv_time.py against several library variants (TRUNCGPTQ_LIB)
and compare their eigenvalues with the first one (development tool).
    python tools/variant_ab.py gptq-svd_amd/variants/lib_bulge_v*.so"""
import os
import subprocess
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
out = os.path.join(os.path.dirname(here), "gpurun_out")
os.makedirs(out, exist_ok=True)
ref = None
for i, so in enumerate(sys.argv[1:]):
    f = os.path.join(out, f"eig_v{i}.npy")
    for stats in ("", "1"):
        env = dict(os.environ, TRUNCGPTQ_LIB=os.path.abspath(so))
        if stats:
            env.update(TG_BULGE_STATS="1", REPS="1")
        r = subprocess.run([sys.executable, os.path.join(here, "eigv_time.py"), f], env=env,
                           capture_output=True, text=True, timeout=240)
        info = " ".join(ln for ln in r.stderr.splitlines()
                        if "bulge" in ln or "per-wave" in ln or "Error" in ln)
        print(r.stdout.strip(), "|", info[-600:], flush=True)
        if r.returncode:
            print("FAILED", r.returncode, r.stderr[-1500:], flush=True)
            break
    if not os.path.exists(f):
        continue
    w = np.load(f)
    if ref is None:
        ref = w
    print(f"   max |w - w_v0| = {np.abs(w - ref).max():.3e}  "
          f"(bit-identical: {np.array_equal(w, ref)})", flush=True)
