"""Time the two-stage eigensolver stages for TG_BULGE_G in {4, 8} (development tool)."""
import os
import subprocess
import sys

for g in ("4", "8"):
    env = dict(os.environ, TG_BULGE_G=g)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "eigh_time.py"),
                        sys.argv[1] if len(sys.argv) > 1 else "4096"], env=env,
                       capture_output=True, text=True)
    print(f"G={g}\n{r.stdout}{r.stderr[-2000:]}", flush=True)
