"""Time eigh_vectors for several invit layouts (development tool)."""
import os
import subprocess
import sys

for v in ("64", "32", "16", "8"):
    env = dict(os.environ, TG_INVIT_VPW=v)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "eigh_time.py"), "4096"],
                       env=env, capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if "two_stage=1" in l]
    print(f"vpw={v}: {lines[-1] if lines else r.stderr[-500:]}", flush=True)
