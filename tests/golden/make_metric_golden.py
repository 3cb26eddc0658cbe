"""Golden values of the A6 metric (relative prediction error) produced by the
REFERENCE's own ``log_quantization_error`` (gptq_utils.py:275-291) on the
committed pipeline fixtures that carry R_x.  Runs only in the build container
(imports the reference through make_golden.install_shim).  Output:
``a6_metric.json`` = {fixture: {"value": float, "line": logged text}}.

    python tests/golden/make_metric_golden.py
"""
import glob
import json
import logging
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import install_shim  # noqa: E402


class _Grab(logging.Handler):
    def __init__(self):
        super().__init__()
        self.lines = []

    def emit(self, record):
        self.lines.append(record.getMessage())


def main():
    g = install_shim()
    grab = _Grab()
    root = logging.getLogger()
    root.setLevel(logging.INFO)
    root.addHandler(grab)
    out = {}
    for f in sorted(glob.glob(os.path.join(HERE, "[ps]_*.npz"))):
        z = np.load(f)
        if "Rx" not in z.files:
            continue
        name = os.path.basename(f)[:-4]
        W = torch.from_numpy(z["W"])
        Wq = torch.from_numpy(z["final_W"])
        Rx = torch.from_numpy(z["Rx"])
        perm = torch.from_numpy(z["perm"])
        grab.lines.clear()
        g.log_quantization_error(W, Wq, Rx, perm)
        line = [ln for ln in grab.lines if "Relative prediction error" in ln][-1]
        out[name] = {"value": float(line.rsplit(":", 1)[1]), "line": line}
        print(name, line)
    with open(os.path.join(HERE, "a6_metric.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
