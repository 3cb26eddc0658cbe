"""Per-module parity of the harness counterpart vs the reference's loop
(tests/golden/h_*.npz): fraction of weights that differ, and rank match."""
import json
import sys

import numpy as np

sys.path.insert(0, "tests")
from conftest import golden_names, load_golden  # noqa: E402
from test_gpu_harness import run  # noqa: E402

for name in golden_names("h_"):
    d = load_golden(name)
    model, res = run(d)
    sd = model.state_dict()
    ranks_ok = [s["rank"] for s in res["layer_stats"]] == [r for _, r in json.loads(str(d["ranks"]))]
    tot = dif = 0
    per = []
    for k in d:
        if k.startswith("final/"):
            key = k[6:]
            g = sd[key].float().cpu().numpy()
            nd = int(np.sum(g != d[k]))
            tot += g.size
            dif += nd
            per.append(f"{'.'.join(key.split('.')[2:4])}:{nd}")
    print(f"{name}: ranks equal {ranks_ok}; {dif}/{tot} = {dif / tot:.2e} weights differ; "
          + " ".join(per))
