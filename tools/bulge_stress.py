"""Run-to-run determinism of the band -> tridiagonal stage (development
tool): tg_band_tridiag on the band of a random symmetric matrix REPS times
per width, the dataflow kernel's d / e / reflector records hashed per run and
compared with the step kernel's.  Prints the number of distinct results."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

dev = torch.device("cuda")
B, LDB = 32, 64
for n in [int(x) for x in os.environ.get("N", "1024,1100,2048,4096").split(",")]:
    rng = np.random.default_rng(n)
    A = np.zeros((n, n))
    for dg in range(B + 1):
        v = rng.standard_normal(n - dg)
        A[np.arange(dg, n), np.arange(n - dg)] = v
        A[np.arange(n - dg), np.arange(dg, n)] = v
    Ad = torch.from_numpy(A).to(dev)
    ws = lib.workspace(lib.lib.tg_band_tridiag_workspace_size(n), dev)
    res = {}
    reps = int(os.environ.get("REPS", "100"))
    for df in ("0", "1"):
        os.environ["TG_BULGE_DF"] = df
        seen = {}
        for r in range(reps if df == "1" else 3):
            d = torch.empty(n, dtype=torch.float64, device=dev)
            e = torch.empty(n, dtype=torch.float64, device=dev)
            if r % 2:  # alternate a zeroed and a reused workspace
                ws.zero_()
            lib.call("tg_band_tridiag", lib.stream(), lib.ptr(Ad), n, n, lib.ptr(d), lib.ptr(e),
                     lib.ptr(ws), ws.numel())
            off = n * LDB * 8
            nsw, smax = n - 2, (n - 3) // B + 1
            v2 = ws[off: off + nsw * smax * B * 8].view(torch.float64).view(nsw, smax, B)
            # the records of tasks that exist (sweep j has (n - 3 - j) // B + 1)
            used = torch.arange(smax, device=dev)[None, :] < (
                (n - 3 - torch.arange(nsw, device=dev)) // B + 1)[:, None]
            v2u = v2[used]
            key = tuple(hashlib.sha1(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]
                        for t in (d, e, v2u))
            seen[key] = seen.get(key, 0) + 1
        res[df] = seen
    same = set(res["0"]) == set(res["1"]) and len(res["1"]) == 1
    parts = {df: [len({k[i] for k in res[df]}) for i in range(3)] for df in res}
    print(f"n={n}: step {len(res['0'])} distinct, dataflow {len(res['1'])} distinct over {reps}, "
          f"dataflow == step: {same}; distinct (d, e, records): step {parts['0']}, "
          f"dataflow {parts['1']}", flush=True)
