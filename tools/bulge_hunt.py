"""Rare-race hunt in the band -> tridiagonal stage (development tool):
tg_band_tridiag on a fixed random band, REPS calls per width, each (d, e)
compared on the device with the first call's.  Prints the number of calls
that differ silently and of calls the tridiagonal guard rejected (the call
raises, outputs poisoned), and for the first few where they differ.
    TRUNCGPTQ_LIB=variant.so N=384,1024 REPS=20000 python tools/bulge_hunt.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gptq_svd_amd import _lib as lib  # noqa: E402

dev = torch.device("cuda")
B = 32
tag = os.path.basename(lib.LIB_PATH) + (" DF=" + os.environ["TG_BULGE_DF"]
                                         if "TG_BULGE_DF" in os.environ else "")
for n in [int(x) for x in os.environ.get("N", "384,1024").split(",")]:
    rng = np.random.default_rng(n)
    A = np.zeros((n, n))
    for dg in range(B + 1):
        v = rng.standard_normal(n - dg)
        A[np.arange(dg, n), np.arange(n - dg)] = v
        A[np.arange(n - dg), np.arange(dg, n)] = v
    Ad = torch.from_numpy(A).to(dev)
    ws = lib.workspace(lib.lib.tg_band_tridiag_workspace_size(n), dev)
    d = torch.empty(n, dtype=torch.float64, device=dev)
    e = torch.empty(n, dtype=torch.float64, device=dev)
    ref = None
    bad, shown = 0, 0
    reps = int(os.environ.get("REPS", "20000"))
    t0 = time.time()
    caught = 0
    for r in range(reps):
        try:
            lib.call("tg_band_tridiag", lib.stream(), lib.ptr(Ad), n, n, lib.ptr(d), lib.ptr(e),
                     lib.ptr(ws), ws.numel())
        except RuntimeError as exc:  # the tridiagonal guard fired: outputs poisoned
            caught += 1
            if caught <= 5:
                print(f"  n={n} call {r}: guard: {exc}", flush=True)
                if os.environ.get("TG_TRI_GUARD_NOPOISON") and ref is not None:
                    # values kept: where and by how much they differ
                    dd = (d != ref[0]).nonzero().flatten().cpu().numpy()
                    de = (e[:n - 1] != ref[1]).nonzero().flatten().cpu().numpy()
                    print(f"    d differs at {dd[:8]} ({dd.size}), e at {de[:8]} ({de.size}); "
                          f"max |dd| {float((d - ref[0]).abs().max()):.2e} "
                          f"max |de| {float((e[:n - 1] - ref[1]).abs().max()):.2e}", flush=True)
            continue
        if ref is None:
            ref = (d.clone(), e[:n - 1].clone())
            continue
        if not (torch.equal(d, ref[0]) and torch.equal(e[:n - 1], ref[1])):
            bad += 1
            if shown < 5:
                shown += 1
                dd = (d != ref[0]).nonzero().flatten().cpu().numpy()
                de = (e[:n - 1] != ref[1]).nonzero().flatten().cpu().numpy()
                print(f"  n={n} call {r}: d differs at {dd[:6]} ({dd.size}), e at {de[:6]} "
                      f"({de.size}); max |dd| {float((d - ref[0]).abs().max()):.2e}", flush=True)
        if r % 5000 == 0:
            print(f"  n={n} call {r} ({time.time() - t0:.0f} s)", flush=True)
    print(f"{tag} n={n}: {bad} of {reps - 1} calls differ silently, {caught} caught by the "
          f"tridiagonal guard ({time.time() - t0:.0f} s)", flush=True)
