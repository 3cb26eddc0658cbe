"""Interleaved A/B of the SYRK tail chunk count TG_SYRK_NC (development tool):
median TF/s of 5 calls per setting at n = 4096 (262,144 and 65,536 rows) and
12,288 (65,536 rows)."""
import os, sys, time, statistics, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import gptq_svd_amd.gptq_utils as g
dev = "cuda:0"
for n, rows in ((4096, 262144), (4096, 65536), (12288, 65536)):
    torch.manual_seed(0)
    X = torch.randn(rows, n, device=dev).half()
    acc = g.HessianAccumulator(n, dev)
    nt = -(-n // 128); flops = 2.0 * rows * (nt * (nt + 1) // 2) * 128 * 128
    ts = {nc: [] for nc in ("8", "10", "12", "14", "16")}
    for r in range(6):
        for nc in ts:
            os.environ["TG_SYRK_NC"] = nc
            torch.cuda.synchronize(); t0 = time.perf_counter()
            acc.add_batch(X)
            torch.cuda.synchronize()
            if r: ts[nc].append(time.perf_counter() - t0)
    print(f"n={n} rows={rows}: " + ", ".join(f"NC={nc} {flops / statistics.median(v) / 1e12:.1f} TF" for nc, v in ts.items()), flush=True)
    del X, acc; torch.cuda.empty_cache()
