#!/usr/bin/env python3
"""Throughput of the MI355X-native TruncGPTQ per-layer solver.

BASELINE.json metric: "weight-cols quantized/sec at d_in=4096".  One step =
one full solve of an independent synthetic layer per rank, with the Hessian
already resident in HBM:

    process_hessian_alt(H, 1e-4, "energy")     eigh, rank rule, pivot order, R_x, U
    gptq_fwrd(W, U, Quantizer(4, 128), perm, block_size=1024)
    pack_quantized(...)                        AutoGPTQ-style int32 packing
    [N > 1] RCCL all_gather of the packed weights (the only collective)

Workload (BASELINE.json configs[1]): X = randn(3072, 4096)
fp32 -> fp16 (seed = rank), H = X^T X / 3072 in float64 (FP64 SYRK on the GPU,
outside the timed region, reported separately), W = randn(4096, 4096) f32,
4-bit asym g128, eps = 1e-4 energy (k ~ 3058), block 1024.

Launch (driver contract):
    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import logging
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAKS = {  # MI355X_MICROARCH.md chip table (spec / dense)
    "hbm": ("GB/s", 8000.0),
    "fp32_mfma": ("TFLOP/s", 157.3),
    "fp64_mfma": ("TFLOP/s", 78.6),
    "fp64": ("TFLOP/s", 78.6),  # FP64 vector peak = FP64 matrix peak on MI355X
}
# kernel class -> roofline it is bound by
BOUND = {
    "tri_symv": ("hbm", "bytes"),
    "cross_gemm": ("fp32_mfma", "flops"),
    "quant_block": ("hbm", "bytes"),
    "tri_syr2k": ("fp64_mfma", "flops"),
    "pivot_step": ("hbm", "bytes"),
    "bisect": ("hbm", "bytes"),
    "inverse_iteration": ("hbm", "bytes"),
    "back_transform": ("fp64_mfma", "flops"),
    "bulge_chase": ("fp64", "flops"),     # latency-bound pipeline (see bulge_chain)
    "tsqr_leaf": ("fp64", "flops"),       # latency-bound (32 dependent columns)
    "band_update": ("hbm", "bytes"),
    "q1_apply": ("hbm", "bytes"),
    "q2_apply": ("hbm", "bytes"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n", type=int, default=4096, help="in_features (d_in)")
    p.add_argument("--m", type=int, default=4096, help="out_features")
    p.add_argument("--tokens", type=int, default=3072, help="calibration rows of X")
    p.add_argument("--bits", type=int, default=4)
    p.add_argument("--group", type=int, default=128)
    p.add_argument("--sym", action="store_true")
    p.add_argument("--eps", type=float, default=1e-4)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--prof-every", type=int, default=8,
                   help="sample every k-th launch of each kernel class with HIP events")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-syrk", action="store_true")
    p.add_argument("--no-large-n", action="store_true",
                   help="skip the n = 8192 / 12288 / 14336 / 28672 solve timings in the extras")
    p.add_argument("--no-e2e", action="store_true",
                   help="skip the end-to-end Qwen3-8B-shaped quantize wall-clock")
    p.add_argument("--e2e-layers", type=int, default=36, help="layers of the Qwen3-8B-shaped run")
    p.add_argument("--e2e-only", default="",
                   help="comma list of e2e_qwen3_8b_shape, e2e_llama3_8b_shape, "
                        "layer_llama3_70b_shape (default: all three)")
    p.add_argument("--e2e-samples", type=int, default=128)
    return p.parse_args()


def make_problem(args, rank, device):
    torch.manual_seed(rank)
    X = torch.randn(args.tokens, args.n).half()
    W = torch.randn(args.m, args.n)
    return X, W


def solve(g, H, W, args, gather=None):
    R, R_x, perm = g.process_hessian_alt(H, args.eps, "energy")
    q = g.Quantizer(args.bits, args.group, args.sym)
    Wq, k = g.gptq_fwrd(W, R, q, perm, block_size=args.block, use_triton=True)
    qweight, qzeros, scales = g.pack_quantized(q)
    if gather is not None:
        gather(qweight)
    return k, qweight


def phases(g, H, W, args):
    """One instrumented solve: wall ms per stage (device-synchronised)."""
    from gptq_svd_amd import _lib
    from gptq_svd_amd._lib import call, ptr, stream, workspace
    dev = H.device
    n = H.shape[0]
    sync = torch.cuda.synchronize
    out = {}

    def tick(name, t0):
        sync()
        out[name] = round((time.perf_counter() - t0) * 1e3, 3)
        return time.perf_counter()

    sync()
    t = time.perf_counter()
    A = H.contiguous().clone()
    ws = workspace(_lib.lib.tg_eigh_workspace_size(n), dev)
    w = torch.empty(n, dtype=torch.float64, device=dev)
    call("tg_eigh_values", stream(), ptr(A), n, n, ptr(w), ptr(ws), ws.numel())
    t = tick("eigh_values", t)
    S = torch.empty(n, dtype=torch.float64, device=dev)
    kd = torch.empty(1, dtype=torch.int32, device=dev)
    call("tg_truncation_rank", stream(), ptr(w), n, args.eps, 1, ptr(S), ptr(kd))
    k = int(kd.item())
    t = tick("rank", t)
    sp = g._complement_count(w, k)
    nc = sp.nc
    path = g.spectral_path(n, k, sp)
    phases.path = f"{path} (nc={nc})"
    t = time.perf_counter()
    perm = torch.empty(n, dtype=torch.int64, device=dev)
    Rx = torch.empty((k, n), dtype=torch.float64, device=dev)
    U = torch.empty((k, n), dtype=torch.float64, device=dev)
    if path == "kept":
        Vh = torch.empty((k, n), dtype=torch.float64, device=dev)
        call("tg_eigh_vectors", stream(), n, ptr(w), k, ptr(Vh), n, ptr(ws), ws.numel())
        t = tick("eigh_vectors", t)
        del ws, A
        ws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
        call("tg_pivoted_factor", stream(), ptr(Vh), n, ptr(S), n, k, ptr(perm), ptr(Rx), n,
             ptr(ws), ws.numel())
        t = tick("pivot_order_Rx", t)
        ws = workspace(_lib.lib.tg_ufactor_workspace_size(n, k), dev)
        call("tg_u_factor", stream(), ptr(Vh), n, ptr(S), ptr(perm), n, k, ptr(U), n, ptr(ws),
             ws.numel())
    else:
        Vc = torch.empty((max(nc, 1), n), dtype=torch.float64, device=dev)
        if nc:
            call("tg_eigh_vectors_range", stream(), n, ptr(w), k, nc, ptr(Vc), n, ptr(ws),
                 ws.numel())
        t = tick("eigh_vectors", t)
        del ws, A
        ws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
        call("tg_pivoted_factor_complement", stream(), ptr(H), n, ptr(Vc), n,
             ptr(S[k:]) if nc else None, nc, n, k, ptr(perm), ptr(Rx), n, ptr(ws), ws.numel())
        t = tick("pivot_order_Rx", t)
        ws = workspace(_lib.lib.tg_ufactor_rx_workspace_size(n, k), dev)
        call("tg_u_factor_rx", stream(), ptr(Rx), n, n, k, ptr(U), n, ptr(ws), ws.numel())
    t = tick("u_factor", t)
    q = g.Quantizer(args.bits, args.group, args.sym)
    g.gptq_fwrd(W, U, q, perm, block_size=args.block)
    t = tick("quantize", t)
    g.pack_quantized(q)
    tick("pack", t)
    return out, k


def syrk_bench(g, args, device):
    """Hessian accumulation (A1), reported separately.
    `tflops_kernel` counts the flops the kernel issues (the lower 128 x 128
    tiles, diagonal tiles whole: 2 N T 128^2), so its fraction of the FP64
    MFMA peak is <= 1; `tflops_reference_count` is the reference's full
    2 N n^2 addmm count (the kernel does about half of it)."""
    res = {}
    n = args.n
    for rows, reps in ((args.tokens, 1), (65536, 4)):
        X = torch.randn(rows, n, device=device).half()
        acc = g.HessianAccumulator(n, device)
        acc.add_batch(X)  # warm
        torch.cuda.synchronize()
        acc = g.HessianAccumulator(n, device)
        t0 = time.perf_counter()
        for _ in range(reps):
            acc.add_batch(X)
        acc.get_hessian()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        N = rows * reps
        nt = -(-n // 128)
        kernel_flops = 2.0 * N * (nt * (nt + 1) // 2) * 128 * 128  # lower 128-tiles
        tf = kernel_flops / dt / 1e12
        res[f"N{N}"] = dict(ms=round(dt * 1e3, 3),
                            flops_kernel=kernel_flops, tflops_kernel=round(tf, 2),
                            frac_fp64_mfma_peak=round(tf / PEAKS["fp64_mfma"][1], 4),
                            tflops_reference_count=round(2.0 * N * n * n / dt / 1e12, 2))
        del X
    return res


def large_n(g, args, device):
    """The real models' widths (Llama-3-70B q/o n = 8192, Qwen3-8B down
    n = 12288, Llama-3-8B down n = 14336, Llama-3-70B down n = 28672):
    process_hessian_alt + quantize on a synthetic H of 3n/4
    calibration rows (as tests/test_gpu_fullsize.py), one warm-up solve and
    one timed, with phases; at n = 12288 also the TSQR band reduction
    (TG_SB_TSQR=1, the round-1 path these widths took before) for the
    eigenvalue phase it changes."""
    import copy
    out = {}
    for n in (8192, 12288, 14336, 28672):
        torch.manual_seed(1)
        acc = g.HessianAccumulator(n, device)
        acc.add_batch(torch.randn(3 * n // 4, n, device=device).half())
        H = acc.get_hessian()
        del acc
        a2 = copy.copy(args)
        a2.n, a2.m = n, 4096
        W = torch.randn(a2.m, n, device=device)
        # one warm-up solve at every width: a cold call also pays the caching
        # allocator's first hipMalloc of each workspace (two cold n = 28,672
        # calls on identical U-factor code timed that phase at 0.77 and 1.24 s)
        phases(g, H, W, a2)
        ph, k = phases(g, H, W, a2)
        ent = dict(rank_k=k, path=phases.path, solve_ms=round(sum(ph.values()), 3), phases_ms=ph)
        if n == 12288:
            prev = os.environ.get("TG_SB_TSQR")
            os.environ["TG_SB_TSQR"] = "1"
            try:
                phases(g, H, W, a2)
                ph2, _ = phases(g, H, W, a2)
            finally:
                if prev is None:
                    del os.environ["TG_SB_TSQR"]
                else:
                    os.environ["TG_SB_TSQR"] = prev
            ent["tsqr_band_reduction"] = dict(solve_ms=round(sum(ph2.values()), 3),
                                              eigh_values_ms=ph2["eigh_values"])
        out[f"n{n}"] = ent
        del H, W
        torch.cuda.empty_cache()
    return out


QWEN3_8B = dict(vocab_size=151936, hidden_size=4096, intermediate_size=12288,
                num_hidden_layers=36, num_attention_heads=32, num_key_value_heads=8, head_dim=128,
                max_position_embeddings=40960, rope_theta=1000000.0, rms_norm_eps=1e-6,
                tie_word_embeddings=False)
# Meta-Llama-3-8B / -70B config.json dimensions (BASELINE configs[2], [4])
LLAMA3_8B = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336,
                 num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                 max_position_embeddings=8192, rope_theta=500000.0, rms_norm_eps=1e-5,
                 tie_word_embeddings=False)
LLAMA3_70B = dict(LLAMA3_8B, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                  num_attention_heads=64)
MODEL_SHAPES = {"qwen3_8b": ("qwen3", QWEN3_8B), "llama3_8b": ("llama", LLAMA3_8B),
                "llama3_70b": ("llama", LLAMA3_70B)}


def random_causal_lm(shape: str, layers: int, device, seed: int = 0):
    """A random-init fp16 model with the named model's exact config
    dimensions (no weights exist in this image): N(0, 0.02) matrices, unit
    norm weights, built on the meta device and materialised on `device`."""
    from transformers import LlamaConfig, LlamaForCausalLM, Qwen3Config, Qwen3ForCausalLM
    arch, dims = MODEL_SHAPES[shape]
    Cfg, Model = (Qwen3Config, Qwen3ForCausalLM) if arch == "qwen3" else (LlamaConfig,
                                                                           LlamaForCausalLM)
    cfg = Cfg(**dict(dims, num_hidden_layers=layers))
    cfg._attn_implementation = "sdpa"
    with torch.device("meta"):
        model = Model(cfg)
    model = model.to(dtype=torch.float16).to_empty(device=device)
    gen = torch.Generator(device=device).manual_seed(seed)
    with torch.no_grad():
        for _, p in model.named_parameters():
            if p.dim() == 2:
                p.normal_(0.0, 0.02, generator=gen)
            else:
                p.fill_(1.0)
        model.model.rotary_emb = type(model.model.rotary_emb)(config=cfg, device=device)
    model.eval()
    return model, gen


E2E_NOTE = ("random-init weights with the named model's dimensions and random token ids: a "
            "timing of every stage at production shape, not the reference's workload -- no "
            "PPL; the ranks k come out near n (random activations) where real models keep "
            "fewer; each layer's calibration forward runs once, group by group from "
            "activations cached between the groups (the reference re-runs the whole layer "
            "for every group, quantize.py:139-148); the model stays resident in HBM "
            "(the reference moves each layer CPU<->GPU, quantize.py:101, :250) and no "
            "per-batch cleanup()/synchronize (quantize.py:28-35, :148)")


def e2e_model_shape(shape: str, args, device, layers: int, samples: int,
                    reference_total: str = None):
    """End-to-end quantize wall-clock of a random-init model with a real
    model's shape (the reference's `metrics.total_time`, quantize.py:101,
    :257-260): 2048-token random sequences in batches of 32
    (run_benchmark.py:111-127), eigh 4-bit asym g128, eps 1e-4 energy.
    Per-stage device time from harness.StageClock."""
    from gptq_svd_amd import harness
    t0 = time.perf_counter()
    model, gen = random_causal_lm(shape, layers, device)
    ids = torch.randint(0, model.config.vocab_size, (samples, 2048), generator=gen,
                        device=device).cpu()
    ids = [ids[i:i + 1] for i in range(ids.shape[0])]
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t0
    clock = harness.StageClock()
    # one progress line per layer on stderr (a long run must not look hung)
    log = logging.getLogger()
    hd = logging.StreamHandler(sys.stderr)
    hd.addFilter(lambda r: "completed in" in r.getMessage())
    old_level = log.level
    log.addHandler(hd)
    log.setLevel(logging.INFO)
    try:
        res = harness.quantize_model(model, ids, mode="eigh", w_bits=4, group_size=128,
                                     sym=False, eps=1e-4, threshold_method="energy",
                                     batch_size=32, device=device, clock=clock)
    finally:
        log.removeHandler(hd)
        log.setLevel(old_level)
    stages = {k: round(v, 3) for k, v in sorted(clock.totals().items())}
    ranks = {}
    for st in res["layer_stats"]:
        nm = st["name"].split(".", 1)[1]
        ranks.setdefault(nm, []).append(st["rank"])
    med = {nm: int(sorted(v)[len(v) // 2]) for nm, v in ranks.items()}
    del model
    torch.cuda.empty_cache()
    out = dict(total_s=round(res["total_time"], 2), layers=layers, samples=samples, seq_len=2048,
               batch_size=32, stages_s=stages, stage_counts=dict(sorted(clock.counts.items())),
               median_rank=med, model_init_s=round(t_init, 2))
    if reference_total:
        out["reference_total_s"] = reference_total
    out["note"] = E2E_NOTE
    return out


def e2e_extras(args, device):
    """BASELINE's model-level configs on one MI355X: the Qwen3-8B-shaped
    (configs[3]'s model; the reference's 1522-1534 s run) and Llama-3-8B-shaped
    (configs[2]) full-model quantize, and one Llama-3-70B-shaped layer
    (configs[4]'s layer: hidden 8192, intermediate 28,672) with its stage
    times -- the measured per-layer inputs of DESIGN.md §6's 8-GPU bound."""
    out = {}
    runs = [("e2e_qwen3_8b_shape", "qwen3_8b", args.e2e_layers,
             "1522-1534 (A100 40GB, real weights, 36 layers)"),
            ("e2e_llama3_8b_shape", "llama3_8b", 32, None),
            ("layer_llama3_70b_shape", "llama3_70b", 1, None)]
    for key, shape, layers, ref in runs:
        if args.e2e_only and key not in args.e2e_only.split(","):
            continue
        try:
            out[key] = e2e_model_shape(shape, args, device, layers, args.e2e_samples, ref)
        except Exception as exc:  # the solver line stands without it
            out[key] = dict(error=f"{type(exc).__name__}: {exc}")
        torch.cuda.empty_cache()
    return out


def ar1_solve(g, args, device):
    """SURVEY.md §8(d)'s second synthetic distribution, timed like the main
    layer: X = Z L^T with L L^T the AR(1) rho = 0.9 covariance + 1e-6 I
    (gaussian_corr, benchmarks.py:18-28, :50-54), 3072 x 4096 fp16 rows;
    k ~ 2982 at eps 1e-4 in the survey's run."""
    n = args.n
    idx = torch.arange(n, device=device)
    Sigma = 0.9 ** (idx[None, :] - idx[:, None]).abs().double()
    L = torch.linalg.cholesky(Sigma + 1e-6 * torch.eye(n, dtype=torch.float64, device=device))
    gen = torch.Generator(device=device).manual_seed(7)
    X = (torch.randn(args.tokens, n, generator=gen, device=device) @ L.float().T).half()
    acc = g.HessianAccumulator(n, device)
    acc.add_batch(X)
    H = acc.get_hessian()
    W = torch.randn(args.m, n, generator=gen, device=device)
    del acc, X, L, Sigma
    solve(g, H, W, args)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        k, _ = solve(g, H, W, args)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    ph, _ = phases(g, H, W, args)
    return dict(rank_k=k, ms_per_solve=round(ms, 3), cols_per_s=round(n / ms * 1e3, 1),
                path=phases.path, phases_ms=ph)


def phase_roofline(ph, n, m, k, bits):
    """SURVEY.md §8(d)'s roofline, per phase: the floor max(flops/peak,
    bytes/BW) from the survey's algorithmic work table (n = m = 4096, k =
    3058: eigh (10/3)n^3 = 229 GFLOP FP64; pivoted QR and U-QR 2k^2 n - 2k^3/3
    = 57.5 GFLOP FP64 each; propagation 2m(k(n-1) - k(k-1)/2) = 64.3 GFLOP
    FP32 on MFMA; quantize / pack 4 m n bytes read + m n b / 8 written)
    divided by the phase's measured time (`phases_ms`), and the solve's
    time-weighted total (sum of floors / sum of times; the survey's floor is
    ~5 ms).  The eigh row counts the whole (10/3)n^3 the reference's
    torch.linalg.eigh spends (gptq_utils.py:93), though this path forms only
    the eigenvalues and the few eigenvectors it needs; its BLAS2 bytes are a
    one-stage tridiagonalisation's and are not part of this two-stage path."""
    fp64, fp32, bw = PEAKS["fp64_mfma"][1] * 1e12, PEAKS["fp32_mfma"][1] * 1e12, \
        PEAKS["hbm"][1] * 1e9
    qr = 2.0 * k * k * n - 2.0 * k ** 3 / 3.0
    rows = [
        ("eigh", ("eigh_values", "rank", "eigh_vectors"), 10.0 / 3.0 * n ** 3, 0.0, fp64,
         "fp64_mfma", "gptq_utils.py:93-108"),
        ("pivoted_qr", ("pivot_order_Rx",), qr, 0.0, fp64, "fp64_mfma", "gptq_utils.py:112-117"),
        ("u_qr", ("u_factor",), qr, 0.0, fp64, "fp64_mfma", "gptq_utils.py:118-124"),
        ("quantize_propagate", ("quantize", "pack"),
         2.0 * m * (k * (n - 1) - k * (k - 1) / 2.0), 4.0 * m * n + m * n * bits / 8.0, fp32,
         "fp32_mfma", "gptq_utils.py:459-565"),
    ]
    out, floor_tot, t_tot = [], 0.0, 0.0
    for name, keys, flops, nbytes, peak, kind, ref in rows:
        t = sum(ph.get(x, 0.0) for x in keys)
        f_c, f_m = flops / peak * 1e3, nbytes / bw * 1e3
        floor = max(f_c, f_m)
        floor_tot += floor
        t_tot += t
        out.append(dict(phase=name, phases_ms=list(keys), reference=ref, gflop=round(flops / 1e9, 2),
                        mbytes=round(nbytes / 1e6, 1), bound=kind if f_c >= f_m else "hbm",
                        floor_ms=round(floor, 4), measured_ms=round(t, 3),
                        frac=round(floor / t, 4) if t > 0 else None))
    return dict(phases=out, solve=dict(floor_ms=round(floor_tot, 3), measured_ms=round(t_tot, 3),
                                       frac=round(floor_tot / t_tot, 4) if t_tot else None,
                                       weighting="time-weighted: sum of floors / sum of phase times"))


def cpu_baseline(H, W, args):
    """The oracle's CPU restatement of the reference path (numpy eigh, LAPACK
    dgeqp3, numpy QR, exact C block loop + torch SGEMM), timed on this host."""
    import numpy as np
    from oracle import oracle as o
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    Hn = H.cpu().numpy()
    Wn = W.cpu().numpy()
    t0 = time.perf_counter()
    f = o.process_hessian_alt(Hn, args.eps, "energy")
    t1 = time.perf_counter()
    _, k, codes = o.gptq_fwrd(Wn, f.U, f.perm, args.bits, args.group, args.sym, args.block,
                              gemm="torch", impl="c", return_codes=True, nthreads=cores)
    s, z = o.find_params(Wn, args.bits, args.group, args.sym)
    o.pack_weights(codes, s, z, args.bits, args.sym)
    t2 = time.perf_counter()
    dt = t2 - t0
    return dict(value=round(args.n / dt, 2), unit="cols/s", cores=cores, kind="port",
                sample=(f"one full {args.m}x{args.n} solve (k={f.k}) of the same synthetic layer: "
                        f"factorisation {t1 - t0:.2f}s + quantize/pack {t2 - t1:.2f}s"))


PMC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06",
                        "pmc_traffic.json")
if not os.path.exists(PMC_FILE):  # until this round's profile is committed
    PMC_FILE = PMC_FILE.replace("r06", "r05")
LATENCY_BOUND = {"bulge_chase", "tsqr_leaf"}
BULGE_DG = 2  # csrc/bulge.hip TG_BULGE_DF_GSW: sweeps per workgroup of the dataflow kernel


def bulge_chain(n, avg_ms):
    """The bulge pipeline's critical path (Two-stage 2.): the
    dataflow kernel's sweep groups of DG sweeps hand the band from one CU to
    the next through L2, and group G + 1 trails group G by a fixed latency
    (two task periods of the chain's pace + the L2 hand-off + one task per
    sweep of the group), so one launch is about groups x that lag."""
    groups = -(-(n - 2) // BULGE_DG)
    return dict(dependent_groups=groups, sweeps=n - 2,
                us_per_group=round(avg_ms * 1e3 / groups, 3),
                us_per_sweep=round(avg_ms * 1e3 / (n - 2), 3),
                model=f"groups of {BULGE_DG} sweeps chained through L2 hand-offs (dataflow kernel)")


def pmc_traffic(cls, args):
    """HBM bytes per launch of kernel class `cls` from the committed rocprofv3
    PMC passes (tools/profile_round.sh + tools/pmc_traffic.py; FETCH_SIZE
    doubled per the gfx950 correction).  Counters cannot be read inside a
    timed run, so the value comes from the profile of the same default
    workload; null for other workloads or classes without a PMC pass."""
    default = (args.n, args.m, args.tokens, args.bits, args.group, args.sym) == (
        4096, 4096, 3072, 4, 128, False)
    if not default or not os.path.exists(PMC_FILE):
        return {}
    ent = json.load(open(PMC_FILE)).get(cls)
    if not ent:
        return {}
    return dict(traffic=ent["traffic_bytes"], traffic_unit="bytes/launch",
                traffic_source=os.path.relpath(PMC_FILE, os.path.dirname(PMC_FILE) + "/../.."))


def pmc_summary(args):
    """Time-weighted HBM bandwidth of every class with PMC passes (the same
    committed profile as `pmc_traffic`; default workload only)."""
    default = (args.n, args.m, args.tokens, args.bits, args.group, args.sym) == (
        4096, 4096, 3072, 4, 128, False)
    if not default or not os.path.exists(PMC_FILE):
        return None
    out = {}
    for cls, ent in json.load(open(PMC_FILE)).items():
        if "bandwidth_GBs" in ent:
            out[cls] = dict(bytes_per_launch=ent["traffic_bytes"], GBs=ent["bandwidth_GBs"],
                            hbm_frac=ent["hbm_frac"])
    return out or None


def launch_plan(gpus: int, env=None):
    """How `bench.py --gpus N` runs (driver contract).  Under a launcher
    (WORLD_SIZE set) the world size must equal --gpus.  Without one, N > 1
    spawns N fresh processes (one per GPU) before anything touches the GPU
    in this one.  Returns ("run", world) or ("spawn", N); raises on a mismatch."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} "
                             "ranks; they must agree")
        return "run", world
    return ("spawn", gpus) if gpus > 1 else ("run", 1)


def _spawned(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = argv
    run(parse())


def main():
    args = parse()
    mode, world = launch_plan(args.gpus)
    if mode == "spawn":
        import socket
        import torch.multiprocessing as mp
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        # fresh interpreters (start method "spawn"): this process never touches the GPU
        mp.spawn(_spawned, args=(world, port, list(sys.argv)), nprocs=world, join=True)
        return
    run(args)


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")

    import gptq_svd_amd.gptq_utils as g
    from gptq_svd_amd import _lib

    X, W_cpu = make_problem(args, rank, device)
    acc = g.HessianAccumulator(args.n, device)
    acc.add_batch(X.to(device))
    H = acc.get_hessian()
    W = W_cpu.to(device)
    del acc

    gather = None
    gathered = {"calls": 0, "bytes": 0}
    if world > 1:
        from gptq_svd_amd.dist import gather_packed

        def gather(t):
            out = gather_packed(t)
            gathered["calls"] += 1
            gathered["bytes"] += out.numel() * out.element_size()
            return out

    for _ in range(args.warmup):
        solve(g, H, W, args, gather)
    torch.cuda.synchronize()

    _lib.profile_reset()
    _lib.profile_enable(True, args.prof_every)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k, _ = solve(g, H, W, args, gather)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    gather_bytes_per_step = gathered["bytes"] // max(1, gathered["calls"])
    _lib.profile_enable(False)
    prof = _lib.profile_query()
    if world > 1:
        tt = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    value = world * args.n * args.steps / dt

    # roofline of the dominant kernel class (largest estimated share of step time)
    best = None
    for name, p in prof.items():
        if p["sampled"] == 0:
            continue
        est_total = p["ms"] * p["launches"] / p["sampled"]
        if best is None or est_total > best[1]:
            best = (name, est_total, p)
    roof = None
    shares = {}
    for name, p in prof.items():
        if p["sampled"]:
            shares[name] = round(p["ms"] * p["launches"] / p["sampled"] / args.steps, 3)
    if best is not None:
        name, _, p = best
        kind, field = BOUND[name]
        unit, peak = PEAKS[kind]
        avg_ms = p["ms"] / p["sampled"]
        per_launch = p[field] / p["sampled"]
        if field == "bytes":
            achieved = per_launch / (avg_ms * 1e-3) / 1e9
        else:
            achieved = per_launch / (avg_ms * 1e-3) / 1e12
        bound = "hbm" if kind == "hbm" else ("latency" if name in LATENCY_BOUND else "mfma")
        roof = dict(kernel=name, bound=bound,
                    peak_kind=kind,
                    achieved=round(achieved, 3), peak=peak, unit=unit,
                    frac=round(achieved / peak, 4), traffic=None,
                    avg_launch_ms=round(avg_ms, 5), launches_per_step=p["launches"] // args.steps)
        roof.update(pmc_traffic(name, args))
        if name == "bulge_chase":
            roof["chain"] = bulge_chain(args.n, avg_ms)

    extra = {}
    if rank == 0:
        ph, _ = phases(g, H, W, args)
        extra["phases_ms"] = ph
        extra["spectral_path"] = phases.path
        if roof is not None:
            roof.update(phase_roofline(ph, args.n, args.m, k, args.bits))
        extra["kernel_ms_per_step"] = shares
        if (args.n, args.m) == (4096, 4096):
            extra["ar1_rho0.9"] = ar1_solve(g, args, device)
        pm = pmc_summary(args)
        if pm:
            extra["pmc_hbm"] = pm
        if not args.no_syrk:
            extra["syrk"] = syrk_bench(g, args, device)
        if not args.no_large_n and (args.n, args.m) == (4096, 4096):
            extra["large_n"] = large_n(g, args, device)
        if not args.no_e2e and world == 1:
            extra.update(e2e_extras(args, device))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(H, W, args)

    if rank == 0:
        line = {
            "metric": "weight-cols quantized/sec at d_in=4096",
            "value": round(value, 2),
            "unit": "cols/s",
            "n_gpus": world,
            "world_size": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32",
            "data": "synthetic (X randn fp16 3072x4096 -> H=X^T X/N f64; W randn f32)",
            "config": {
                "workload": (f"single synthetic {args.n}x{args.n} Hessian per rank, full solver "
                             f"(eigh, rank rule, pivot order, U, {args.bits}-bit "
                             f"{'sym' if args.sym else 'asym'} g{args.group} quantize, pack)"),
                "n": args.n, "m": args.m, "calib_rows": args.tokens, "rank_k": k,
                "eps": args.eps, "threshold_method": "energy", "block_size": args.block,
                "parallelism": (f"independent layer per rank x{world}"
                                + (", RCCL all_gather of packed weights" if world > 1 else "")),
                "allgather_bytes_per_step": gather_bytes_per_step if world > 1 else 0,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            **extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
