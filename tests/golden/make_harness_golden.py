"""Golden vectors for the harness counterpart (§8(f) rank 1): run the
REFERENCE's own layer loop, ``quantize.main()``
(/root/reference/src/TruncGPTQ/quantize.py:47-252), on a tiny random Qwen3
in this container, and record the quantized weights and per-layer ranks.

Offline stand-ins are patched in for what needs the network or a GPU:
argument parsing (a fixed namespace), model loading (the tiny model below,
float32 so that GPU-vs-CPU forward rounding stays ~1e-7), the calibration
loader (seeded random token ids) and the PPL evaluation (skipped).  The loop
itself -- capture, hooks, HessianAccumulator, process_hessian(_alt),
gptq_fwrd, re-forward -- is the reference's code, unchanged.  Uses the same
jax shim / Triton interpreter as make_golden.py.

    python tests/golden/make_harness_golden.py
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402  (installs nothing at import)

HERE = os.path.dirname(os.path.abspath(__file__))

TINY = dict(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
            num_attention_heads=4, num_key_value_heads=2, head_dim=32,
            max_position_embeddings=64, rms_norm_eps=1e-6, tie_word_embeddings=False)
N_SAMPLES, SEQ_LEN, BATCH = 8, 32, 4

CASES = [
    # name, mode, bits, group, sym, eps, threshold_method, actorder
    ("h_qwen3tiny_eigh_w4a", "eigh", 4, 128, False, 1e-4, "energy", False),
    ("h_qwen3tiny_eigh_w3s_mt", "eigh", 3, 128, True, 1e-2, "mean_trimmed", False),
    ("h_qwen3tiny_gptq_w4a", "gptq", 4, 128, False, 1e-2, "energy", True),
]


def tiny_model(seed):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = Qwen3Config(**TINY)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    m = Qwen3ForCausalLM(cfg).float().eval()
    return m


def run_case(spec, seed):
    name, mode, bits, group, sym, eps, method, actorder = spec
    make_golden.install_shim()
    import quantize  # the reference harness (REF on sys.path via the shim)
    model = tiny_model(seed)
    init = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    gen = torch.Generator().manual_seed(seed + 1)
    ids = [torch.randint(0, TINY["vocab_size"], (1, SEQ_LEN), generator=gen)
           for _ in range(N_SAMPLES)]
    out_dir = tempfile.mkdtemp()
    args = argparse.Namespace(
        model_id="tiny-qwen3", device="cpu", seed=seed, dataset="wikitext2",
        n_samples=N_SAMPLES, seq_len=SEQ_LEN, batch_size=BATCH, w_bits=bits,
        group_size=group, sym=sym, eps=eps, sketch_ratio=4.0, mode=mode,
        threshold_method=method, actorder=actorder, damp_percent=0.01, adaptive_eps=False,
        save_path=out_dir, no_save=True)
    quantize.get_args = lambda: args
    quantize.setup_logging = lambda *a, **k: None
    quantize.model_utils.get_model = lambda *a, **k: (model, None)
    quantize.data_utils.get_loaders = lambda *a, **k: [t.clone() for t in ids]
    quantize.eval_utils.evaluate_perplexity = lambda *a, **k: 0.0
    quantize.main()
    log = json.load(open(os.path.join(out_dir, "results.json")))
    final = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    out = {"ids": torch.cat(ids).numpy().astype(np.int64), "bits": np.int64(bits),
           "group": np.int64(group), "sym": np.bool_(sym), "eps": np.float64(eps),
           "method": np.str_(method), "mode": np.str_(mode), "actorder": np.bool_(actorder),
           "batch": np.int64(BATCH), "config": np.str_(json.dumps(TINY)),
           "ranks": np.str_(json.dumps([(s["name"], s["rank"]) for s in log["layer_stats"]]))}
    for k, v in init.items():
        out["init/" + k] = v
    for k, v in final.items():
        if k.endswith("proj.weight"):
            out["final/" + k] = v
    return name, out


def main():
    only = set(sys.argv[1:])
    for i, spec in enumerate(CASES):
        if only and spec[0] not in only:
            continue
        name, d = run_case(spec, 4000 + i)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, d["ranks"])


if __name__ == "__main__":
    main()
