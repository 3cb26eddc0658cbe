"""BASELINE config 1 (OPT-125M, 4-bit asym g128) at its layer shapes.

1. Solver goldens at OPT shapes (tests/golden/make_golden.py OPT list: the
   REFERENCE's own HessianAccumulator / process_hessian_alt / gptq_fwrd ran
   on seeded gaussian inputs; the test regenerates the inputs from the seed):
   q/k/v/out_proj (n = m = 768), fc1 (n = 768, m = 3072), fc2 (n = 3072,
   m = 768).  End to end on the GPU (own H, eigh, perm, U, codes):
     k, perm identical; S rel <= 1e-12; U through 4 probe vectors rel <= 1e-8
     (bar 1e-3); codes mismatch <= 6e-4 (the reference's own Triton-vs-loop
     disagreement); the A6 log line's value within the reference's 6th decimal.
2. The harness on a tiny random OPT (the reference harness cannot run OPT:
   quantize.py:98 reads model.model.rotary_emb): every linear of every
   layer quantised once in the reference's group order, ranks in range,
   weights on their quantisation grid, and layer 0's q_proj equal to the
   CPU oracle's whole path on the same captured calibration inputs.
"""
import logging
import os
import sys

import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from synth import make_x  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("name", golden_names("o_opt_"))
def test_opt_shapes_end_to_end(name, caplog):
    import gptq_svd_amd.gptq_utils as g
    d = load_golden(name)
    seed, N, n, m = (int(d[k]) for k in ("seed", "N", "n", "m"))
    gen = torch.Generator().manual_seed(seed)
    X = make_x("gaussian", N, n, gen)
    W = torch.randn(m, n, generator=gen) * 0.05
    acc = g.HessianAccumulator(n, DEV)
    acc.add_batch(X.to(DEV))
    H = acc.get_hessian()
    U, R_x, perm, S, k = g.truncated_spectral_factor(H, float(d["eps"]), str(d["method"]))
    assert k == int(d["k"])
    assert np.array_equal(perm.cpu().numpy(), d["perm"].astype(np.int64))
    assert rel(S.cpu().numpy(), d["S"]) <= 1e-12
    probes = torch.randn(n, 4, generator=torch.Generator().manual_seed(seed + 99),
                         dtype=torch.float64)
    assert rel((U.cpu() @ probes).numpy(), d["Uprobe"]) <= 1e-8
    q = g.Quantizer(int(d["bits"]), int(d["group"]), bool(d["sym"]))
    with caplog.at_level(logging.INFO):
        Wq, kq = g.gptq_fwrd(W.to(DEV), U, q, perm, block_size=int(d["block_size"]), R_x=R_x)
    assert kq == k
    assert np.array_equal(q.scale.squeeze(-1).cpu().numpy(), d["scale"])
    assert np.array_equal(q.zero.squeeze(-1).cpu().numpy(), d["zero"])
    codes = q.codes.cpu().numpy()
    mism = float(np.mean(codes != d["codes"]))
    print(f"{name}: k={k}, code mismatch vs reference {mism:.2e}")
    assert mism <= 6e-4
    # the A6 line: extract_log.py:20's pattern, the value within the 6th
    # decimal of the reference's (its FP32 sums vs our FP64 sums of squares)
    import re
    lines = [r.getMessage() for r in caplog.records if "Relative prediction error" in r.getMessage()]
    pat = re.compile(r"Relative prediction error:\s+([\d\.]+)")
    got = float(pat.search(lines[-1]).group(1))
    ref = float(pat.search(str(d["metric_line"])).group(1))
    assert abs(got - ref) <= 1.5e-6, (lines[-1], str(d["metric_line"]))


def tiny_opt(seed):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(vocab_size=256, hidden_size=128, ffn_dim=512, num_hidden_layers=2,
                    num_attention_heads=4, max_position_embeddings=64, word_embed_proj_dim=128,
                    do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    return OPTForCausalLM(cfg).float().eval()


def test_harness_tiny_opt(oracle_mod):
    from gptq_svd_amd.harness import get_sequenced_groups, quantize_model
    model = tiny_opt(11).to(DEV)
    gen = torch.Generator().manual_seed(12)
    ids = [torch.randint(0, 256, (1, 32), generator=gen) for _ in range(8)]
    layer0 = model.model.decoder.layers[0]
    assert get_sequenced_groups(layer0) == [
        ["self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"], ["self_attn.out_proj"],
        ["fc1"], ["fc2"]]
    W0 = layer0.self_attn.q_proj.weight.detach().float().cpu().numpy().copy()
    captured = []
    h = layer0.self_attn.q_proj.register_forward_hook(
        lambda mod, a, o: captured.append(a[0].detach().reshape(-1, a[0].shape[-1]).cpu()))
    try:
        res = quantize_model(model, ids, mode="eigh", w_bits=4, group_size=128, sym=False,
                             eps=1e-4, threshold_method="energy", batch_size=4, device=DEV,
                             pack=True)
    finally:
        h.remove()
    names = [s["name"] for s in res["layer_stats"]]
    assert names == [f"layer_{i}.{x}" for i in range(2) for x in (
        "self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "self_attn.out_proj", "fc1",
        "fc2")]
    for s in res["layer_stats"]:
        n = 512 if s["name"].endswith("fc2") else 128
        assert 1 <= s["rank"] <= n
    assert len(res["packed"]) == 12
    # every weight on its grid: W = (code - z) s with integer codes in [0, 15]
    for name_mod, t in res["packed"].items():
        W = model.get_submodule(name_mod).weight.detach().float().cpu().numpy()
        m, n = W.shape
        codes = oracle_mod.unpack_rows_bitstream(t["qweight"].cpu().numpy(), 4, n).T
        zeros = oracle_mod.unpack_rows_bitstream(t["qzeros"].cpu().numpy().T, 4, m)
        scales = t["scales"].float().cpu().numpy()
        gi = np.arange(n) // 128
        deq = (codes.astype(np.float32) - zeros[:, gi].astype(np.float32)) * scales.T[:, gi]
        assert np.array_equal(deq, W), name_mod
    # layer 0 q_proj against the oracle on the calibration inputs it saw (the
    # first 8 hook calls are the accumulation pass, two batches of 4)
    X = torch.cat(captured[:2]).numpy()
    acc = oracle_mod.HessianAccumulator(X.shape[1])
    acc.add_batch(X)
    f = oracle_mod.process_hessian_alt(acc.get_hessian(), 1e-4, "energy")
    assert res["layer_stats"][0]["rank"] == f.k
    ref, _ = oracle_mod.gptq_fwrd(W0, f.U, f.perm, 4, 128, False, 1024, gemm="torch", impl="c")
    got = layer0.self_attn.q_proj.weight.detach().float().cpu().numpy()
    mism = float(np.mean(got != ref))
    print(f"tiny OPT layer-0 q_proj vs oracle: k={f.k}, weight mismatch {mism:.2e}")
    assert mism <= 6e-4
