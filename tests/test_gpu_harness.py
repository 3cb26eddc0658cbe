"""Harness counterpart (§8(f) rank 1) and packed exporter (rank 2) on a tiny
random Qwen3, against the REFERENCE's own layer loop
(tests/golden/make_harness_golden.py ran quantize.main() on the same model,
same calibration ids, in the build container).

Bars: every module's rank identical; quantised weights equal the
reference's except where a code sits on a rounding tie (the forward runs on
the GPU in rocBLAS order instead of the CPU, so H may differ in the last
bits, and a flipped code in layer 0 would perturb layer 1's inputs): at most
1e-3 of the first group's and 1e-2 of all weights.  Measured in round 1
(tools/harness_parity.py): 0 of 294,912 weights differ in each of the three
cases -- the whole two-layer model is bit-identical to the reference's loop.
Exporter: packed codes / zeros / scales decode to exactly the weights the
harness wrote back.
"""
import json

import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def build(d):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = Qwen3Config(**json.loads(str(d["config"])))
    cfg._attn_implementation = "eager"
    m = Qwen3ForCausalLM(cfg).float().eval()
    sd = {k[len("init/"):]: torch.from_numpy(d[k]) for k in d if k.startswith("init/")}
    m.load_state_dict(sd)
    return m.to(DEV)


def run(d, pack=False):
    from gptq_svd_amd.harness import quantize_model
    model = build(d)
    ids = [torch.from_numpy(r[None]) for r in d["ids"]]
    res = quantize_model(model, ids, mode=str(d["mode"]), w_bits=int(d["bits"]),
                         group_size=int(d["group"]), sym=bool(d["sym"]), eps=float(d["eps"]),
                         threshold_method=str(d["method"]), actorder=bool(d["actorder"]),
                         batch_size=int(d["batch"]), device=DEV, pack=pack)
    return model, res


@pytest.mark.parametrize("name", golden_names("h_"))
def test_harness_matches_reference_loop(name):
    d = load_golden(name)
    model, res = run(d)
    ref_ranks = json.loads(str(d["ranks"]))
    got = [(s["name"], s["rank"]) for s in res["layer_stats"]]
    assert [n for n, _ in got] == [n for n, _ in ref_ranks]
    assert [r for _, r in got] == [r for _, r in ref_ranks]
    sd = model.state_dict()
    total = diff = 0
    for k in d:
        if not k.startswith("final/"):
            continue
        key = k[len("final/"):]
        ref = d[k]
        got_w = sd[key].float().cpu().numpy()
        nd = int(np.sum(got_w != ref))
        total += ref.size
        diff += nd
        if key.startswith("model.layers.0.self_attn.") and key.split(".")[-2] in ("q_proj", "k_proj",
                                                                             "v_proj"):
            assert nd <= 1e-3 * ref.size, f"{key}: {nd} of {ref.size} weights differ"
    assert diff <= 1e-2 * total, f"{diff} of {total} weights differ"


@pytest.mark.parametrize("name", golden_names("h_")[:1] + golden_names("h_")[-1:])
def test_export_roundtrip(name, tmp_path, oracle_mod):
    from gptq_svd_amd.export import read_quantized, save_quantized
    d = load_golden(name)
    bits, group, sym = int(d["bits"]), int(d["group"]), bool(d["sym"])
    model, res = run(d, pack=True)
    save_quantized(str(tmp_path), model, res["packed"], bits, group, sym,
                   extra_config={"mode": str(d["mode"])}, scale_dtype=torch.float32)
    tensors, qc = read_quantized(str(tmp_path))
    assert qc["bits"] == bits and qc["sym"] == sym and qc["checkpoint_format"] == "gptq_v2"
    sd = model.state_dict()
    assert len(res["packed"]) == 14
    for name_mod in res["packed"]:
        W = sd[name_mod + ".weight"].float().cpu().numpy()
        m, n = W.shape
        g = group if group > 0 else n
        codes = oracle_mod.unpack_rows_bitstream(tensors[name_mod + ".qweight"].numpy(), bits, n).T
        zeros = oracle_mod.unpack_rows_bitstream(tensors[name_mod + ".qzeros"].numpy().T, bits, m)
        scales = tensors[name_mod + ".scales"].numpy()          # (G, m)
        gi = np.arange(n) // g
        assert np.array_equal(tensors[name_mod + ".g_idx"].numpy(), gi)
        deq = (codes.astype(np.float32) - zeros[:, gi].astype(np.float32)) * scales.T[:, gi]
        assert np.array_equal(deq, W), f"{name_mod}: {np.mean(deq != W)} differ"
        assert name_mod + ".weight" not in tensors
    # non-quantised tensors travel unchanged
    assert torch.equal(tensors["model.embed_tokens.weight"], sd["model.embed_tokens.weight"].cpu())


@pytest.mark.parametrize("shape", ["tiny", "llama3_8b"])
def test_staged_matches_generic(shape):
    """quantize_model's staged layer path (cached activations between the
    groups, the default for Llama/Qwen decoder layers) against the generic
    path (every group's calibration pass re-runs the layer from its input):
    same ranks, same quantised weights and same model output, bit for bit,
    on the GPU -- the tiny Qwen3 golden in f32 and one Llama-3-8B layer in
    fp16 (8 x 1024 random tokens, a short last batch of 3)."""
    import bench
    from gptq_svd_amd import harness
    out = []
    for staged in (True, False):
        if shape == "tiny":
            d = load_golden(golden_names("h_")[0])
            model = build(d)
            ids = [torch.from_numpy(r[None]) for r in d["ids"]]
            kw = dict(mode=str(d["mode"]), w_bits=int(d["bits"]), group_size=int(d["group"]),
                      sym=bool(d["sym"]), eps=float(d["eps"]),
                      threshold_method=str(d["method"]), batch_size=int(d["batch"]))
        else:
            torch.cuda.empty_cache()
            model, gen = bench.random_causal_lm(shape, 1, DEV, seed=3)
            t = torch.randint(0, model.config.vocab_size, (8, 1024), generator=gen, device=DEV)
            ids = [t[i:i + 1].cpu() for i in range(8)]
            kw = dict(mode="eigh", w_bits=4, group_size=128, sym=False, eps=1e-4,
                      threshold_method="energy", batch_size=5)
        assert harness._staged_layer(harness.get_layers(model)[0])
        res = harness.quantize_model(model, ids, device=DEV, staged=staged, **kw)
        with torch.no_grad():
            y = model.model(torch.cat(ids[:2]).to(DEV)).last_hidden_state
        w = {n: p.detach().clone() for n, p in model.named_parameters() if "layers" in n}
        out.append(([s["rank"] for s in res["layer_stats"]], w, y))
        del model
    (r1, w1, y1), (r2, w2, y2) = out
    assert r1 == r2
    for n in w1:
        assert torch.equal(w1[n], w2[n]), n
    assert torch.equal(y1, y2)
