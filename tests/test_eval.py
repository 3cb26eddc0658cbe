"""§8(f)4: perplexity evaluator and calibration sampler, against the values
the REFERENCE's own eval_utils.evaluate_perplexity / data_utils.get_wikitext2
produced on the same synthetic corpus, byte tokenizer and tiny Qwen3
(tests/golden/make_eval_golden.py -> e_eval.npz).

CPU: same device and dtype as the fixture run, so the PPL must agree to
1e-9 relative and the calibration windows exactly.  GPU: the model forward on
cuda:0 (other GEMM/softmax rounding), PPL to 1e-6 relative."""
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from eval_corpus import ByteTokenizer, corpus  # noqa: E402

from gptq_svd_amd import evaluate as ev  # noqa: E402

E = np.load(os.path.join(HERE, "golden", "e_eval.npz"))
CASES = sorted(k[len("ppl/"):] for k in E.files if k.startswith("ppl/"))


def model(weights, device):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    d = np.load(os.path.join(HERE, "golden", "h_qwen3tiny_eigh_w4a.npz"))
    cfg = Qwen3Config(**json.loads(str(d["config"])))
    cfg._attn_implementation = "eager"
    m = Qwen3ForCausalLM(cfg).float().eval()
    sd = {k[len("init/"):]: torch.from_numpy(d[k]) for k in d if k.startswith("init/")}
    if weights == "final":
        sd.update({k[len("final/"):]: torch.from_numpy(d[k]) for k in d if k.startswith("final/")})
    m.load_state_dict(sd)
    return m.to(device)


def run_case(name, device):
    n_lines, bs, stride = (int(x) for x in E[f"cfg/{name}"])
    lines = corpus(7 + n_lines, n_lines)
    m = model(str(E[f"weights/{name}"]), device)
    return ev.evaluate_perplexity(m, ByteTokenizer(), "wikitext2", device=device, batch_size=bs,
                                  stride=stride, text=lines)


def test_windows_cover_every_token_once():
    for n, L, s in ((1000, 64, 16), (1000, 64, 512), (64, 64, 16), (65, 64, 64), (7, 64, 3)):
        plan = ev.eval_windows(n, L, s)
        scored = sum(ev._active(e - b, t) for b, e, t in plan)
        if s <= L:  # overlapping windows reach the end and score each token exactly once
            assert plan[-1][1] == n and scored == n
        else:       # stride past the window: the reference skips tokens (its default 512 / 64)
            assert scored == sum(e - b for b, e, _ in plan) < n


@pytest.mark.parametrize("name", CASES[:2])
def test_ppl_cpu_matches_reference(name):
    ppl = run_case(name, "cpu")
    ref = float(E[f"ppl/{name}"])
    assert abs(ppl - ref) <= 1e-9 * ref, (ppl, ref)


def test_calibration_windows_match_reference():
    seeds = json.loads(str(E["corpus_seeds"]))
    train = corpus(seeds["train"], seeds["lines"])
    for key in (k for k in E.files if k.startswith("calib/")):
        seed, n, L = (int(x) for x in key[len("calib/"):].split("_"))
        got = ev.get_loaders("wikitext2", ByteTokenizer(), n, L, seed, text=train)
        assert np.array_equal(torch.cat(got).numpy(), E[key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_ppl_gpu_matches_reference(name):
    ppl = run_case(name, "cuda:0")
    ref = float(E[f"ppl/{name}"])
    assert abs(ppl - ref) <= 1e-6 * ref, (ppl, ref)
