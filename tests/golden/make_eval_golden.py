"""Golden values for the PPL evaluator and the calibration sampler (§8(f)4):
run the REFERENCE's own ``eval_utils.evaluate_perplexity``
(/root/reference/src/TruncGPTQ/eval_utils.py:17-108) and
``data_utils.get_wikitext2`` (data_utils.py:34-63) in this container.

Offline stand-ins: ``load_dataset`` returns a fixed synthetic corpus (the
lines below, seeded), the tokenizer is a byte-level stub (id = byte), the
model is the tiny random Qwen3 of the harness fixture
h_qwen3tiny_eigh_w4a (its initial and its quantised weights, float32, CPU).
Everything else is the reference's code.  Output: ``e_eval.npz``.

    python tests/golden/make_eval_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402

from eval_corpus import ByteTokenizer, corpus  # noqa: E402  (shared with the tests)


def load_model(weights):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    d = np.load(os.path.join(HERE, "h_qwen3tiny_eigh_w4a.npz"))
    cfg = Qwen3Config(**json.loads(str(d["config"])))
    cfg._attn_implementation = "eager"
    m = Qwen3ForCausalLM(cfg).float().eval()
    sd = {k[len("init/"):]: torch.from_numpy(d[k]) for k in d if k.startswith("init/")}
    if weights == "final":
        sd.update({k[len("final/"):]: torch.from_numpy(d[k]) for k in d if k.startswith("final/")})
    m.load_state_dict(sd)
    return m


# name, weights, corpus lines, batch_size, stride
CASES = [
    ("init_b4_s16", "init", 400, 4, 16),
    ("final_b4_s16", "final", 400, 4, 16),
    ("init_b3_s512", "init", 2500, 3, 512),   # the reference default stride (window 64 < stride)
    ("final_b1_s40", "final", 120, 1, 40),
]


def main():
    make_golden.install_shim()
    import data_utils
    import eval_utils
    out = {}
    test_lines = {}
    for name, weights, n_lines, bs, stride in CASES:
        lines = corpus(7 + n_lines, n_lines)
        test_lines[name] = lines
        eval_utils.load_dataset = lambda *a, _l=lines, **k: {"text": _l}
        model = load_model(weights)
        with torch.no_grad():
            ppl = eval_utils.evaluate_perplexity(model, ByteTokenizer(), "wikitext2", device="cpu",
                                                 batch_size=bs, stride=stride)
        out[f"ppl/{name}"] = np.float64(ppl)
        out[f"cfg/{name}"] = np.array([n_lines, bs, stride], dtype=np.int64)
        out[f"weights/{name}"] = np.str_(weights)
        print(name, ppl)
    # calibration sampler: random 2048-token windows -> here 32-token windows
    train = corpus(1234, 3000)
    data_utils.load_dataset = lambda *a, **k: {"text": train}
    for seed, n, L in ((42, 16, 32), (3, 5, 100)):
        chunks = data_utils.get_wikitext2(ByteTokenizer(), n, L, seed)
        out[f"calib/{seed}_{n}_{L}"] = torch.cat(chunks).numpy().astype(np.int64)
    out["corpus_seeds"] = np.str_(json.dumps({"train": 1234, "lines": 3000}))
    np.savez_compressed(os.path.join(HERE, "e_eval.npz"), **out)
    print("wrote e_eval.npz")


if __name__ == "__main__":
    main()
