"""Synthetic corpus + byte tokenizer shared by make_eval_golden.py (which ran
the reference's evaluator on them) and tests/test_gpu_eval.py (which runs
ours).  Test data, not product code."""
import random
import types

import torch

WORDS = ["the", "of", "and", "quantization", "error", "matrix", "hessian", "layer", "rank",
         "column", "group", "scale", "model", "token", "weight", "a", "is", "in", "to", "="]


def corpus(seed, n_lines):
    rng = random.Random(seed)
    lines = []
    for i in range(n_lines):
        if rng.random() < 0.15:
            lines.append("")
        elif rng.random() < 0.1:
            lines.append(f" = = Section {i} = = ")
        else:
            lines.append(" ".join(rng.choice(WORDS) for _ in range(rng.randint(3, 14))) + " .")
    return lines


class ByteTokenizer:
    """Stub tokenizer: one token per UTF-8 byte (vocab 256), no specials."""
    pad_token_id = None
    eos_token_id = 0

    def __call__(self, text, return_tensors="pt", add_special_tokens=True, **kw):
        ids = torch.tensor([list(text.encode("utf-8"))], dtype=torch.long)
        return types.SimpleNamespace(input_ids=ids)
