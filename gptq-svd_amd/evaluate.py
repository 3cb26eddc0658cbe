"""Perplexity evaluation and calibration sampling: counterparts of the
reference's ``eval_utils.evaluate_perplexity``
(/root/reference/src/TruncGPTQ/eval_utils.py:17-108) and
``data_utils.get_loaders`` / ``get_wikitext2`` (data_utils.py:16-63), §8(f)4.

Same windows, same sampling, same arithmetic:
* PPL: the test split joined with "\\n\\n", tokenised once; windows of
  ``max_length`` tokens (``model.seqlen``, else
  ``config.max_position_embeddings``, else 2048) start every ``stride``
  tokens; a window scores only the tokens past the previous window's end
  (earlier targets are -100); short windows are right-padded (pad id, else
  eos) with a zero attention mask.  NLL = sum over batches of the model's
  mean loss (float32) x the batch's active target count, PPL =
  exp(float32(NLL / tokens)).
* Calibration: the train split joined and tokenised without special tokens,
  ``random.seed(seed)``, ``n_samples`` windows ``ids[i : i + seq_len]`` with
  ``i = random.randint(0, len - seq_len - 1)``.

What differs, deliberately: the loop never synchronises per batch -- the
active-token counts come from the window plan on the host and the NLL is
accumulated on the device in float64 (the reference's Python-float
arithmetic, op for op), one read at the end; ``text=`` supplies the corpus
directly (this image has no network; ``load_dataset`` is used otherwise).
"""
from __future__ import annotations

import logging
import random
from typing import List, Optional, Sequence, Tuple

import torch

__all__ = ["eval_windows", "evaluate_perplexity", "sample_windows", "get_loaders",
           "get_wikitext2"]

logger = logging.getLogger(__name__)


def _wikitext2(split: str, text: Optional[Sequence[str]]):
    if text is None:
        from datasets import load_dataset
        text = load_dataset("wikitext", "wikitext-2-raw-v1", split=split)["text"]
    return "\n\n".join(text)


def eval_windows(n_tokens: int, max_length: int, stride: int) -> List[Tuple[int, int, int]]:
    """(begin, end, target_len) of every evaluation window (eval_utils.py:51-65)."""
    out = []
    prev_end = 0
    for begin in range(0, n_tokens, stride):
        end = min(begin + max_length, n_tokens)
        out.append((begin, end, end - prev_end))
        prev_end = end
        if end == n_tokens:
            break
    return out


def _active(length: int, target_len: int) -> int:
    """Targets left by `tar[:, :-target_len] = -100` on a row of `length`
    (target_len >= 1 always: windows end strictly later than the last)."""
    return length if target_len >= length else target_len


@torch.no_grad()
def evaluate_perplexity(model, tokenizer, dataset: str = "wikitext2", device="cuda",
                        batch_size: int = 4, stride: int = 512,
                        text: Optional[Sequence[str]] = None) -> float:
    """Strided sliding-window perplexity (eval_utils.py:17-108)."""
    logger.info(f"  [eval] Loading {dataset}...")
    if dataset != "wikitext2":
        return -1
    enc = tokenizer(_wikitext2("test", text), return_tensors="pt")
    ids = enc.input_ids
    if hasattr(model, "seqlen"):
        max_length = model.seqlen
    elif hasattr(model.config, "max_position_embeddings"):
        max_length = model.config.max_position_embeddings
    else:
        max_length = 2048
    pad_id = tokenizer.pad_token_id if tokenizer.pad_token_id is not None else tokenizer.eos_token_id
    n_tokens = ids.size(1)
    logger.info(f"  [eval] Dataset tokens: {n_tokens} | Window: {max_length} | Stride: {stride}")
    plan = eval_windows(n_tokens, max_length, stride)
    model.eval()
    total_nll = torch.zeros((), dtype=torch.float64, device=device)
    total_tokens = 0
    for i in range(0, len(plan), batch_size):
        rows, tars, masks = [], [], []
        active = 0
        for begin, end, target_len in plan[i: i + batch_size]:
            inp = ids[:, begin:end]
            tar = inp.clone()
            tar[:, :-target_len] = -100
            active += _active(inp.shape[1], target_len)
            pad = max_length - inp.shape[1]
            mask = torch.ones_like(inp)
            if pad > 0:
                inp = torch.cat([inp, torch.full((1, pad), pad_id)], dim=1)
                tar = torch.cat([tar, torch.full((1, pad), -100)], dim=1)
                mask = torch.cat([mask, torch.zeros((1, pad), dtype=torch.long)], dim=1)
            rows.append(inp)
            tars.append(tar)
            masks.append(mask)
        out = model(torch.cat(rows).to(device), labels=torch.cat(tars).to(device),
                    attention_mask=torch.cat(masks).to(device))
        if active > 0:
            # float(loss_f32) * active in float64, then the running sum (:95-97)
            total_nll += out.loss.float().double() * active
            total_tokens += active
    if total_tokens == 0:
        return float("inf")
    return torch.exp(torch.tensor(total_nll.item() / total_tokens)).item()


def sample_windows(input_ids: torch.Tensor, n_samples: int, seq_len: int,
                   seed: int = 42) -> List[torch.Tensor]:
    """n_samples random (1, seq_len) windows of a (1, N) token tensor
    (data_utils.py:52-60: Python's `random`, seeded once)."""
    full_len = input_ids.shape[1]
    random.seed(seed)
    out = []
    for _ in range(n_samples):
        i = random.randint(0, full_len - seq_len - 1)
        out.append(input_ids[:, i: i + seq_len].clone())
    return out


def get_wikitext2(tokenizer, n_samples: int, seq_len: int, seed: int = 42,
                  text: Optional[Sequence[str]] = None) -> List[torch.Tensor]:
    """Calibration windows from the WikiText-2 train split (data_utils.py:34-63)."""
    logging.info(f"Loading wikitext2... (total samples: {n_samples})")
    enc = tokenizer(_wikitext2("train", text), return_tensors="pt", add_special_tokens=False)
    logging.info(f"[DATA] Full dataset tokens: {enc.input_ids.shape[1]}")
    out = sample_windows(enc.input_ids, n_samples, seq_len, seed)
    logging.info(f"[DATA] Collected {len(out)} random batches of length {seq_len}.")
    return out


def get_loaders(name: str, tokenizer, n_samples: int = 128, seq_len: int = 2048, seed: int = 42,
                text: Optional[Sequence[str]] = None) -> List[torch.Tensor]:
    """data_utils.py:16-31 (wikitext2; C4 streaming needs the network and is
    not offered here)."""
    if name == "wikitext2":
        return get_wikitext2(tokenizer, n_samples, seq_len, seed, text)
    raise ValueError(f"Unknown dataset: {name}")
