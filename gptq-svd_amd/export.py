"""Packed checkpoint exporter (§8(f) rank 2; A13 -- the reference saves only
dequantised FP16 weights, quantize.py:262-273, README.md:133).

Layout (AutoGPTQ / GPTQModel "gptq_v2" checkpoint format, static groups):
for every quantised linear ``<name>``
  ``<name>.qweight`` int32 (in*b/32, out)  codes packed along in_features,
  ``<name>.qzeros``  int32 (G, out*b/32)   zero points packed along out_features
                                           (true zeros: v2, not the v1 "zero - 1"),
  ``<name>.scales``  fp16  (G, out)        (or fp32 with scale_dtype=torch.float32),
  ``<name>.g_idx``   int32 (in,)           = column // group_size (static groups
                                           in the original column order, so it
                                           is only the trivial map),
  ``<name>.bias``    as in the model;
every other tensor of the state dict as is.  ``quantize_config.json`` records
bits / group_size / sym / desc_act=false / static_groups=true and the
TruncGPTQ settings and per-layer ranks.  Dequantisation:
W[:, j] = (code_u[:, j] - zero_u[:, g(j)]) * scale[:, g(j)], with symmetric
codes stored +2^(b-1) (so zero_u = 2^(b-1)).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional

import torch

__all__ = ["save_quantized", "read_quantized"]


def save_quantized(path: str, model: torch.nn.Module, packed: Dict[str, Dict[str, torch.Tensor]],
                   w_bits: int, group_size: int, sym: bool,
                   extra_config: Optional[Dict[str, Any]] = None,
                   scale_dtype: torch.dtype = torch.float16) -> str:
    """Write ``model.safetensors`` + ``quantize_config.json`` (+ ``config.json``
    when the model has a HF config) into `path`; returns the tensor file path."""
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    sd = model.state_dict()
    tensors: Dict[str, torch.Tensor] = {}
    for name, t in packed.items():
        in_features = t["qweight"].shape[0] * 32 // w_bits
        g = group_size if group_size > 0 else in_features
        tensors[f"{name}.qweight"] = t["qweight"].contiguous().cpu()
        tensors[f"{name}.qzeros"] = t["qzeros"].contiguous().cpu()
        tensors[f"{name}.scales"] = t["scales"].to(scale_dtype).contiguous().cpu()
        tensors[f"{name}.g_idx"] = (torch.arange(in_features, dtype=torch.int32) // g)
    for k, v in sd.items():
        mod = k.rsplit(".", 1)[0]
        if mod in packed and k.endswith(".weight"):
            continue  # replaced by the packed tensors
        tensors[k] = v.detach().contiguous().cpu()
    # tied parameters share storage: safetensors refuses aliases, so clone
    seen = {}
    for k in list(tensors):
        key = (tensors[k].untyped_storage().data_ptr(), tensors[k].storage_offset())
        if key in seen:
            tensors[k] = tensors[k].clone()
        seen[key] = k
    fn = os.path.join(path, "model.safetensors")
    save_file(tensors, fn, metadata={"format": "pt"})
    qc = {"bits": int(w_bits), "group_size": int(group_size), "sym": bool(sym),
          "desc_act": False, "static_groups": True, "true_sequential": True,
          "quant_method": "gptq", "checkpoint_format": "gptq_v2",
          "scale_dtype": str(scale_dtype).replace("torch.", "")}
    if extra_config:
        qc["truncgptq"] = extra_config
    with open(os.path.join(path, "quantize_config.json"), "w") as f:
        json.dump(qc, f, indent=2)
    cfg = getattr(model, "config", None)
    if cfg is not None and hasattr(cfg, "save_pretrained"):
        cfg.save_pretrained(path)
    return fn


def read_quantized(path: str):
    """(tensors dict, quantize_config dict) of a checkpoint written by
    save_quantized (plain reads; unpacking lives with the consumer)."""
    from safetensors.torch import load_file
    tensors = load_file(os.path.join(path, "model.safetensors"))
    with open(os.path.join(path, "quantize_config.json")) as f:
        qc = json.load(f)
    return tensors, qc
