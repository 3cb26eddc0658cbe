"""Layer-sequential quantization loop: counterpart of the reference harness
(/root/reference/src/TruncGPTQ/quantize.py:89-252 and model_utils.py:52-181),
§8(f) rank 1.

The reference's data flow is kept exactly: capture the inputs of the first
decoder layer; for each layer and each sequenced group (q/k/v -> o ->
gate/up -> down), hook the group's first linear, run every calibration batch
through the layer to accumulate H (FP64 MFMA SYRK), factorise once per group
(``process_hessian_alt`` for "eigh", ``process_hessian`` for "gptq"),
quantize each linear of the group with ``gptq_fwrd`` (block 1024) and write
the dequantised weight back; then re-run the calibration batches through the
quantised layer to produce the next layer's inputs.

What differs, deliberately:
* a calibration pass stops each batch at the group's first linear (a
  forward pre-hook accumulates its input and ends the pass): the reference
  runs the whole layer and throws the output away (quantize.py:139-148), so
  H is the same and the layer's remaining work is skipped;
* no ``cleanup()`` (gc + empty_cache + device synchronize) after every batch
  and every module (quantize.py:28-35): activations and H stay resident and
  the work is stream-ordered -- 288 GB of HBM holds a whole layer's
  calibration set several times over;
* the re-forward stores each batch's actual size (the reference indexes with
  the accumulation loop's last ``curr_batch_size``, quantize.py:233-234,
  which drops rows when n_samples % batch_size != 0), and a short last batch
  gets the captured keyword tensors (attention mask ...) cut to its size;
* OPT works: its sublayer names (``self_attn.out_proj``, ``fc1``, ``fc2``)
  are sequenced, and no ``model.model.rotary_emb`` is required
  (quantize.py:98 reads it and never uses it);
* optional packing: with ``pack=True`` every quantised linear's AutoGPTQ
  tensors are kept (``export.save_quantized`` writes them);
* multi-GPU (one process per GPU, ``torch.distributed`` initialised): the
  calibration sequences are sharded over the ranks (rank r takes sequences
  r, r + world, ...) and stay sharded through the whole model; each group's H
  is the all-reduce (SUM) of the ranks' FP64 sums x^T x and sample counts,
  divided by the total count -- the single-process H up to the order of the
  FP64 additions; every rank factorises that H (the solver is
  deterministic, so every rank holds the same U, perm -- checked by a
  fingerprint reduction before any row is quantised); each linear's rows
  are quantised by their owning rank (``dist.shard_rows``; rows are
  independent given U and perm) and all-gathered, so every rank writes the
  same dequantised weight.  The reference has no multi-GPU mode: it loads
  the model on one device (model_utils.py:45, ``device_map=device``) and
  moves one layer at a time to it (quantize.py:101, :250).  Here each GPU
  holds the whole model (288 GB) and the ranks split the calibration forward
  passes, the H accumulation and the quantisation.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Dict, List, Optional, Sequence

import torch
from torch import nn

from . import dist as tgdist
from .gptq_utils import (HessianAccumulator, Quantizer, gptq_fwrd, log_quantization_error,
                         pack_quantized, process_hessian, process_hessian_alt)

__all__ = ["get_layers", "get_sequenced_groups", "capture_initial_inputs", "quantize_model",
           "adaptive_eps", "StageClock", "check_factor_agrees", "run_and_record"]


def get_layers(model: nn.Module) -> nn.ModuleList:
    """Decoder layers of Llama/Qwen (model.model.layers), OPT
    (model.model.decoder.layers), GPT-style (transformer.h); model_utils.py:52-74."""
    inner = getattr(model, "model", None)
    if inner is not None:
        if hasattr(inner, "layers"):
            return inner.layers
        if hasattr(inner, "decoder") and hasattr(inner.decoder, "layers"):
            return inner.decoder.layers
    if hasattr(model, "layers"):
        return model.layers
    if hasattr(model, "transformer") and hasattr(model.transformer, "h"):
        return model.transformer.h
    raise ValueError("Could not find layers in model architecture")


# Sublayers that read the same input share one Hessian (model_utils.py:77-108),
# in dependency order.  OPT's names are added (its out_proj / fc1 / fc2).
_GROUPS = [
    ["self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"],
    ["self_attn.o_proj", "self_attn.out_proj"],
    ["mlp.gate_proj", "mlp.up_proj", "fc1"],
    ["mlp.down_proj", "fc2"],
]


def get_sequenced_groups(layer: nn.Module) -> List[List[str]]:
    names = {n for n, _ in layer.named_modules()}
    groups = []
    for cand in _GROUPS:
        g = [n for n in cand if n in names]
        if g:
            groups.append(g)
    return groups


def adaptive_eps(layer_name: str, base_eps: float) -> float:
    """quantize.py:17-20: down_proj / o_proj use a 10x smaller eps."""
    if any(x in layer_name for x in ["down_proj", "o_proj"]):
        return base_eps * 0.1
    return base_eps


def _to(v, device):
    if isinstance(v, torch.Tensor):
        return v.to(device)
    if isinstance(v, (list, tuple)):
        return type(v)(_to(x, device) for x in v)
    return v


def _batch_slice(v, cap: int, b: int):
    """Keyword tensors captured with a batch of `cap` sequences (attention
    masks, position embeddings of some models), cut to a batch of b < cap."""
    if isinstance(v, torch.Tensor):
        return v[:b] if v.dim() > 0 and v.shape[0] == cap else v
    if isinstance(v, (list, tuple)):
        return type(v)(_batch_slice(x, cap, b) for x in v)
    return v


def _submodule(root: nn.Module, name: str) -> nn.Module:
    cur = root
    for p in name.split("."):
        cur = getattr(cur, p)
    return cur


class _Stop(Exception):
    pass


# Decoder layers whose forward is, line for line (transformers 5.x,
# modeling_llama.py LlamaDecoderLayer.forward / LlamaMLP.forward):
#   h = x + self_attn(input_layernorm(x)); out = h + mlp(post_attention_layernorm(h))
#   mlp(m) = down_proj(act_fn(gate_proj(m)) * up_proj(m))
_STAGED_LAYERS = {"LlamaDecoderLayer", "Qwen2DecoderLayer", "Qwen3DecoderLayer",
                  "MistralDecoderLayer"}
_STAGED_MLPS = {"LlamaMLP", "Qwen2MLP", "Qwen3MLP", "MistralMLP"}


def _staged_layer(layer: nn.Module) -> bool:
    """True when the quantisation loop may run `layer` group by group from
    cached activations (``quantize_model(staged=True)``): one of the decoder
    layer classes above, with its standard submodules and no hooks of its
    own that a partial forward would skip."""
    if type(layer).__name__ not in _STAGED_LAYERS:
        return False
    mlp, attn = getattr(layer, "mlp", None), getattr(layer, "self_attn", None)
    if mlp is None or attn is None or type(mlp).__name__ not in _STAGED_MLPS:
        return False
    need = ("input_layernorm", "post_attention_layernorm")
    if not all(hasattr(layer, n) for n in need) or not hasattr(attn, "o_proj"):
        return False
    for m in (layer, mlp):
        if m._forward_hooks or m._forward_pre_hooks:
            return False
    return True


class StageClock:
    """Per-stage device time of the layer loop, from HIP events recorded on
    the current stream (no host sync until ``totals()``).  Stage names:
    capture, calib_forward, syrk, allreduce, factor_n<n>, quantize,
    reforward; ``calib_forward`` excludes the SYRK launches inside it."""

    def __init__(self):
        self._spans: Dict[str, list] = {}
        self.counts: Dict[str, int] = {}

    def start(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, name: str, ev0) -> None:
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self._spans.setdefault(name, []).append((ev0, ev1))
        self.counts[name] = self.counts.get(name, 0) + 1

    def totals(self) -> Dict[str, float]:
        torch.cuda.synchronize()
        out = {k: sum(a.elapsed_time(b) for a, b in v) / 1e3 for k, v in self._spans.items()}
        if "calib_forward" in out and "syrk" in out:
            out["calib_forward"] -= out["syrk"]
        return out


def capture_initial_inputs(model: nn.Module, input_ids_list: Sequence[torch.Tensor],
                           device="cuda", batch_size: int = 1):
    """Inputs of the first decoder layer for every calibration sequence, plus
    the keyword arguments the model passes it (model_utils.py:123-181)."""
    layers = get_layers(model)
    ids = torch.cat(list(input_ids_list), dim=0)
    n_samples, seq_len = ids.shape
    dtype = next(model.parameters()).dtype
    inps = torch.zeros((n_samples, seq_len, model.config.hidden_size), dtype=dtype, device=device)
    state: Dict[str, Any] = {"i": 0, "kwargs": None}
    first = layers[0]

    def pre_hook(mod, args, kwargs):
        x = args[0] if args else kwargs["hidden_states"]
        b = x.shape[0]
        inps[state["i"]: state["i"] + b] = x.to(device)
        state["i"] += b
        if state["kwargs"] is None:
            state["kwargs"] = {k: v for k, v in kwargs.items() if k != "hidden_states"}
        raise _Stop

    h = first.register_forward_pre_hook(pre_hook, with_kwargs=True)
    cfg = getattr(model, "config", None)
    use_cache = getattr(cfg, "use_cache", None)
    if cfg is not None:
        cfg.use_cache = False  # as quantize.py:67: no KV cache object in the captured kwargs
    try:
        model_device = next(model.parameters()).device
        for i in range(0, n_samples, batch_size):
            try:
                model(ids[i: i + batch_size].to(model_device), use_cache=False)
            except _Stop:
                pass
    finally:
        h.remove()
        if cfg is not None:
            cfg.use_cache = use_cache
    kw = state["kwargs"] or {}
    for k in ("past_key_values", "past_key_value"):
        kw.pop(k, None)
    return inps, kw


def _world(pg):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(pg), dist.get_rank(pg)


def allreduce_hessian(acc, pg=None) -> None:
    """Sum the ranks' unnormalised H (FP64) and sample counts in place, so
    ``acc.get_hessian()`` is the H of all ranks' rows together."""
    world, _ = _world(pg)
    if world == 1:
        return
    acc.H.copy_(tgdist.all_reduce_sum(acc.H, pg))
    cnt = torch.tensor([float(acc.n_samples)], dtype=torch.float64, device=acc.H.device)
    acc.n_samples = int(tgdist.all_reduce_sum(cnt, pg).item())


def check_factor_agrees(R: torch.Tensor, perm: torch.Tensor, pg=None) -> None:
    """Every rank factorises the same all-reduced H and must hold the same
    (U, perm, k); rows quantised with different factors would be stitched
    into one weight silently.  A fingerprint (k, a position-weighted sum of
    perm, sum and sum of squares of U) is reduced by MIN and MAX; any
    difference raises on every rank."""
    import torch.distributed as dist
    world, _ = _world(pg)
    if world == 1:
        return
    n = perm.numel()
    pos = torch.arange(1, n + 1, dtype=torch.float64, device=perm.device)
    Rd = R.to(torch.float64)
    fp = torch.stack([torch.tensor(float(R.shape[0]), dtype=torch.float64, device=R.device),
                      (perm.to(torch.float64) * pos).sum(), Rd.sum(), (Rd * Rd).sum()])
    # compared as bit patterns: a NaN or Inf in a (shared) factor must not read
    # as a disagreement between ranks (NaN != NaN as floats)
    bits = fp.view(torch.int64)
    lo, hi = bits.clone(), bits.clone()
    if fp.is_cuda and dist.get_backend(pg) == "gloo":
        lo, hi = lo.cpu(), hi.cpu()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=pg)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=pg)
    if not torch.equal(lo, hi):
        raise RuntimeError("ranks disagree on the factorisation of the shared Hessian "
                           f"(fingerprint min {lo.view(torch.float64).tolist()} "
                           f"max {hi.view(torch.float64).tolist()})")
    if not bool(torch.isfinite(fp).all()):
        raise RuntimeError("the shared factorisation is not finite on every rank "
                           f"(fingerprint {fp.tolist()}): check the layer's Hessian")


def quantize_linear_sharded(W: torch.Tensor, R: torch.Tensor, perm: torch.Tensor,
                            w_bits: int, group_size: int, sym: bool, block_size: int,
                            use_triton: bool, pg=None):
    """gptq_fwrd over this rank's rows of W, gathered: returns (dequantised W,
    rank, Quantizer holding the gathered codes / scale / zero) on every rank."""
    world, rank = _world(pg)
    m, n = W.shape
    r0, r1 = tgdist.shard_rows(m, world, rank)
    q = Quantizer(w_bits=w_bits, group_size=group_size, sym=sym)
    G = n // (group_size if group_size > 0 else n)
    if r1 > r0:
        Wq, k = gptq_fwrd(W[r0:r1], R, q, perm, block_size=block_size, use_triton=use_triton)
        Wq = Wq.to(W.dtype)
        codes = q.codes.to(torch.uint8)
        scale, zero = q.scale.squeeze(-1).float(), q.zero.squeeze(-1).float()
    else:
        # no rows here (m < world): still join every gather
        k = R.shape[0]
        Wq = torch.empty((0, n), dtype=W.dtype, device=W.device)
        codes = torch.empty((0, n), dtype=torch.uint8, device=W.device)
        scale = torch.empty((0, G), dtype=torch.float32, device=W.device)
        zero = torch.empty((0, G), dtype=torch.float32, device=W.device)
    Wq = tgdist.all_gather_rows(Wq, m, pg)
    q.codes = tgdist.all_gather_rows(codes, m, pg)
    q.scale = tgdist.all_gather_rows(scale, m, pg).unsqueeze(-1)
    q.zero = tgdist.all_gather_rows(zero, m, pg).unsqueeze(-1)
    return Wq, k, q


@torch.no_grad()
def quantize_model(model: nn.Module, input_ids_list: Sequence[torch.Tensor], mode: str = "eigh",
                   w_bits: int = 4, group_size: int = -1, sym: bool = False, eps: float = 1e-2,
                   threshold_method: str = "mean_trimmed", actorder: bool = False,
                   damp_percent: float = 0.01, use_adaptive_eps: bool = False,
                   batch_size: int = 8, device="cuda", block_size: int = 1024,
                   pack: bool = False, offload: bool = False, pg=None, early_stop: bool = True,
                   clock: Optional[StageClock] = None, save_path: Optional[str] = None,
                   run_config: Optional[Dict[str, Any]] = None,
                   staged: Optional[bool] = None) -> Dict[str, Any]:
    """Quantise every sequenced linear of `model` in place (layer by layer).

    mode "eigh" = TruncGPTQ (process_hessian_alt + gptq_fwrd(use_triton=True));
    mode "gptq" = the GPTQ comparator (process_hessian + use_triton=False).
    `offload`: move each layer to `device` for its turn and back to the CPU
    afterwards (the reference's policy, quantize.py:101, :239); by default
    the model stays where it is (a whole 8B/70B model fits in 288 GB).
    `pg`: process group of the multi-GPU mode (module docstring); it is on
    whenever torch.distributed is initialised with more than one rank.
    `early_stop`: a calibration pass ends each batch at the group's first
    linear -- its input is accumulated into H, then the rest of the layer is
    skipped (the reference runs the whole layer and discards the output,
    quantize.py:139-148, so H is the same).  `staged` (default: `early_stop`
    and not `offload`): Llama / Qwen2 / Qwen3 / Mistral decoder layers keep
    each batch's intermediate activations between groups instead of re-running
    the layer from its input for every group (``_staged_layer``; bit-identical
    result, about a third of the forward work).  Its memory cost is about
    tokens x (2 hidden + intermediate) x 2 bytes on the device (13 GB for
    128 x 2048 tokens at Qwen3-8B widths, ~19 GB at Llama-3-70B's), which the
    per-group passes never hold -- hence off by default with `offload`, the
    memory-tight mode.  `clock`: a StageClock that
    receives per-stage device times.
    `save_path`: write the run's ``quantization.log`` and ``results.json`` there
    in the reference's schema (``runlog.py``; rank 0 only in multi-GPU mode);
    `run_config` adds to / overrides the ``config`` block (e.g. model_id,
    n_samples, seq_len).  ``quantized_ppl`` is added by ``runlog.RunLog.finish``
    when the caller evaluates afterwards (see ``run_and_record``).
    Returns {"layer_stats": [...], "total_time": s, "packed": {name: tensors}}.
    """
    if mode not in ("eigh", "gptq"):
        raise ValueError(f"mode must be 'eigh' or 'gptq', got {mode!r}")
    if save_path is not None:
        res = run_and_record(model, input_ids_list, save_path, run_config, mode=mode,
                             w_bits=w_bits, group_size=group_size, sym=sym, eps=eps,
                             threshold_method=threshold_method, actorder=actorder,
                             damp_percent=damp_percent, use_adaptive_eps=use_adaptive_eps,
                             batch_size=batch_size, device=device, block_size=block_size,
                             pack=pack, offload=offload, pg=pg, early_stop=early_stop, clock=clock,
                             staged=staged)
        return res
    t_start = time.time()
    world, rank = _world(pg)
    if world > 1:
        input_ids_list = list(input_ids_list)
        # the same test on every rank, so all of them raise together
        if len(input_ids_list) < world:
            raise ValueError(f"fewer calibration sequences ({len(input_ids_list)}) than ranks "
                             f"({world})")
        input_ids_list = input_ids_list[rank::world]
    ev = clock.start() if clock else None
    inps, layer_kwargs = capture_initial_inputs(model, input_ids_list, device=device,
                                                batch_size=batch_size)
    if clock:
        clock.stop("capture", ev)
    kw = {k: _to(v, device) for k, v in layer_kwargs.items()}
    kw["use_cache"] = False
    outs = torch.zeros_like(inps)
    n_samples = inps.shape[0]
    layers = get_layers(model)
    qual = {id(m): n for n, m in model.named_modules()}  # packed tensors use state-dict names
    stats: List[Dict[str, Any]] = []
    packed: Dict[str, Dict[str, torch.Tensor]] = {}

    cap = min(batch_size, n_samples)  # batch the keyword tensors were captured with

    def run_layer(layer, dst: Optional[torch.Tensor]):
        for j in range(0, n_samples, batch_size):
            x = inps[j: j + batch_size]
            kwb = kw if x.shape[0] == cap else {k: _batch_slice(v, cap, x.shape[0])
                                                 for k, v in kw.items()}
            try:
                out = layer(x, **kwb)
            except _Stop:
                continue
            if dst is not None:
                out = out[0] if isinstance(out, (tuple, list)) else out
                dst[j: j + out.shape[0]] = out

    def accumulate(acc):
        def hook(mod, args, kwargs):
            x = args[0] if args else kwargs["input"]
            ev = clock.start() if clock else None
            acc.add_batch(x.detach())
            if clock:
                clock.stop("syrk", ev)
            if early_stop:
                raise _Stop
        return hook

    def solve_group(i, layer, names, acc):
        """All-reduce, factorise and quantise one sequenced group."""
        cur_eps = adaptive_eps(names[0], eps) if use_adaptive_eps else eps
        ev = clock.start() if clock else None
        allreduce_hessian(acc, pg)
        if clock and world > 1:
            clock.stop("allreduce", ev)
            ev = clock.start()
        H = acc.get_hessian()
        if mode == "eigh":
            R, R_x, perm = process_hessian_alt(H, threshold=cur_eps,
                                               threshold_method=threshold_method)
        else:
            R, perm = process_hessian(H, actorder=actorder, damp_percent=damp_percent)
            R_x = None
        if clock:
            clock.stop(f"factor_n{H.shape[0]}", ev)
        del H
        if world > 1:
            check_factor_agrees(R, perm, pg)
        ev = clock.start() if clock else None
        for name in names:
            sub = _submodule(layer, name)
            q = Quantizer(w_bits=w_bits, group_size=group_size, sym=sym)
            t0 = time.time()
            if world > 1:
                W = sub.weight.data.float()
                Wq, k, q = quantize_linear_sharded(W, R, perm, w_bits, group_size, sym,
                                                   block_size, mode == "eigh", pg)
                if R_x is not None and rank == 0:
                    log_quantization_error(W, Wq, R_x, perm)
            else:
                Wq, k = gptq_fwrd(sub.weight.data.float(), R, q, perm,
                                  block_size=block_size, use_triton=(mode == "eigh"), R_x=R_x)
            sub.weight.copy_(Wq)
            full = f"layer_{i}.{name}"
            if pack:
                qw, qz, sc = pack_quantized(q)
                packed[qual.get(id(sub), full)] = dict(qweight=qw, qzeros=qz, scales=sc)
            dt = time.time() - t0
            used = k if mode == "eigh" else "N/A"
            logging.info(f"   {name: <15} | Rank: {str(used): <4} | Time: {dt:.2f}s")
            stats.append({"name": full, "rank": used, "time": dt})
        if clock:
            clock.stop("quantize", ev)

    def batches():
        for j in range(0, n_samples, batch_size):
            x = inps[j: j + batch_size]
            kwb = kw if x.shape[0] == cap else {k: _batch_slice(v, cap, x.shape[0])
                                                 for k, v in kw.items()}
            yield j, x, kwb

    def add(acc, x):
        ev = clock.start() if clock else None
        acc.add_batch(x)
        if clock:
            clock.stop("syrk", ev)

    def layer_generic(i, layer):
        for gi, names in enumerate(get_sequenced_groups(layer)):
            logging.info(f"[Layer {i + 1}/{len(layers)}] Group {gi + 1}: {', '.join(names)}")
            first = _submodule(layer, names[0])
            acc = HessianAccumulator(first.weight.shape[1], device=device)
            hook = first.register_forward_pre_hook(accumulate(acc), with_kwargs=True)
            ev = clock.start() if clock else None
            try:
                run_layer(layer, None)
            finally:
                hook.remove()
            if clock:
                clock.stop("calib_forward", ev)
            solve_group(i, layer, names, acc)
            del acc
        ev = clock.start() if clock else None
        run_layer(layer, outs)
        if clock:
            clock.stop("reforward", ev)

    def layer_staged(i, layer):
        """The same four groups and the same H inputs as ``layer_generic``,
        computed once each: every batch's intermediate activations (attention
        output, post-attention residual, MLP input, gated MLP activation) are
        kept, so each group's calibration pass runs only the sublayers between
        the previous group's linears (quantised by then) and its own, and the
        re-forward is the last residual add.  The operations and their order
        are those of the decoder layer's forward, so H, the quantised weights
        and the next layer's inputs are bit-identical to ``layer_generic``."""
        attn, mlp = layer.self_attn, layer.mlp
        groups = [["self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"],
                  ["self_attn.o_proj"], ["mlp.gate_proj", "mlp.up_proj"], ["mlp.down_proj"]]
        cache: Dict[str, List[torch.Tensor]] = {"a": [], "h": [], "m": [], "d": []}

        def grab(mod, args, kwargs):
            cache["a"].append(args[0] if args else kwargs["input"])
            raise _Stop

        for gi, names in enumerate(groups):
            logging.info(f"[Layer {i + 1}/{len(layers)}] Group {gi + 1}: {', '.join(names)}")
            acc = HessianAccumulator(_submodule(layer, names[0]).weight.shape[1], device=device)
            ev = clock.start() if clock else None
            for bi, (j, x, kwb) in enumerate(batches()):
                if gi == 0:
                    add(acc, layer.input_layernorm(x))
                elif gi == 1:
                    hook = attn.o_proj.register_forward_pre_hook(grab, with_kwargs=True)
                    try:
                        attn(hidden_states=layer.input_layernorm(x), **kwb)
                    except _Stop:
                        pass
                    finally:
                        hook.remove()
                    add(acc, cache["a"][bi])
                elif gi == 2:
                    h = x + attn.o_proj(cache["a"][bi])
                    cache["a"][bi] = None
                    m = layer.post_attention_layernorm(h)
                    cache["h"].append(h)
                    cache["m"].append(m)
                    add(acc, m)
                else:
                    m = cache["m"][bi]
                    cache["m"][bi] = None
                    d = mlp.act_fn(mlp.gate_proj(m)) * mlp.up_proj(m)
                    cache["d"].append(d)
                    add(acc, d)
            if clock:
                clock.stop("calib_forward", ev)
            solve_group(i, layer, names, acc)
            del acc
        ev = clock.start() if clock else None
        for bi, (j, x, kwb) in enumerate(batches()):
            out = cache["h"][bi] + mlp.down_proj(cache["d"][bi])
            cache["h"][bi] = cache["d"][bi] = None
            outs[j: j + out.shape[0]] = out
        if clock:
            clock.stop("reforward", ev)

    for i, layer in enumerate(layers):
        t_layer = time.time()
        if offload:
            layer = layer.to(device)
        use_staged = (early_stop and not offload) if staged is None else staged
        if use_staged and _staged_layer(layer):
            layer_staged(i, layer)
        else:
            layer_generic(i, layer)
        inps, outs = outs, inps
        if offload:
            layers[i] = layer.to("cpu")
        logging.info(f"[*] Layer {i + 1}/{len(layers)} completed in {time.time() - t_layer:.2f}s")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return {"layer_stats": stats, "total_time": time.time() - t_start, "packed": packed}


def run_and_record(model: nn.Module, input_ids_list: Sequence[torch.Tensor], save_path: str,
                   run_config: Optional[Dict[str, Any]] = None, evaluate=None,
                   **kw) -> Dict[str, Any]:
    """``quantize_model`` with the reference's run records (quantize.py:48-66,
    :254-284): ``<save_path>/quantization.log`` receives every log line of the
    run in the reference's format and ``<save_path>/results.json`` the config,
    the per-module ``layer_stats`` and the metrics.  ``evaluate`` (optional):
    a callable ``model -> ppl`` run after quantisation (e.g.
    ``evaluate.evaluate_perplexity`` bound to a tokenizer); its value becomes
    ``metrics.quantized_ppl`` as at quantize.py:281.  In multi-GPU mode only
    rank 0 writes the files; every rank runs the same quantisation."""
    from . import runlog
    input_ids_list = list(input_ids_list)
    world, rank = _world(kw.get("pg"))
    cfg = runlog.reference_config(
        device=str(kw.get("device", "cuda")), n_samples=len(list(input_ids_list)),
        seq_len=int(input_ids_list[0].shape[-1]) if len(input_ids_list) else 0,
        batch_size=kw.get("batch_size", 8), w_bits=kw.get("w_bits", 4),
        group_size=kw.get("group_size", -1), sym=bool(kw.get("sym", False)),
        eps=kw.get("eps", 1e-2), mode=kw.get("mode", "eigh"),
        threshold_method=kw.get("threshold_method", "mean_trimmed"),
        actorder=bool(kw.get("actorder", False)), damp_percent=kw.get("damp_percent", 0.01),
        adaptive_eps=bool(kw.get("use_adaptive_eps", False)), save_path=save_path, no_save=True)
    mid = getattr(getattr(model, "config", None), "_name_or_path", None)
    if mid:
        cfg["model_id"] = mid
    cfg.update(run_config or {})
    if rank != 0:
        res = quantize_model(model, input_ids_list, **kw)
        if evaluate is not None:
            evaluate(model)
        return res
    with runlog.RunLog(save_path, cfg) as rl:
        res = quantize_model(model, input_ids_list, **kw)
        ppl = None
        if evaluate is not None:
            runlog.substep("Running final evaluation...")
            ppl = float(evaluate(model))
        rl.finish(res["layer_stats"], res["total_time"], ppl)
    return res
