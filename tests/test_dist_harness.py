"""CPU multi-process (gloo, world_size 2) coverage of the harness's multi-GPU
mode (harness.py module docstring): calibration sequences sharded over the
ranks, each group's H all-reduced (FP64 sums + counts), rows of every linear
quantised by their owning rank and all-gathered.

The solver calls are replaced by the CPU oracle (tests only: the HIP library
needs a GPU), so this checks the distributed plumbing: against the
single-process run with the same stand-ins every H agrees to FP64 rounding
(only the order of the additions differs), every rank ends with the same
weights bit for bit, and the weights equal the single-process ones.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def tiny_opt(seed):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(vocab_size=256, hidden_size=64, ffn_dim=256, num_hidden_layers=2,
                    num_attention_heads=4, max_position_embeddings=64, word_embed_proj_dim=64,
                    do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    return OPTForCausalLM(cfg).float().eval()


def tiny_decoder(kind, seed):
    """Tiny random Llama / Qwen3 (the harness's staged layer path)."""
    import transformers as tf
    cls = {"llama": (tf.LlamaConfig, tf.LlamaForCausalLM),
           "qwen3": (tf.Qwen3Config, tf.Qwen3ForCausalLM)}[kind]
    cfg = cls[0](vocab_size=256, hidden_size=64, intermediate_size=192, num_hidden_layers=2,
                 num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64,
                 head_dim=16)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    return cls[1](cfg).float().eval()


def tiny_model(kind, seed):
    return tiny_opt(seed) if kind == "opt" else tiny_decoder(kind, seed)


def _patch(harness, hs):
    """CPU stand-ins for the HIP solver calls; `hs` collects every group's H."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as o

    class CpuAcc:
        def __init__(self, n, device=None):
            self.H = torch.zeros((n, n), dtype=torch.float64)
            self.n_samples = 0

        def add_batch(self, x):
            x = x.reshape(-1, x.shape[-1]).double()
            self.H += x.T @ x
            self.n_samples += x.shape[0]

        def get_hessian(self):
            H = self.H / self.n_samples
            hs.append(H.clone())
            return H

    def solve(H, threshold=1e-4, threshold_method="energy"):
        f = o.process_hessian_alt(H.numpy(), threshold, threshold_method)
        return (torch.from_numpy(np.ascontiguousarray(f.U)),
                torch.from_numpy(np.ascontiguousarray(f.R_x)), torch.from_numpy(f.perm))

    def fwrd(W, R, q, perm, block_size=1024, use_triton=True, R_x=None):
        Wn = W.float().numpy()
        Wq, k, codes = o.gptq_fwrd(Wn, R.numpy(), perm.numpy(), q.w_bits, q.group_size, q.sym,
                                   block_size, gemm="fma", impl="c", return_codes=True)
        s, z = o.find_params(Wn, q.w_bits, q.group_size, q.sym)
        q.codes = torch.from_numpy(codes)
        q.scale = torch.from_numpy(np.asarray(s, np.float32)).reshape(W.shape[0], -1, 1)
        q.zero = torch.from_numpy(np.asarray(z, np.float32)).reshape(W.shape[0], -1, 1)
        return torch.from_numpy(Wq), k

    harness.HessianAccumulator = CpuAcc
    harness.process_hessian_alt = solve
    harness.gptq_fwrd = fwrd
    harness.log_quantization_error = lambda *a, **k: None


def _run(ids, kind="opt"):
    import gptq_svd_amd.harness as harness
    hs = []
    _patch(harness, hs)
    model = tiny_model(kind, 5)
    res = harness.quantize_model(model, ids, mode="eigh", w_bits=4, group_size=64, sym=False,
                                 eps=1e-3, threshold_method="energy", batch_size=2, device="cpu")
    W = {n: p.detach().clone().numpy() for n, p in model.named_parameters()
         if n.endswith("weight") and "layers" in n and p.dim() == 2}
    return hs, res, W


def _worker(rank, world, port, ids, out, kind):
    torch.set_num_threads(1)
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs, res, W = _run(ids, kind)
        out[rank] = dict(H=[h.numpy() for h in hs], W=W,
                         ranks=[s["rank"] for s in res["layer_stats"]])
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["opt", "llama"])
def test_token_sharded_harness_matches_single(kind):
    """OPT runs the generic per-group layer passes, Llama the staged ones."""
    torch.set_num_threads(2)
    gen = torch.Generator().manual_seed(9)
    ids = [torch.randint(0, 256, (1, 16), generator=gen) for _ in range(6)]
    hs1, res1, W1 = _run(ids, kind)
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_worker, args=(2, _free_port(), ids, out, kind), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert len(r0["H"]) == len(hs1) == 8  # 2 layers x 4 groups
    for a, b, c in zip(r0["H"], r1["H"], hs1):
        assert np.array_equal(a, b)  # every rank factorises the same H
        c = c.numpy()
        assert np.abs(a - c).max() <= 1e-12 * np.abs(c).max()
    assert r0["ranks"] == r1["ranks"] == [s["rank"] for s in res1["layer_stats"]]
    assert W1.keys() == r0["W"].keys() == r1["W"].keys()
    for name in W1:
        assert np.array_equal(r0["W"][name], r1["W"][name]), name
        assert np.array_equal(r0["W"][name], W1[name]), name


def test_early_stop_matches_full_layer_passes():
    """A calibration pass that stops at the group's first linear (forward
    pre-hook, harness.quantize_model(early_stop=True)) accumulates the same
    H, hence the same weights, as running the whole layer (the reference,
    quantize.py:139-148, discards the output)."""
    import gptq_svd_amd.harness as harness
    gen = torch.Generator().manual_seed(4)
    ids = [torch.randint(0, 256, (1, 16), generator=gen) for _ in range(5)]
    out = []
    for early in (True, False):
        hs = []
        _patch(harness, hs)
        model = tiny_opt(5)
        harness.quantize_model(model, ids, mode="eigh", w_bits=4, group_size=64, sym=False,
                               eps=1e-3, threshold_method="energy", batch_size=2, device="cpu",
                               early_stop=early)
        out.append((hs, {n: p.detach().clone() for n, p in model.named_parameters()}))
    (h1, w1), (h2, w2) = out
    assert len(h1) == len(h2) == 8
    for a, b in zip(h1, h2):
        assert torch.equal(a, b)
    for n in w1:
        assert torch.equal(w1[n], w2[n]), n


@pytest.mark.parametrize("kind", ["llama", "qwen3"])
def test_staged_layers_match_generic(kind, monkeypatch):
    """harness.quantize_model(staged=True) -- each group's calibration pass
    starts from the previous group's cached activations -- accumulates the
    same H, and produces the same weights and next-layer inputs, bit for bit,
    as re-running every layer from its input per group (staged=False).  Five
    sequences in batches of 2: a short last batch included."""
    import gptq_svd_amd.harness as harness
    for name in ("HessianAccumulator", "process_hessian_alt", "gptq_fwrd",
                 "log_quantization_error"):
        monkeypatch.setattr(harness, name, getattr(harness, name))
    torch.set_num_threads(2)
    gen = torch.Generator().manual_seed(6)
    ids = [torch.randint(0, 256, (1, 16), generator=gen) for _ in range(5)]
    assert harness._staged_layer(harness.get_layers(tiny_model(kind, 0))[0])
    out = []
    for staged in (True, False):
        hs = []
        _patch(harness, hs)
        model = tiny_model(kind, 5)
        res = harness.quantize_model(model, ids, mode="eigh", w_bits=4, group_size=32,
                                     sym=False, eps=1e-3, threshold_method="energy",
                                     batch_size=2, device="cpu", staged=staged)
        with torch.no_grad():
            logits = model(torch.cat(ids)).logits
        out.append((hs, {n: p.detach().clone() for n, p in model.named_parameters()}, logits,
                    [s["rank"] for s in res["layer_stats"]]))
    (h1, w1, l1, r1), (h2, w2, l2, r2) = out
    assert len(h1) == len(h2) == 8 and r1 == r2
    for a, b in zip(h1, h2):
        assert torch.equal(a, b)
    for n in w1:
        assert torch.equal(w1[n], w2[n]), n
    assert torch.equal(l1, l2)


def test_staged_layer_eligibility():
    import gptq_svd_amd.harness as harness
    assert not harness._staged_layer(harness.get_layers(tiny_opt(0))[0])
    layer = harness.get_layers(tiny_decoder("llama", 0))[0]
    assert harness._staged_layer(layer)
    h = layer.mlp.register_forward_hook(lambda *a: None)
    assert not harness._staged_layer(layer)  # a user hook would be skipped
    h.remove()


def _factor_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from gptq_svd_amd.harness import check_factor_agrees, quantize_model
        R = torch.arange(12, dtype=torch.float64).reshape(3, 4)
        perm = torch.tensor([2, 0, 3, 1])
        check_factor_agrees(R, perm)  # identical on both ranks: passes
        res = {}
        R2 = R.clone()
        if rank == 1:
            R2[1, 2] += 1e-13  # one rank's factor differs in the last bits
        try:
            check_factor_agrees(R2, perm)
            res["mismatch"] = "no error"
        except RuntimeError as e:
            res["mismatch"] = "RuntimeError" if "disagree" in str(e) else str(e)
        # identical non-finite factors: reported as non-finite, not as a disagreement
        R3 = R.clone()
        R3[0, 0] = float("nan")
        try:
            check_factor_agrees(R3, perm)
            res["nan"] = "no error"
        except RuntimeError as e:
            res["nan"] = "not finite" if "not finite" in str(e) else str(e)
        # fewer calibration sequences than ranks: every rank raises before a collective
        try:
            quantize_model(torch.nn.Linear(2, 2), [torch.zeros(1, 4, dtype=torch.long)],
                           device="cpu")
            res["few"] = "no error"
        except ValueError as e:
            res["few"] = "ValueError" if "fewer calibration sequences" in str(e) else str(e)
        out[rank] = res
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_factor_agreement_and_short_calibration_raise_on_every_rank():
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_factor_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in (0, 1):
        assert out[r]["mismatch"] == "RuntimeError", out[r]
        assert out[r]["nan"] == "not finite", out[r]
        assert out[r]["few"] == "ValueError", out[r]


def test_allreduce_hessian_single_process_is_noop():
    from gptq_svd_amd.harness import allreduce_hessian

    class A:
        H = torch.ones(3, 3, dtype=torch.float64)
        n_samples = 4
    a = A()
    allreduce_hessian(a)
    assert a.n_samples == 4 and float(a.H.sum()) == 9.0


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
