"""The harness's multi-GPU mode on the HIP path: two ranks (gloo, both on
cuda:0 -- the test box has one GPU; RCCL needs a GPU per rank) quantise a
tiny random OPT with the calibration sequences sharded between them.
Every rank must end with the same weights bit for bit, and those must match
the single-process run (same model, same sequences): the H differ only in
the order of the FP64 additions.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_opt(seed):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(vocab_size=256, hidden_size=128, ffn_dim=512, num_hidden_layers=2,
                    num_attention_heads=4, max_position_embeddings=64, word_embed_proj_dim=128,
                    do_layer_norm_before=True, dropout=0.0, attention_dropout=0.0)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    return OPTForCausalLM(cfg).float().eval()


def _quantize(ids):
    from gptq_svd_amd.harness import quantize_model
    model = _tiny_opt(21).to(DEV)
    res = quantize_model(model, ids, mode="eigh", w_bits=4, group_size=128, sym=False, eps=1e-4,
                         threshold_method="energy", batch_size=2, device=DEV, pack=True)
    W = {n: p.detach().float().cpu().numpy() for n, p in model.named_parameters()
         if n.endswith("weight") and "layers" in n and p.dim() == 2}
    return res, W


def _worker(rank, world, port, ids, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res, W = _quantize(ids)
        out[rank] = dict(W=W, ranks=[s["rank"] for s in res["layer_stats"]],
                         packed=sorted(res["packed"]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_token_sharded_harness_on_gpu():
    gen = torch.Generator().manual_seed(22)
    ids = [torch.randint(0, 256, (1, 32), generator=gen) for _ in range(6)]
    res1, W1 = _quantize(ids)
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_worker, args=(2, _free_port(), ids, out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0["ranks"] == r1["ranks"]
    assert r0["packed"] == r1["packed"] == sorted(res1["packed"])
    worst = 0.0
    for name in W1:
        assert np.array_equal(r0["W"][name], r1["W"][name]), name
        worst = max(worst, float(np.mean(r0["W"][name] != W1[name])))
    print(f"2-rank vs 1-rank: ranks {r0['ranks']} vs {[s['rank'] for s in res1['layer_stats']]}, "
          f"worst weight mismatch {worst:.2e}")
    assert r0["ranks"] == [s["rank"] for s in res1["layer_stats"]]
    assert worst <= 1e-3
