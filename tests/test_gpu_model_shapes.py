"""BASELINE's model-level configs at their real layer shapes on one MI355X
(the harness counterpart of quantize.py:101-260 on one decoder layer):

  configs[2]  Llama-3-8B,  4-bit asym g128: hidden 4096, intermediate 14,336
  configs[3]  Qwen3-8B,    3-bit sym  g128: hidden 4096, intermediate 12,288
  configs[4]  Llama-3-70B, 4-bit asym g128: hidden 8192, intermediate 28,672

No weights exist in this image: random-init models with the exact config
dimensions (bench.random_causal_lm), 16 random 2048-token sequences (32,768
calibration rows, so every H up to n = 28,672 is full rank), eps 1e-4 energy.
What is checked, per quantised linear:
  * the rank is in range (0 < k <= n) and the group's linears share it;
  * every written-back weight lies on its quantisation grid: decoding the
    packed AutoGPTQ tensors ((code - zero) * scale, f32) and rounding to the
    model's fp16 gives the weight bit for bit (packed round trip exact);
  * codes are within [0, 2^b) after the storage offset.
PPL parity (configs[3]) needs the real weights and WikiText-2, absent here.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def unpack_rows(words: torch.Tensor, bits: int, R: int) -> torch.Tensor:
    """Inverse of the little-endian b-bit bit stream along axis 0 (oracle
    pack_rows_bitstream), on the device: (R*b/32, C) int32 -> (R, C) int64."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    i = torch.arange(R, device=words.device)
    wi, sh = (i * bits) // 32, (i * bits) % 32
    lo = w[wi] >> sh[:, None]
    nxt = w[torch.clamp(wi + 1, max=w.shape[0] - 1)]
    hi = torch.where((sh + bits > 32)[:, None], nxt << (32 - sh)[:, None], torch.zeros_like(lo))
    return (lo | hi) & ((1 << bits) - 1)


@pytest.mark.parametrize("shape,bits,sym", [("llama3_8b", 4, False), ("qwen3_8b", 3, True),
                                            ("llama3_70b", 4, False)])
def test_one_layer_at_model_shape(shape, bits, sym):
    import bench
    from gptq_svd_amd import harness
    torch.cuda.empty_cache()
    model, gen = bench.random_causal_lm(shape, 1, DEV, seed=11)
    ids = torch.randint(0, model.config.vocab_size, (16, 2048), generator=gen, device=DEV).cpu()
    res = harness.quantize_model(model, [ids[i:i + 1] for i in range(16)], mode="eigh",
                                 w_bits=bits, group_size=128, sym=sym, eps=1e-4,
                                 threshold_method="energy", batch_size=8, device=DEV, pack=True)
    cfg = model.config
    h, f = cfg.hidden_size, cfg.intermediate_size
    kv = cfg.num_key_value_heads * (h // cfg.num_attention_heads)
    want = {"self_attn.q_proj": (h, h), "self_attn.k_proj": (kv, h), "self_attn.v_proj": (kv, h),
            "self_attn.o_proj": (h, h), "mlp.gate_proj": (f, h), "mlp.up_proj": (f, h),
            "mlp.down_proj": (h, f)}
    stats = {s["name"].split(".", 1)[1]: s["rank"] for s in res["layer_stats"]}
    assert set(stats) == set(want)
    print(f"{shape} {bits}-bit {'sym' if sym else 'asym'}: ranks {stats}")
    for nm, (m, n) in want.items():
        assert 0 < stats[nm] <= n, (nm, stats[nm])
    assert stats["self_attn.q_proj"] == stats["self_attn.k_proj"] == stats["self_attn.v_proj"]
    assert stats["mlp.gate_proj"] == stats["mlp.up_proj"]
    sd = model.state_dict()
    assert len(res["packed"]) == 7
    for nm, (m, n) in want.items():
        key = f"model.layers.0.{nm}"
        t = res["packed"][key]
        W = sd[key + ".weight"]
        assert W.shape == (m, n) and W.dtype == torch.float16
        codes = unpack_rows(t["qweight"], bits, n).T                  # (m, n)
        zeros = unpack_rows(t["qzeros"].T.contiguous(), bits, m)      # (m, G)
        assert int(codes.min()) >= 0 and int(codes.max()) < 2 ** bits
        gi = torch.arange(n, device=DEV) // 128
        deq = (codes.float() - zeros[:, gi].float()) * t["scales"].T[:, gi]
        bad = int((deq.half() != W).sum())
        assert bad == 0, f"{key}: {bad} of {W.numel()} weights off the quantisation grid"
        del codes, zeros, deq
    del model, res, sd
    torch.cuda.empty_cache()
