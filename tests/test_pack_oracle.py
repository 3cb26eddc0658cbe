"""CPU: packing format (A13) -- AutoGPTQ bit-stream layout round trips."""
import numpy as np
import pytest


@pytest.mark.parametrize("bits", [2, 3, 4, 8])
def test_pack_roundtrip(oracle_mod, bits):
    rng = np.random.default_rng(bits)
    n, m = 256, 64
    codes = rng.integers(0, 2 ** bits, size=(m, n))
    qw = oracle_mod.pack_rows_bitstream(codes.T.astype(np.uint64), bits)
    assert qw.shape == (n * bits // 32, m) and qw.dtype == np.int32
    back = oracle_mod.unpack_rows_bitstream(qw, bits, n)
    assert np.array_equal(back.T, codes)


def test_3bit_layout_is_autogptq(oracle_mod):
    """32 values in 3 words: value 10 straddles words 0/1, value 21 words 1/2."""
    vals = np.arange(32, dtype=np.uint64) % 8
    qw = oracle_mod.pack_rows_bitstream(vals[:, None], 3).view(np.uint32)[:, 0].astype(np.int64)
    w0, w1, w2 = qw
    for i in range(10):
        assert (w0 >> (3 * i)) & 7 == vals[i]
    assert ((w0 >> 30) & 3) | ((w1 & 1) << 2) == vals[10]
    for i in range(10):
        assert (w1 >> (3 * i + 1)) & 7 == vals[11 + i]
    assert ((w1 >> 31) & 1) | ((w2 & 3) << 1) == vals[21]
    for i in range(10):
        assert (w2 >> (3 * i + 2)) & 7 == vals[22 + i]


def test_export_files_cpu(tmp_path, oracle_mod):
    """save_quantized / read_quantized on oracle-packed tensors (host side
    only: no GPU needed to write or read a checkpoint)."""
    import torch
    from gptq_svd_amd.export import read_quantized, save_quantized
    lin = torch.nn.Linear(256, 64, bias=True)
    model = torch.nn.Sequential()
    model.add_module("proj", lin)
    rng = np.random.default_rng(0)
    codes = rng.integers(0, 16, size=(64, 256))
    scale = rng.random((64, 2)).astype(np.float32) + 0.1
    zero = rng.integers(0, 16, size=(64, 2)).astype(np.float32)
    qw, qz, sc = oracle_mod.pack_weights(codes, scale, zero, 4, False)
    packed = {"proj": dict(qweight=torch.from_numpy(qw), qzeros=torch.from_numpy(qz),
                           scales=torch.from_numpy(sc))}
    save_quantized(str(tmp_path), model, packed, 4, 128, False, extra_config={"eps": 1e-4})
    t, qc = read_quantized(str(tmp_path))
    assert set(t) == {"proj.qweight", "proj.qzeros", "proj.scales", "proj.g_idx", "proj.bias"}
    assert t["proj.scales"].dtype == torch.float16 and t["proj.g_idx"].dtype == torch.int32
    assert np.array_equal(oracle_mod.unpack_rows_bitstream(t["proj.qweight"].numpy(), 4, 256).T,
                          codes)
    assert qc["group_size"] == 128 and qc["static_groups"] and qc["truncgptq"]["eps"] == 1e-4
