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
