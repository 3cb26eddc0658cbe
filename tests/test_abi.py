"""CPU: the C-ABI library loads and exports every entry point include/truncgptq.h
declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "truncgptq.h")
LIB = os.path.join(ROOT, "gptq-svd_amd", "libtruncgptq.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tg_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "gptq-svd_amd"), "-j8"], check=True)
    return ctypes.CDLL(LIB)


def test_header_declares_the_path():
    names = declared()
    for must in ("tg_syrk_accum", "tg_eigh_values", "tg_eigh_vectors", "tg_truncation_rank",
                 "tg_pivoted_factor", "tg_u_factor", "tg_group_params", "tg_process_block",
                 "tg_gptq_quantize", "tg_pack_codes", "tg_pack_zeros"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    import gptq_svd_amd._lib as L
    assert set(declared()) <= set(L._SIGS), set(declared()) - set(L._SIGS)
    assert set(declared()) <= set(L.EXPORTED)


def test_host_only_calls(lib):
    lib.tg_version.restype = ctypes.c_int
    assert lib.tg_version() >= 1
    lib.tg_quantize_workspace_size.restype = ctypes.c_size_t
    assert lib.tg_quantize_workspace_size(4096, 4096, 1024) > 4096 * 4096 * 9
    lib.tg_eigh_workspace_size.restype = ctypes.c_size_t
    assert lib.tg_eigh_workspace_size(256) > 256 * 256 * 8


def test_argument_errors_without_gpu(lib):
    """Invalid arguments are rejected before any device work (error codes
    follow the header's convention; the message names the argument)."""
    lib.tg_group_params.restype = ctypes.c_int
    rc = lib.tg_group_params(None, None, 4, 256, 256, 128, 4, 0, None, None)
    assert rc == -2
    lib.tg_last_error.restype = ctypes.c_char_p
    assert b"argument 2" in lib.tg_last_error()
    rc = lib.tg_group_params(None, ctypes.c_void_p(16), 4, 250, 250, 128, 4, 0,
                             ctypes.c_void_p(16), ctypes.c_void_p(16))
    assert rc == -6 and b"group" in lib.tg_last_error()


def test_no_cpu_fallback():
    """The product path refuses CPU tensors (no silent fallback)."""
    import torch
    import gptq_svd_amd.gptq_utils as g
    with pytest.raises(RuntimeError):
        g.HessianAccumulator(8, "cpu")
    q = g.Quantizer(4, 128, False)
    with pytest.raises(RuntimeError):
        q.find_params(torch.zeros(4, 128))
