"""ctypes binding of the HIP C-ABI library ``libtruncgptq.so`` (include/truncgptq.h).

There is no fallback: if the library is missing or fails to load, importing
this module raises, and every solver entry point of the package fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TRUNCGPTQ_LIB", os.path.join(_HERE, "libtruncgptq.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} not found: build the HIP library first "
        "(`make -C gptq-svd_amd` or `python -c 'import __graft_entry__ as g; g.build()'`)")

lib = ctypes.CDLL(LIB_PATH)

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t
_d = ctypes.c_double

_SIGS = {
    "tg_last_error": ([], ctypes.c_char_p),
    "tg_version": ([], _i),
    "tg_syrk_accum": ([_vp, _vp, _i, _i64, _i, _i64, _vp, _i], _i),
    "tg_syrk_workspace_size": ([_i], _sz),
    "tg_syrk_accum_ws": ([_vp, _vp, _i, _i64, _i, _i64, _vp, _i, _vp, _sz], _i),
    "tg_scale_f64": ([_vp, _vp, _i64, _d, _vp], _i),
    "tg_profile_enable": ([_i, _i], _i),
    "tg_profile_reset": ([], _i),
    "tg_profile_query": ([_i, ctypes.POINTER(_d), ctypes.POINTER(_i64), ctypes.POINTER(_d),
                          ctypes.POINTER(_d), ctypes.POINTER(_i64)], _i),
    "tg_dgemm": ([_vp, _i, _i, _i, _i, _i, _d, _vp, _i, _vp, _i, _d, _vp, _i], _i),
    "tg_eigh_workspace_size": ([_i], _sz),
    "tg_eigh_values": ([_vp, _vp, _i, _i, _vp, _vp, _sz], _i),
    "tg_eigh_vectors": ([_vp, _i, _vp, _i, _vp, _i, _vp, _sz], _i),
    "tg_eigh_vectors_range": ([_vp, _i, _vp, _i, _i, _vp, _i, _vp, _sz], _i),
    "tg_band_tridiag_workspace_size": ([_i], _sz),
    "tg_band_tridiag": ([_vp, _vp, _i, _i, _vp, _vp, _vp, _sz], _i),
    "tg_truncation_rank": ([_vp, _vp, _i, _d, _i, _vp, _vp], _i),
    "tg_pivot_workspace_size": ([_i, _i], _sz),
    "tg_pivoted_factor": ([_vp, _vp, _i, _vp, _i, _i, _vp, _vp, _i, _vp, _sz], _i),
    "tg_ufactor_workspace_size": ([_i, _i], _sz),
    "tg_u_factor": ([_vp, _vp, _i, _vp, _vp, _i, _i, _vp, _i, _vp, _sz], _i),
    "tg_pivoted_factor_complement": ([_vp, _vp, _i, _vp, _i, _vp, _i, _i, _i, _vp, _vp, _i, _vp,
                                      _sz], _i),
    "tg_ufactor_rx_workspace_size": ([_i, _i], _sz),
    "tg_u_factor_rx": ([_vp, _vp, _i, _i, _i, _vp, _i, _vp, _sz], _i),
    "tg_urx_c": ([_vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _sz], _i),
    "tg_urx_u11": ([_vp, _vp, _i, _i, _i, _vp, _i, _vp, _i, _vp, _sz], _i),
    "tg_urx_u12": ([_vp, _vp, _i, _i, _vp, _i, _i, _vp, _i], _i),
    "tg_group_params": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp], _i),
    "tg_process_block_workspace_size": ([_i], _sz),
    "tg_process_block": ([_vp, _vp, _i, _vp, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _i,
                          _vp, _i, _vp, _sz], _i),
    "tg_quantize_workspace_size": ([_i, _i, _i], _sz),
    "tg_gptq_quantize": ([_vp, _vp, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _vp,
                          _vp, _vp, _sz], _i),
    "tg_gptq_quantize_loop": ([_vp, _vp, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i,
                               _vp, _vp, _vp, _sz], _i),
    "tg_hinv_chol_workspace_size": ([_i], _sz),
    "tg_hinv_chol": ([_vp, _vp, _i, _i, _vp, _d, _i, _vp, _i, ctypes.POINTER(_i), _vp, _sz], _i),
    "tg_pred_error_workspace_size": ([_i, _i, _i], _sz),
    "tg_pred_error": ([_vp, _vp, _vp, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _sz], _i),
    "tg_pack_codes": ([_vp, _vp, _i, _i, _i, _vp], _i),
    "tg_pack_zeros": ([_vp, _vp, _i, _i, _i, _i, _vp], _i),
}

EXPORTED = []
for _name, (_args, _res) in _SIGS.items():
    _fn = getattr(lib, _name, None)
    if _fn is None:
        continue
    _fn.argtypes = _args
    _fn.restype = _res
    EXPORTED.append(_name)

TG_F16, TG_BF16, TG_F32, TG_F64 = 0, 1, 2, 3
RULES = {"none": 0, "energy": 1, "mean_trimmed": 2}
DTYPES = {torch.float16: TG_F16, torch.bfloat16: TG_BF16, torch.float32: TG_F32,
          torch.float64: TG_F64}


PROF_CLASSES = ["tri_symv", "cross_gemm", "quant_block", "tri_syr2k", "pivot_step", "bisect",
                "inverse_iteration", "back_transform", "bulge_chase", "tsqr_leaf", "band_update",
                "q1_apply", "q2_apply"]


def profile_enable(on: bool = True, every: int = 1) -> None:
    lib.tg_profile_enable(int(on), int(every))


def profile_reset() -> None:
    lib.tg_profile_reset()


def profile_query() -> dict:
    """{class: dict(ms, sampled, launches, bytes, flops)} over sampled launches."""
    out = {}
    for i, name in enumerate(PROF_CLASSES):
        ms, b, f = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        s, tot = ctypes.c_int64(), ctypes.c_int64()
        lib.tg_profile_query(i, ctypes.byref(ms), ctypes.byref(s), ctypes.byref(b), ctypes.byref(f),
                             ctypes.byref(tot))
        out[name] = dict(ms=ms.value, sampled=s.value, launches=tot.value, bytes=b.value,
                         flops=f.value)
    return out


def last_error() -> str:
    return lib.tg_last_error().decode(errors="replace")


def call(name: str, *args) -> None:
    """Invoke a C-ABI entry point; raise RuntimeError (the reference's error
    type for linalg failures, gptq_utils.py:159) on a non-zero status."""
    fn = getattr(lib, name, None)
    if fn is None:
        raise RuntimeError(f"{name} is not exported by {LIB_PATH}")
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {last_error()}")


def ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def workspace(nbytes: int, device) -> torch.Tensor:
    """Caller-owned scratch from the PyTorch caching allocator."""
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what} must be a GPU tensor (the MI355X path has no CPU fallback)")
