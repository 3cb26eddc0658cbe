"""Drop-in counterpart of the reference solver API on MI355X.

Mirrors the names, argument meaning and error behaviour of
``/root/reference/src/TruncGPTQ/gptq_utils.py`` so the layer-sequential harness
(``quantize.py:14``) only has to change its import line:

    from gptq_svd_amd.gptq_utils import (gptq_fwrd, Quantizer, process_hessian_alt,
                                         HessianAccumulator)

Every numerical stage runs in the HIP library (``libtruncgptq.so``, C ABI in
``include/truncgptq.h``) on the caller's current HIP stream; torch provides
device memory, streams and the caching allocator only.  There is no CPU
fallback: CPU tensors raise ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import logging
from typing import NamedTuple, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream, workspace

__all__ = [
    "HessianAccumulator", "process_hessian_alt", "process_hessian", "Quantizer", "gptq_fwrd",
    "triton_process_block", "log_quantization_error", "next_power_of_2",
    "truncated_spectral_factor", "pack_quantized",
]


# ---------------------------------------------------------------------------
# A1  (gptq_utils.py:213-228)
# ---------------------------------------------------------------------------
class HessianAccumulator:
    """H += x^T x in float64 (FP64 MFMA SYRK kernel; fp16 / bf16 inputs take
    the dedicated 16-bit SYRK of syrk.hip); get_hessian() = H / N."""

    def __init__(self, in_features, device, dtype=torch.float64):
        if dtype != torch.float64:
            raise RuntimeError("HessianAccumulator: only float64 accumulation is supported")
        self.H = torch.zeros((in_features, in_features), device=device, dtype=dtype)
        _lib.require_cuda(self.H, "HessianAccumulator device")
        self.n_samples = 0
        self._ws = None

    def add_batch(self, x):                                   # gptq_utils.py:218-223
        if x.dim() == 3:
            x = x.reshape(-1, x.shape[-1])
        _lib.require_cuda(x, "add_batch input")
        if x.dtype not in _lib.DTYPES:
            x = x.to(torch.float64)
        if x.stride(-1) != 1:
            x = x.contiguous()
        rows, n = x.shape
        if n != self.H.shape[0]:
            raise RuntimeError(f"add_batch: expected {self.H.shape[0]} features, got {n}")
        if rows:
            with torch.cuda.device(self.H.device):
                # the 16-bit SYRK's partial-tile scratch, only for inputs that
                # take it (fp16 / bf16, n and the row stride multiples of 8,
                # 16-byte aligned); everything else runs the generic path
                b16 = (x.dtype in (torch.float16, torch.bfloat16) and n % 8 == 0
                       and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0)
                if b16 and self._ws is None:
                    self._ws = workspace(_lib.lib.tg_syrk_workspace_size(n), self.H.device)
                if b16:
                    call("tg_syrk_accum_ws", stream(), ptr(x), _lib.DTYPES[x.dtype], rows, n,
                         x.stride(0), ptr(self.H), self.H.shape[0], ptr(self._ws),
                         self._ws.numel())
                else:
                    call("tg_syrk_accum", stream(), ptr(x), _lib.DTYPES[x.dtype], rows, n,
                         x.stride(0), ptr(self.H), self.H.shape[0])
        self.n_samples += rows

    def get_hessian(self):                                    # gptq_utils.py:225-228
        if self.n_samples == 0:
            return self.H
        out = torch.empty_like(self.H)
        with torch.cuda.device(self.H.device):
            call("tg_scale_f64", stream(), ptr(self.H), self.H.numel(),
                 -float(self.n_samples), ptr(out))
        return out


# ---------------------------------------------------------------------------
# A2-A5  (gptq_utils.py:87-126)
# ---------------------------------------------------------------------------
class SpectrumSplit(NamedTuple):
    """What the complement path needs to know about the dropped spectrum."""
    nc: int          # dropped eigenvalues above the rounding threshold tau = n*eps*lambda_max
    lam_k: float     # smallest kept eigenvalue
    psd: bool        # every dropped eigenvalue >= -tau
    left: float      # max |lambda| of the dropped eigenvalues at or below tau


def _complement_count(w_asc, k: int) -> SpectrumSplit:
    """Split of the ascending spectrum at rank k (a device tensor: one 8n-byte
    copy; or a host numpy array).  numpy on the host copy: a handful of torch
    CPU ops cost ~0.3 ms of host time between two GPU phases."""
    w = w_asc.double().cpu().numpy() if isinstance(w_asc, torch.Tensor) else np.asarray(w_asc)
    n = w.shape[0]
    tau = n * 2.220446049250313e-16 * max(float(w[-1]), 0.0)
    dropped = w[:n - k]
    low = dropped[dropped <= tau]
    return SpectrumSplit(int(np.count_nonzero(dropped > tau)), float(w[n - k]),
                         bool(float(w[0]) >= -tau),
                         float(np.abs(low).max()) if low.size else 0.0)


def spectral_path(n: int, k: int, sp: SpectrumSplit) -> str:
    """'complement' when the dropped eigenpairs that matter are fewer than
    the kept ones (k > n/2 in practice) and the complement form is exact to
    ~1e-9: no kept eigenvalue is clamped by sqrt(max(L, 1e-12))
    (gptq_utils.py:94); no dropped eigenvalue is below -tau; and the dropped
    eigenvalues H_k = H - B_c^T B_c keeps (those at or below tau) are below
    1e-9 lambda_k, since they perturb the pseudo-inverse by ~left / lambda_k
    (graded spectra reaching down to rounding level fail this, the kept path
    is exact for them).  Else 'kept'.  TG_SPECTRAL_PATH = kept | complement
    forces one (complement only where it is defined)."""
    import os
    force = os.environ.get("TG_SPECTRAL_PATH", "auto")
    defined = sp.lam_k >= 1e-12 and sp.nc <= k and k + sp.nc <= n and sp.psd
    if force == "kept" or not defined:
        return "kept"
    if force == "complement":
        return "complement"
    exact = sp.left <= 1e-9 * sp.lam_k
    return "complement" if sp.nc < k and exact else "kept"


def truncated_spectral_factor(H: torch.Tensor, threshold: float = 0.0005,
                              threshold_method: str = "mean_trimmed", want_rx: bool = True):
    """Native pipeline behind process_hessian_alt.  Returns (U, R_x, perm, S, k).

    eigh (two-stage reduction + bisection) -> rank rule -> then either
      kept path:       eigenvectors of the k kept eigenvalues, greedy-pivoted
                       factor of H_k = S_k^T S_k (the dgeqp3 pivot order and
                       R_x), U = R(QR(diag(1/S_k) Vh_k P));
      complement path: eigenvectors of the nc dropped eigenvalues above the
                       rounding threshold only, H_k = H - B_c^T B_c, the same
                       pivoting, U = R(QR(S^-1 R_x)), S = R_x R_x^T
    whichever needs fewer eigenvectors.
    """
    _lib.require_cuda(H, "process_hessian_alt H")
    n = H.shape[0]
    if H.dim() != 2 or H.shape[1] != n:
        raise RuntimeError("process_hessian_alt: H must be square")
    dev = H.device
    rule = _lib.RULES.get(threshold_method, 0)
    with torch.cuda.device(dev):
        Hd = H.to(dtype=torch.float64).contiguous()
        A = Hd.clone()
        ws = workspace(_lib.lib.tg_eigh_workspace_size(n), dev)
        w = torch.empty(n, dtype=torch.float64, device=dev)
        call("tg_eigh_values", stream(), ptr(A), n, n, ptr(w), ptr(ws), ws.numel())
        S = torch.empty(n, dtype=torch.float64, device=dev)
        kdev = torch.empty(1, dtype=torch.int32, device=dev)
        call("tg_truncation_rank", stream(), ptr(w), n, float(threshold), rule, ptr(S), ptr(kdev))
        # one host sync for the rank and the spectrum split (the reference syncs
        # here too, gptq_utils.py:100, :106)
        wk = torch.cat((w, kdev.to(torch.float64))).cpu().numpy()
        k = int(wk[n])
        if k < 1:
            raise RuntimeError("process_hessian_alt: truncation rank is 0 "
                               "(threshold keeps no eigenvalue)")
        del A
        sp = _complement_count(wk[:n], k)
        nc = sp.nc
        path = spectral_path(n, k, sp)
        perm = torch.empty(n, dtype=torch.int64, device=dev)
        R_x = torch.empty((k, n), dtype=torch.float64, device=dev)
        U = torch.empty((k, n), dtype=torch.float64, device=dev)
        if path == "kept":
            Vh = torch.empty((k, n), dtype=torch.float64, device=dev)
            call("tg_eigh_vectors", stream(), n, ptr(w), k, ptr(Vh), n, ptr(ws), ws.numel())
            del ws
            pws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
            call("tg_pivoted_factor", stream(), ptr(Vh), n, ptr(S), n, k, ptr(perm), ptr(R_x),
                 n, ptr(pws), pws.numel())
            del pws
            uws = workspace(_lib.lib.tg_ufactor_workspace_size(n, k), dev)
            call("tg_u_factor", stream(), ptr(Vh), n, ptr(S), ptr(perm), n, k, ptr(U), n,
                 ptr(uws), uws.numel())
        else:
            Vc = torch.empty((max(nc, 1), n), dtype=torch.float64, device=dev)
            if nc:
                call("tg_eigh_vectors_range", stream(), n, ptr(w), k, nc, ptr(Vc), n, ptr(ws),
                     ws.numel())
            del ws
            pws = workspace(_lib.lib.tg_pivot_workspace_size(n, k), dev)
            call("tg_pivoted_factor_complement", stream(), ptr(Hd), n, ptr(Vc), n,
                 ptr(S[k:]) if nc else None, nc, n, k, ptr(perm), ptr(R_x), n, ptr(pws),
                 pws.numel())
            del pws, Vc
            uws = workspace(_lib.lib.tg_ufactor_rx_workspace_size(n, k), dev)
            call("tg_u_factor_rx", stream(), ptr(R_x), n, n, k, ptr(U), n, ptr(uws),
                 uws.numel())
        truncated_spectral_factor.last_path = (path, nc)
    return U, (R_x if want_rx else None), perm, S, k


def process_hessian_alt(H: torch.Tensor, threshold: float = 0.0005,
                        threshold_method: str = "mean_trimmed"
                        ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Returns (R, R_x, perm) exactly like gptq_utils.py:87-126:
    R = U (k x n float64, upper trapezoidal, positive diagonal),
    R_x (k x n float64), perm (n int64)."""
    U, R_x, perm, _, _ = truncated_spectral_factor(H, threshold, threshold_method)
    return U, R_x, perm


# ---------------------------------------------------------------------------
# §8(f) GPTQ comparator factor  (gptq_utils.py:129-165)
# ---------------------------------------------------------------------------
def process_hessian(H: torch.Tensor, actorder: bool = False,
                    damp_percent: float = 0.01) -> Tuple[torch.Tensor, torch.Tensor]:
    """(H_inv_chol, perm): upper Cholesky factor of inv(H_p + damp I) with the
    reference's damping ladder damp = 10^e * damp_percent * mean(diag H),
    e = 0..4 (:148-160).  ActOrder: perm = argsort(diag H, descending) (stable
    on ties; the reference's unstable CUDA sort leaves tie order unspecified).
    When every rung fails the factor is the identity -- the reference's
    intent at :162-164, which as written raises NameError (it tests
    `H_inv_chol` but initialises `H_inv_factor`, :147).
    """
    _lib.require_cuda(H, "process_hessian H")
    Hd = H.to(dtype=torch.float64).contiguous()
    n = Hd.shape[0]
    device = Hd.device
    if actorder:
        perm = torch.argsort(torch.diagonal(Hd), descending=True, stable=True)
    else:
        perm = torch.arange(n, device=device)
    R = torch.empty((n, n), dtype=torch.float64, device=device)
    tries = ctypes.c_int(0)
    max_tries = 5
    with torch.cuda.device(device):
        ws = workspace(_lib.lib.tg_hinv_chol_workspace_size(n), device)
        call("tg_hinv_chol", stream(), ptr(Hd), n, n, ptr(perm) if actorder else None,
             float(damp_percent), max_tries, ptr(R), n, ctypes.byref(tries), ptr(ws), ws.numel())
    if tries.value >= max_tries:
        logging.warning(" Hessian is singular. Using Identity fallback.")
    elif tries.value > 0:
        logging.info(f"  Ref-GPTQ required high damping: {10 ** tries.value * damp_percent}")
    return R, perm


# ---------------------------------------------------------------------------
# A7  (gptq_utils.py:230-272)
# ---------------------------------------------------------------------------
class Quantizer:
    """Static-group min/max (asym) or absmax (sym) quantizer; same fields and
    shapes as the reference (scale/zero: (m, n/g, 1) float32)."""

    def __init__(self, w_bits: int = 4, group_size: int = 128, sym: bool = False):
        self.w_bits = w_bits
        self.group_size = group_size
        self.sym = sym
        if self.sym:
            half_range = 2 ** (w_bits - 1) - 1
            self.max_q = half_range
            self.min_q = -half_range
        else:
            self.max_q = 2 ** w_bits - 1
            self.min_q = 0
        self.scale = None
        self.zero = None

    def find_params(self, weights: torch.Tensor):            # gptq_utils.py:249-266
        _lib.require_cuda(weights, "Quantizer.find_params weights")
        m, n = weights.shape
        g = self.group_size if self.group_size > 0 else n
        assert n % g == 0
        W = weights.to(torch.float32).contiguous()
        G = n // g
        scale = torch.empty((m, G), dtype=torch.float32, device=W.device)
        zero = torch.empty((m, G), dtype=torch.float32, device=W.device)
        with torch.cuda.device(W.device):
            call("tg_group_params", stream(), ptr(W), m, n, n, self.group_size, self.w_bits,
                 int(self.sym), ptr(scale), ptr(zero))
        self.scale = scale.unsqueeze(-1)
        self.zero = zero.unsqueeze(-1)

    def get_expanded_params(self, m, n):                       # gptq_utils.py:268-272
        g = self.group_size if self.group_size > 0 else n
        s_expanded = torch.repeat_interleave(self.scale, g, dim=1)
        z_expanded = torch.repeat_interleave(self.zero, g, dim=1)
        return s_expanded[:, :n].squeeze(-1), z_expanded[:, :n].squeeze(-1)


# ---------------------------------------------------------------------------
# A6  (gptq_utils.py:275-291)
# ---------------------------------------------------------------------------
def log_quantization_error(W_orig, W_quant, R_x, perm):
    """||(W_o - W_q) R_x^T||_F / ||W_o R_x^T||_F with W_o = W_orig[:, perm],
    logged in the reference's format (extract_log.py:20 parses it).  Both
    products run in ONE fused FP32 MFMA pass (tg_pred_error: R_x is read as
    float64 and rounded to float32 like the reference's R_x.to(float32), the
    m x k products never leave the chip, their sums of squares are FP64).
    Returns the value (the reference returns None)."""
    if R_x is None or perm is None:
        return None
    _lib.require_cuda(W_orig, "log_quantization_error W_orig")
    dev = W_orig.device
    W = W_orig.to(torch.float32).contiguous()
    Wq = W_quant.to(device=dev, dtype=torch.float32).contiguous()
    R = R_x.to(device=dev, dtype=torch.float64).contiguous()
    p = perm.to(device=dev, dtype=torch.int64).contiguous()
    m, n = W.shape
    k = R.shape[0]
    if Wq.shape != W.shape or R.shape[1] != n or p.numel() != n:
        raise RuntimeError("log_quantization_error: shape mismatch")
    out = torch.empty(2, dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        ws = workspace(_lib.lib.tg_pred_error_workspace_size(m, n, k), dev)
        call("tg_pred_error", stream(), ptr(W), ptr(Wq), m, n, n, ptr(R), k, n, ptr(p), ptr(out),
             ptr(ws), ws.numel())
    y_orig_sq, y_diff_sq = out.tolist()  # the reference's .item() sync (:290)
    relative_error = (y_diff_sq ** 0.5) / (y_orig_sq ** 0.5)
    logging.info(f"   [Metric] Relative prediction error: {relative_error:.6f}")
    return relative_error


# ---------------------------------------------------------------------------
# A9  (gptq_utils.py:389-453)
# ---------------------------------------------------------------------------
def next_power_of_2(x: int) -> int:
    return 1 if x == 0 else 2 ** (x - 1).bit_length()


def triton_process_block(w_block, s_block, z_block, R_block, quantizer):
    """Quantize one block with in-block error propagation -> (q, e).
    The reference pads to a power of two (:404-420); padding never feeds a
    real column, so the HIP kernel works on the exact width."""
    for t, nm in ((w_block, "w_block"), (s_block, "s_block"), (z_block, "z_block"),
                  (R_block, "R_block")):
        _lib.require_cuda(t, nm)
    m, B = w_block.shape
    f = lambda t: t.to(torch.float32).contiguous()
    w, s, z, R = f(w_block), f(s_block), f(z_block), f(R_block)
    q = torch.empty_like(w)
    e = torch.empty_like(w)
    with torch.cuda.device(w.device):
        ws = workspace(_lib.lib.tg_process_block_workspace_size(B), w.device)
        call("tg_process_block", stream(), ptr(w), B, ptr(s), B, ptr(z), B, ptr(R), B, m, B,
             int(quantizer.min_q), int(quantizer.max_q), ptr(q), B, ptr(e), B, ptr(ws),
             ws.numel())
    return q, e


# ---------------------------------------------------------------------------
# A8-A12  (gptq_utils.py:459-565)
# ---------------------------------------------------------------------------
def gptq_fwrd(weight_mat: torch.Tensor, H_inv_sqrt: torch.Tensor, quantizer: Quantizer,
              perm: torch.Tensor, block_size: int = 128, use_triton: bool = True,
              R_x: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, int]:
    """Column-wise quantize + error propagation driven by U (= H_inv_sqrt).

    Returns (dequantised W in the original column order and dtype, rank).
    use_triton=True: the TruncGPTQ block kernel semantics (:345-386, :537-545);
    use_triton=False: the GPTQ-comparator column loop (:516-534, :544) --
    round-half-even, error divided by U[c, c], raw U rows for propagation.
    The integer codes of the last call are kept on ``quantizer.codes``
    (uint8, original order, +2^(b-1) offset when sym) for packing.
    """
    allow_tf32 = torch.backends.cuda.matmul.allow_tf32       # :474-475, restored :565
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        _lib.require_cuda(weight_mat, "gptq_fwrd weight_mat")
        out_features, in_features = weight_mat.shape
        device = weight_mat.device
        orig_dtype = weight_mat.dtype
        weight_mat = weight_mat.to(device=device, dtype=torch.float32).contiguous()
        U = H_inv_sqrt.to(device=device, dtype=torch.float32).contiguous()
        current_rank = U.shape[0]
        if current_rank < in_features:
            logging.info(f"   Rank percent used: {float(current_rank) / in_features:.2%}")
        quantizer.find_params(weight_mat)
        perm_d = perm.to(device=device, dtype=torch.int64).contiguous()
        scale = quantizer.scale.squeeze(-1).contiguous()
        zero = quantizer.zero.squeeze(-1).contiguous()
        Wq = torch.empty_like(weight_mat)
        codes = torch.empty((out_features, in_features), dtype=torch.uint8, device=device)
        with torch.cuda.device(device):
            ws = workspace(_lib.lib.tg_quantize_workspace_size(out_features, in_features,
                                                               block_size), device)
            call("tg_gptq_quantize" if use_triton else "tg_gptq_quantize_loop", stream(),
                 ptr(weight_mat), out_features, in_features,
                 ptr(U), current_rank, U.shape[1], ptr(perm_d), ptr(scale), ptr(zero),
                 quantizer.group_size, quantizer.w_bits, int(quantizer.sym), block_size,
                 ptr(Wq), ptr(codes), ptr(ws), ws.numel())
        quantizer.codes = codes
        if R_x is not None:
            log_quantization_error(weight_mat, Wq, R_x, perm_d)
        return Wq.to(dtype=orig_dtype), current_rank
    finally:
        torch.backends.cuda.matmul.allow_tf32 = allow_tf32


# ---------------------------------------------------------------------------
# A13  packing (new; the reference saves dequantised FP16 only, README.md:133)
# ---------------------------------------------------------------------------
def pack_quantized(quantizer: Quantizer, codes: Optional[torch.Tensor] = None):
    """AutoGPTQ-style tensors from the last gptq_fwrd: qweight int32
    (n*b/32, m), qzeros int32 (n/g, m*b/32), scales float32 (n/g, m).
    Static groups in original column order, so no g_idx is needed."""
    codes = quantizer.codes if codes is None else codes
    m, n = codes.shape
    b = quantizer.w_bits
    zero = quantizer.zero.squeeze(-1).contiguous()
    G = zero.shape[1]
    dev = codes.device
    qweight = torch.empty((n * b // 32, m), dtype=torch.int32, device=dev)
    qzeros = torch.empty((G, m * b // 32), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        call("tg_pack_codes", stream(), ptr(codes.contiguous()), m, n, b, ptr(qweight))
        call("tg_pack_zeros", stream(), ptr(zero), m, G, b, int(quantizer.sym), ptr(qzeros))
    scales = quantizer.scale.squeeze(-1).t().contiguous()
    return qweight, qzeros, scales
