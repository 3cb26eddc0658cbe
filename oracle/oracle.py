"""CPU oracle for the TruncGPTQ per-layer solver -- TEST INFRASTRUCTURE ONLY.

This module is a plain numpy/scipy restatement of the reference solver in
``/root/reference/src/TruncGPTQ/gptq_utils.py`` (cited per function below).
It exists to *check* the MI355X product path; it is never shipped as the
product.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product package
(``gptq-svd_amd/``) never imports anything under ``oracle/`` and fails loudly
when its HIP library is missing.

Parity pin: the functions here are checked against golden vectors produced by
running the reference's own code in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.

Floating-point conventions (they define "bit-exact" for the HIP kernels):

* the intra-block loop follows the Triton kernel ``gptq_block_kernel``
  (gptq_utils.py:345-386) under Triton-interpreter semantics (IEEE f32
  division, separate multiply and subtract, no FMA contraction);
* the cross-block update ``W[:, i2:] -= E @ (U_cross / diag)``
  (gptq_utils.py:537-545) has an implementation-defined reduction order in
  the reference (MKL/cuBLAS SGEMM).  ``gemm="fma"`` defines it as the
  k-ordered fmaf chain starting from +0 (what the HIP MFMA kernel computes);
  ``gemm="torch"`` uses torch's CPU SGEMM like the reference's CPU run.
* ``Quantizer.find_params`` divides by ``max_q`` with true IEEE division
  (torch CPU semantics, gptq_utils.py:260,265).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import scipy.linalg

F32 = np.float32


# --------------------------------------------------------------------------
# A1  Hessian accumulation   (gptq_utils.py:213-228)
# --------------------------------------------------------------------------
class HessianAccumulator:
    """H += x^T x in float64 over every batch; get_hessian() returns H / N."""

    def __init__(self, in_features: int):
        self.H = np.zeros((in_features, in_features), dtype=np.float64)
        self.n_samples = 0

    def add_batch(self, x: np.ndarray) -> None:      # gptq_utils.py:218-223
        if x.ndim == 3:
            x = x.reshape(-1, x.shape[-1])
        x = x.astype(np.float64)
        self.H += x.T @ x
        self.n_samples += x.shape[0]

    def get_hessian(self) -> np.ndarray:              # gptq_utils.py:225-228
        if self.n_samples == 0:
            return self.H
        return self.H / self.n_samples


# --------------------------------------------------------------------------
# A2-A5  truncated spectral factorisation   (gptq_utils.py:87-126)
# --------------------------------------------------------------------------
def truncation_rank(S: np.ndarray, threshold: float, method: str) -> int:
    """Rank rule of gptq_utils.py:97-108 on descending singular values S."""
    n = len(S)
    if method == "energy":
        energy = S ** 2
        target = (1.0 - threshold) * np.sum(energy)
        k = int(np.sum(np.cumsum(energy) <= target))
        if k < n:
            k += 1
        return k
    if method == "mean_trimmed":
        ref_k = min(33, n)
        ref_val = np.mean(S[1:ref_k]) if n > 1 else S[0]
        return int(np.sum(S > threshold * ref_val))
    return n


@dataclass
class SpectralFactor:
    U: np.ndarray      # k x n float64, upper trapezoidal, positive diagonal ("R")
    R_x: np.ndarray    # k x n float64, sign-normalised R factor of pQR(S_k)
    perm: np.ndarray   # n int64 pivot order
    S: np.ndarray      # n descending sqrt(clamped eigenvalues)
    k: int


def process_hessian_alt(H: np.ndarray, threshold: float = 0.0005,
                        threshold_method: str = "mean_trimmed") -> SpectralFactor:
    """Restates gptq_utils.py:87-126.

    eigh -> descending S = sqrt(max(L, 1e-12)), Vh = V^T flipped (:92-95);
    rank rule (:97-108); S_k = diag(S) Vh_k and LAPACK dgeqp3 on it (the
    reference uses JAX -> MAGMA dgeqp3, the same algorithm) (:109-117);
    U = R of QR(diag(1/S) Vh_k [:, perm]) (:118-120); diagonal sign
    normalisation of U and R_x (:121-124).
    """
    Hd = np.asarray(H, dtype=np.float64)
    L, V = np.linalg.eigh(Hd)
    S = np.sqrt(np.maximum(L, 1e-12))[::-1].copy()
    Vh = V.T[::-1].copy()
    k = truncation_rank(S, threshold, threshold_method)
    if k < 1:
        raise RuntimeError("truncation rank is 0")
    S_k = S[:k]
    Vh_k = Vh[:k]
    H_sqrt = S_k[:, None] * Vh_k
    _, R_x, p = scipy.linalg.qr(H_sqrt, pivoting=True, mode="economic")
    perm = p.astype(np.int64)
    H_inv_perm = ((1.0 / S_k)[:, None] * Vh_k)[:, perm]
    _, Rp = np.linalg.qr(H_inv_perm, mode="reduced")
    U = Rp * np.sign(np.diagonal(Rp))[:, None]
    R_x = R_x * np.sign(np.diagonal(R_x))[:, None]
    return SpectralFactor(U=U, R_x=R_x, perm=perm, S=S, k=k)


# --------------------------------------------------------------------------
# A7  static-group quantizer   (gptq_utils.py:230-272)
# --------------------------------------------------------------------------
def qrange(w_bits: int, sym: bool) -> tuple[int, int]:
    """(min_q, max_q) as gptq_utils.py:239-245."""
    if sym:
        h = 2 ** (w_bits - 1) - 1
        return -h, h
    return 0, 2 ** w_bits - 1


def find_params(W: np.ndarray, w_bits: int, group_size: int, sym: bool):
    """Per-(row, group) scale/zero on the original-order W (gptq_utils.py:249-266).

    Returns scale, zero of shape (m, n // g) float32.
    """
    W = np.asarray(W, dtype=F32)
    m, n = W.shape
    g = group_size if group_size > 0 else n
    assert n % g == 0
    _, maxq = qrange(w_bits, sym)
    w = W.reshape(m, n // g, g)
    if sym:
        amax = np.max(np.abs(w), axis=2)
        amax = np.maximum(amax, F32(1e-5))
        scale = (amax / F32(maxq)).astype(F32)
        zero = np.zeros_like(scale)
    else:
        mn = np.min(w, axis=2)
        mx = np.max(w, axis=2)
        scale = (np.maximum(mx - mn, F32(1e-5)) / F32(maxq)).astype(F32)
        zero = np.clip(np.rint(-mn / scale), F32(0), F32(maxq)).astype(F32)
    return scale, zero


def expand_params(scale, zero, n: int, group_size: int):
    """repeat_interleave over the group (gptq_utils.py:268-272) -> (m, n)."""
    g = group_size if group_size > 0 else n
    return np.repeat(scale, g, axis=1)[:, :n], np.repeat(zero, g, axis=1)[:, :n]


# --------------------------------------------------------------------------
# A9  intra-block quantize + propagate   (gptq_utils.py:298-386, :393-453)
# --------------------------------------------------------------------------
def process_block(w, s, z, R, min_q: int, max_q: int):
    """Triton-interpreter semantics of gptq_block_kernel.

    For each column c: q = clamp(floor(w/s + z + 0.5)); qv = (q - z) s;
    e = w - qv; corr = R[c, :] * (1/R[c, c]); w[:, j>c] -= e * corr.
    The pow2 padding of triton_process_block (:404-420) never feeds a real
    column (padded columns come last), so it is omitted.
    """
    w = np.array(w, dtype=F32, copy=True)
    s = np.asarray(s, dtype=F32)
    z = np.asarray(z, dtype=F32)
    R = np.asarray(R, dtype=F32)
    m, B = w.shape
    q = np.empty_like(w)
    e = np.empty_like(w)
    lo, hi = F32(min_q), F32(max_q)
    for c in range(B):
        wc = w[:, c]
        qi = np.clip(np.floor(wc / s[:, c] + z[:, c] + F32(0.5)), lo, hi)
        qv = (qi - z[:, c]) * s[:, c]
        err = wc - qv
        q[:, c] = qv
        e[:, c] = err
        inv = F32(1.0) / R[c, c]
        corr = R[c, c + 1:] * inv
        w[:, c + 1:] = w[:, c + 1:] - err[:, None] * corr[None, :]
    return q, e


def process_block_loop(w, s, z, Hinv1, min_q: int, max_q: int):
    """The GPTQ-comparator column loop (use_triton=False, gptq_utils.py:516-534).

    For each column i: q = clamp(round_half_even(w/s + z)); qv = (q - z) s;
    err = (w - qv) / Hinv1[i, i]; w[:, i:] -= err * Hinv1[i, i:] (the K=1
    matmul is one rounded product per element).  Returns (Q, Err).
    """
    w = np.array(w, dtype=F32, copy=True)
    s = np.asarray(s, dtype=F32)
    z = np.asarray(z, dtype=F32)
    Hb = np.asarray(Hinv1, dtype=F32)
    m, B = w.shape
    q = np.empty_like(w)
    e = np.empty_like(w)
    lo, hi = F32(min_q), F32(max_q)
    for c in range(B):
        wc = w[:, c].copy()
        qi = np.clip(np.rint(wc / s[:, c] + z[:, c]), lo, hi)
        qv = (qi - z[:, c]) * s[:, c]
        err = (wc - qv) / Hb[c, c]
        q[:, c] = qv
        e[:, c] = err
        w[:, c:] = w[:, c:] - err[:, None] * Hb[c, c:][None, :]
    return q, e


# --------------------------------------------------------------------------
# §8(f) GPTQ comparator factor   (gptq_utils.py:129-165)
# --------------------------------------------------------------------------
def process_hessian(H: np.ndarray, actorder: bool = False, damp_percent: float = 0.01):
    """Restates process_hessian: damped Cholesky ladder, then
    chol_upper(cholesky_inverse(L)) -- LAPACK potrf / potri / potrf, the
    routines torch's CPU path calls.  Returns (H_inv_chol, perm, rung) with
    rung = the damping exponent used (5 = identity fallback, the reference's
    intent; as written it raises NameError there, :147 vs :162)."""
    import scipy.linalg
    Hd = np.asarray(H, dtype=np.float64)
    n = Hd.shape[0]
    if actorder:
        perm = np.argsort(-np.diag(Hd), kind="stable")
        Hd = Hd[perm][:, perm]
    else:
        perm = np.arange(n)
    mean_diag = float(np.mean(np.diag(Hd)))
    if mean_diag == 0:
        mean_diag = 1.0
    for e in range(5):
        damp = 10 ** e * damp_percent
        Hdmp = Hd.copy()
        Hdmp[np.diag_indices(n)] += damp * mean_diag
        try:
            L = np.linalg.cholesky(Hdmp)
            Linv = scipy.linalg.solve_triangular(L, np.eye(n), lower=True)
            Hinv = Linv.T @ Linv
            R = np.linalg.cholesky(Hinv).T
        except np.linalg.LinAlgError:
            continue
        return R, perm, e
    return np.eye(n), perm, 5


# --------------------------------------------------------------------------
# optional C kernel for the exact loop (fast; oracle/quant_ref.c)
# --------------------------------------------------------------------------
_CLIB = None


def _clib():
    global _CLIB
    if _CLIB is None:
        here = os.path.dirname(os.path.abspath(__file__))
        path = os.path.join(here, "_build", "libquant_ref.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        fp = ctypes.POINTER(ctypes.c_float)
        lib.qref_gptq_fwrd.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,  # m n k block
            fp, fp, fp, fp,                                         # Wp S Z U (permuted, f32)
            ctypes.c_int, ctypes.c_int, ctypes.c_int,               # ldu minq maxq
            fp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]       # Q codes nthreads
        lib.qref_gptq_fwrd.restype = ctypes.c_int
        lib.qref_gptq_fwrd_loop.argtypes = lib.qref_gptq_fwrd.argtypes
        lib.qref_gptq_fwrd_loop.restype = ctypes.c_int
        lib.qref_block.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp, fp, fp, fp, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, fp, ctypes.POINTER(ctypes.c_int32), fp, ctypes.c_int]
        lib.qref_block.restype = ctypes.c_int
        _CLIB = lib
    return _CLIB


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def gptq_fwrd(W, U, perm, w_bits=4, group_size=128, sym=False, block_size=1024,
              gemm: str = "fma", impl: str = "numpy", return_codes: bool = False,
              nthreads: int = 1, use_triton: bool = True):
    """Restates gptq_fwrd(use_triton=True) (gptq_utils.py:459-565).

    W (m, n) any float; U (k, n) float64/float32 (cast to f32 like :483);
    perm (n,) int.  Returns (final_W float32 in original column order, k)
    and optionally integer codes (int32, original order, un-offset).
    gemm: "fma" = k-ordered fmaf chain from +0 (HIP kernel definition),
          "torch" = torch CPU SGEMM (the reference's CPU run),
          "numpy" = numpy SGEMM.
    impl: "numpy" (vectorised restatement) or "c" (oracle/quant_ref.c; gemm must be "fma").
    use_triton=False: the GPTQ-comparator loop (:516-534) and the raw cross
    rows (:544) instead of the block kernel and the diagonal-scaled rows.
    """
    W = np.asarray(W, dtype=F32)
    m, n = W.shape
    U32 = np.asarray(U, dtype=F32)
    k = U32.shape[0]
    perm = np.asarray(perm, dtype=np.int64)
    min_q, max_q = qrange(w_bits, sym)
    scale, zero = find_params(W, w_bits, group_size, sym)
    S_full, Z_full = expand_params(scale, zero, n, group_size)
    Wp = np.ascontiguousarray(W[:, perm])
    S = np.ascontiguousarray(S_full[:, perm])
    Z = np.ascontiguousarray(Z_full[:, perm])
    Q = np.zeros_like(Wp)
    codes = np.zeros((m, n), dtype=np.int32)

    if impl == "c" and gemm == "torch":
        assert use_triton, "the torch-SGEMM CPU baseline restates the TruncGPTQ path only"
        # exact C block loop + torch (MKL) SGEMM for the cross-block update: the
        # reference's own CPU semantics, fast enough for the bench CPU baseline
        import torch
        Uc = np.ascontiguousarray(U32)
        E = np.empty((m, block_size), dtype=F32)
        for i1 in range(0, k, block_size):
            i2 = min(i1 + block_size, k)
            bw = i2 - i1
            Eb = np.ascontiguousarray(E[:, :bw])
            rc = _clib().qref_block(m, n, i1, bw, _fp(Wp), _fp(S), _fp(Z), _fp(Uc), n, min_q,
                                    max_q, _fp(Q),
                                    codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    _fp(Eb), nthreads)
            if rc != 0:
                raise RuntimeError(f"qref_block failed ({rc})")
            if i2 < n:
                diag = np.diagonal(U32[i1:i2, i1:i2])
                scale_mat = np.ascontiguousarray(U32[i1:i2, i2:] / diag[:, None])
                delta = (torch.from_numpy(Eb) @ torch.from_numpy(scale_mat)).numpy()
                Wp[:, i2:] = Wp[:, i2:] - delta
        if k < n:
            qt = np.clip(np.rint(Wp[:, k:] / S[:, k:] + Z[:, k:]), F32(min_q), F32(max_q))
            Q[:, k:] = (qt - Z[:, k:]) * S[:, k:]
            codes[:, k:] = qt.astype(np.int32)
    elif impl == "c":
        assert gemm == "fma"
        Uc = np.ascontiguousarray(U32)
        fn = _clib().qref_gptq_fwrd if use_triton else _clib().qref_gptq_fwrd_loop
        rc = fn(m, n, k, block_size, _fp(Wp), _fp(S), _fp(Z), _fp(Uc),
                                    Uc.shape[1], min_q, max_q, _fp(Q),
                                    codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    nthreads)
        if rc != 0:
            raise RuntimeError(f"qref_gptq_fwrd failed ({rc})")
    else:
        for i1 in range(0, k, block_size):
            i2 = min(i1 + block_size, k)
            blk = process_block if use_triton else process_block_loop
            qb, eb = blk(Wp[:, i1:i2], S[:, i1:i2], Z[:, i1:i2], U32[i1:i2, i1:i2], min_q, max_q)
            Q[:, i1:i2] = qb
            if i2 < n:
                diag = np.diagonal(U32[i1:i2, i1:i2])
                if use_triton:
                    scale_mat = (U32[i1:i2, i2:] / diag[:, None]).astype(F32)
                else:
                    scale_mat = np.ascontiguousarray(U32[i1:i2, i2:])
                if gemm == "fma":
                    delta = fma_chain_matmul(eb, scale_mat)
                elif gemm == "torch":
                    import torch
                    delta = (torch.from_numpy(np.ascontiguousarray(eb))
                             @ torch.from_numpy(np.ascontiguousarray(scale_mat))).numpy()
                else:
                    delta = (eb @ scale_mat).astype(F32)
                Wp[:, i2:] = Wp[:, i2:] - delta
        if k < n:                                                   # gptq_utils.py:547-553
            qt = np.clip(np.rint(Wp[:, k:] / S[:, k:] + Z[:, k:]), F32(min_q), F32(max_q))
            Q[:, k:] = (qt - Z[:, k:]) * S[:, k:]
        # integer codes: exact because Q = (q - z) * s was formed from integral q
        codes_p = np.rint(Q / S + Z).astype(np.int32)
        codes = codes_p
        codes = codes[:, np.argsort(perm)]
    inv = np.argsort(perm)                                          # gptq_utils.py:556-557
    final = Q[:, inv]
    if impl == "c":
        codes = codes[:, inv]
    if return_codes:
        return final, k, codes
    return final, k


def fma_chain_matmul(A, B):
    """C[i, j] = fmaf chain over kk = 0..K-1 starting at +0 (exact definition).

    numpy has no fused multiply-add; emulate fmaf exactly in float64: the
    product of two floats is exact in double, and rounding (acc + p) once to
    float32 equals fmaf whenever the double sum is exact, which holds unless
    exponents differ by > 29 bits.  Used only for small test sizes; the C
    oracle (impl="c") is the reference definition for large sizes.
    """
    A = np.asarray(A, dtype=F32)
    B = np.asarray(B, dtype=F32)
    acc = np.zeros((A.shape[0], B.shape[1]), dtype=F32)
    for kk in range(A.shape[1]):
        p = A[:, kk:kk + 1].astype(np.float64) * B[kk:kk + 1, :].astype(np.float64)
        acc = (acc.astype(np.float64) + p).astype(F32)
    return acc


# --------------------------------------------------------------------------
# A6  relative prediction error   (gptq_utils.py:275-291)
# --------------------------------------------------------------------------
def relative_prediction_error(W_orig, W_quant, R_x, perm) -> float:
    R = np.asarray(R_x, dtype=F32)
    Wo = np.asarray(W_orig, dtype=F32)[:, perm]
    Wq = np.asarray(W_quant, dtype=F32)[:, perm]
    num = np.linalg.norm((Wo - Wq) @ R.T)
    den = np.linalg.norm(Wo @ R.T)
    return float(num / den)


# --------------------------------------------------------------------------
# A13  packing (absent in the reference, README.md:133; format defined here)
# --------------------------------------------------------------------------
def code_offset(w_bits: int, sym: bool) -> int:
    """Unsigned storage offset: sym codes [-maxq, maxq] are stored +2^(b-1)."""
    return 2 ** (w_bits - 1) if sym else 0


def pack_rows_bitstream(vals: np.ndarray, w_bits: int) -> np.ndarray:
    """Pack unsigned b-bit values along axis 0 into a little-endian bit stream
    of int32 words: value i of a column occupies bits [i*b, i*b+b).  For
    b in {2,4,8} this is AutoGPTQ's layout; for b=3 it is AutoGPTQ's
    32-values-in-3-words layout.  vals: (R, C) -> (R*b/32, C) int32."""
    vals = np.asarray(vals, dtype=np.uint64)
    R, C = vals.shape
    assert (R * w_bits) % 32 == 0
    out = np.zeros(((R * w_bits) // 32, C), dtype=np.uint64)
    for i in range(R):
        bit = i * w_bits
        wi, sh = divmod(bit, 32)
        out[wi] |= (vals[i] << np.uint64(sh)) & np.uint64(0xFFFFFFFF)
        if sh + w_bits > 32:
            out[wi + 1] |= vals[i] >> np.uint64(32 - sh)
    return out.astype(np.uint32).view(np.int32)


def pack_weights(codes: np.ndarray, scale: np.ndarray, zero: np.ndarray, w_bits: int, sym: bool):
    """codes (m, n) un-offset ints in original column order -> packed layout.

    qweight int32 (n*b/32, m) packs along in_features; qzeros int32
    (n/g, m*b/32) packs along out_features; scales float32 (n/g, m).
    Stored zero = zero + offset (so dequant = (code_u - zero_u) * scale).
    """
    off = code_offset(w_bits, sym)
    cu = (np.asarray(codes, dtype=np.int64) + off).astype(np.uint64)
    qweight = pack_rows_bitstream(cu.T, w_bits)
    zu = (np.rint(np.asarray(zero)).astype(np.int64) + off).astype(np.uint64)   # (m, G)
    qzeros = pack_rows_bitstream(zu, w_bits).T.copy()     # pack along m -> (G, m*b/32)
    scales = np.asarray(scale, dtype=F32).T.copy()        # (G, m)
    return qweight, qzeros, scales


def unpack_rows_bitstream(words: np.ndarray, w_bits: int, R: int) -> np.ndarray:
    w = np.asarray(words).view(np.uint32).astype(np.uint64)
    C = w.shape[1]
    out = np.zeros((R, C), dtype=np.int64)
    mask = np.uint64((1 << w_bits) - 1)
    for i in range(R):
        bit = i * w_bits
        wi, sh = divmod(bit, 32)
        v = w[wi] >> np.uint64(sh)
        if sh + w_bits > 32:
            v |= w[wi + 1] << np.uint64(32 - sh)
        out[i] = (v & mask).astype(np.int64)
    return out
