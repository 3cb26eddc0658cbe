/* truncgptq.h -- C ABI of the MI355X-native TruncGPTQ per-layer solver.
 *
 * Every entry point takes plain device pointers, explicit sizes / leading
 * dimensions (row-major, element units) and the caller's hipStream_t
 * (passed as void* so this header needs no HIP include).  Work is
 * stream-ordered; nothing here synchronises the device unless the comment
 * says so.  Scratch memory comes from the caller (`ws`, `ws_bytes`), sized
 * by the matching *_workspace_size() query; the library allocates nothing.
 *
 * Return value: 0 ok; <0 invalid argument (-(1-based argument index));
 * >0 a hipError_t.  tg_last_error() returns a thread-local message.
 *
 * Reference = /root/reference/src/TruncGPTQ (davidtweedle/gptq-svd).
 */
#ifndef TRUNCGPTQ_H
#define TRUNCGPTQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- misc --------------------------------------------------------------- */
const char *tg_last_error(void);
int tg_version(void);

/* Sampled HIP-event timing of the hot kernel classes (for bench roofline
 * reporting).  Classes: 0 tri_symv, 1 cross_gemm, 2 quant_block, 3 tri_syr2k,
 * 4 pivot_step, 5 bisect, 6 inverse_iteration, 7 back_transform, 8 bulge_chase,
 * 9 tsqr_leaf (the panel QR kernels), 10 band_update, 11 q1_apply, 12 q2_apply
 * (the order of PROF_CLASSES in gptq-svd_amd/_lib.py).
 * tg_profile_query synchronises on the recorded events. */
int tg_profile_enable(int on, int every);
int tg_profile_reset(void);
int tg_profile_query(int id, double *ms, int64_t *sampled, double *bytes, double *flops,
                     int64_t *total_launches);

enum tg_dtype { TG_F16 = 0, TG_BF16 = 1, TG_F32 = 2, TG_F64 = 3 };
enum tg_rank_rule { TG_RULE_NONE = 0, TG_RULE_ENERGY = 1, TG_RULE_MEAN_TRIMMED = 2 };

/* ---- A1: Hessian accumulation -------------------------------------------
 * Replaces HessianAccumulator.add_batch: `self.H.addmm_(x.T, x)` after the
 * cast to float64 (gptq_utils.py:218-223).  H (n x n, ld ldh) += X^T X where
 * X is (rows x n, ld ldx) of dtype x_dtype (products formed in float64).
 * Both triangles of H are written (the reference keeps the full matrix). */
int tg_syrk_accum(void *stream, const void *X, int x_dtype, int64_t rows, int n, int64_t ldx,
                  double *H, int ldh);

/* The same update with a caller workspace (tg_syrk_workspace_size(n) bytes,
 * independent of rows: the partial tiles of the last round of 128 x 128 tiles,
 * Tt = min(tiles, resident workgroups) tiles x 16 chunks x 128 KiB, i.e. about
 * 1 GiB on a 256-CU MI355X once n >= ~4000): fp16 / bf16 X with n and ldx
 * multiples of 8 and a 16-byte aligned X take the dedicated 16-bit SYRK
 * (syrk.hip: X kept 16-bit in LDS, lower 128 x 128 tiles handed out by an
 * atomic queue over a static decomposition whose partial tiles are summed in
 * a fixed order -- deterministic); other inputs fall back to tg_syrk_accum. */
size_t tg_syrk_workspace_size(int n);
int tg_syrk_accum_ws(void *stream, const void *X, int x_dtype, int64_t rows, int n, int64_t ldx,
                     double *H, int ldh, void *ws, size_t ws_bytes);

/* Replaces HessianAccumulator.get_hessian `self.H / self.n_samples`
 * (gptq_utils.py:225-228).  inv_n > 0: out = H * inv_n; inv_n < 0:
 * out = H / (-inv_n) (exact true division, the reference's semantics).
 * out may alias H. */
int tg_scale_f64(void *stream, const double *H, int64_t count, double inv_n, double *out);

/* FP64 MFMA GEMM used by every dense stage (exported for tests / reuse):
 * C = alpha op(A) op(B) + beta C, row-major, op(A) M x K, op(B) K x N.
 * Hand-written kernels only (gemm64.hip: 8-wave 128 x 128 tiles for large
 * products, 64 x 64 tiles otherwise); no vendor BLAS is linked. */
int tg_dgemm(void *stream, int transA, int transB, int M, int N, int K, double alpha,
             const double *A, int lda, const double *B, int ldb, double beta, double *C, int ldc);

/* ---- A2: symmetric eigensolver (torch.linalg.eigh, gptq_utils.py:93) ----
 * Stage 1: A (n x n symmetric, full storage, destroyed) -> tridiagonal
 * (Householder, lower) + all eigenvalues ascending in w_asc (n).  The
 * reflectors stay in ws for stage 2. */
size_t tg_eigh_workspace_size(int n);
int tg_eigh_values(void *stream, double *A, int n, int lda, double *w_asc, void *ws,
                   size_t ws_bytes);
/* Stage 2: eigenvectors of the `k` LARGEST eigenvalues, in DESCENDING order,
 * written as ROWS of Vh (k x n, ld ldv) -- i.e. the reference's
 * `V.T.flip(0)[:k]` (gptq_utils.py:95,110).  Uses the stage-1 workspace. */
int tg_eigh_vectors(void *stream, int n, const double *w_asc, int k, double *Vh, int ldv,
                    void *ws, size_t ws_bytes);
/* Eigenvectors of the eigenvalues first .. first+count-1 in DESCENDING
 * order (rows of Vh, count x n).  tg_eigh_vectors(k) = range(0, k).  The
 * complement path below asks for the dropped eigenpairs k .. k+nc-1. */
int tg_eigh_vectors_range(void *stream, int n, const double *w_asc, int first, int count,
                          double *Vh, int ldv, void *ws, size_t ws_bytes);
/* The band -> tridiagonal stage of tg_eigh_values on its own (tests, tools):
 * A (n x n, full storage, ld lda) holds a symmetric band matrix of
 * half-bandwidth 32 (only the lower band A[c + d][c], d <= 32, is read);
 * on return d (n) / e (n - 1 used) hold a similar symmetric tridiagonal.
 * Bulge chasing as in tg_eigh_values (part of the eigh of
 * gptq_utils.py:93).  Synchronises the stream (reads the stall word);
 * a stalled hand-off returns hipErrorLaunchTimeOut. */
size_t tg_band_tridiag_workspace_size(int n);
int tg_band_tridiag(void *stream, const double *A, int n, int lda, double *d, double *e, void *ws,
                    size_t ws_bytes);

/* ---- A3: truncation rank (gptq_utils.py:97-108) ---------------------------
 * From ascending eigenvalues: S = sqrt(max(L, 1e-12)) descending, then the
 * rank rule.  Writes S_desc (n) and k (int32, device) -- no host sync. */
int tg_truncation_rank(void *stream, const double *w_asc, int n, double threshold, int rule,
                       double *S_desc, int32_t *k_dev);

/* ---- A4: pivot order + R_x (jax.scipy.linalg.qr(pivoting=True) on
 * S_k = diag(S) Vh_k, gptq_utils.py:112-117, 122-123) -----------------------
 * Computes the dgeqp3 column order `perm` (n, int64) and the sign-normalised
 * R_x (k x n upper trapezoidal, ld ldr; may be NULL).  Algorithm: greedy
 * diagonal pivoting on H_k = S_k^T S_k (identical pivot rule to dgeqp3; see
 * DESIGN.md). */
size_t tg_pivot_workspace_size(int n, int k);
int tg_pivoted_factor(void *stream, const double *Vh, int ldv, const double *S, int n, int k,
                      int64_t *perm, double *Rx, int ldr, void *ws, size_t ws_bytes);

/* ---- A5: U = sign-normalised R of QR(diag(1/S) Vh_k[:, perm])
 * (gptq_utils.py:111, 118-124).  U (k x n, ld ldu) upper trapezoidal with
 * positive diagonal; U^T U = P^T H_k^+ P. */
size_t tg_ufactor_workspace_size(int n, int k);
int tg_u_factor(void *stream, const double *Vh, int ldv, const double *S, const int64_t *perm,
                int n, int k, double *U, int ldu, void *ws, size_t ws_bytes);

/* ---- A4/A5 complement path (same outputs, no kept eigenvectors) ----------
 * When the dropped eigenpairs above rounding level are fewer than the kept
 * ones (k > n/2, the usual case: Qwen3-8B keeps ~99.5%), H_k = H - B_c^T B_c
 * with B_c = diag(S_c) Vc (Vc: nc x n rows = eigenvectors k .. k+nc-1 in
 * descending order from tg_eigh_vectors_range, S_c = S_desc[k:k+nc]); the
 * pivot order and R_x come from the same greedy pivoting as
 * tg_pivoted_factor (workspace: tg_pivot_workspace_size(n, k)), and U from
 * R_x alone: U = R(QR(S^-1 R_x)), S = R_x R_x^T. */
int tg_pivoted_factor_complement(void *stream, const double *H, int ldh, const double *Vc,
                                 int ldvc, const double *Sc, int nc, int n, int k, int64_t *perm,
                                 double *Rx, int ldr, void *ws, size_t ws_bytes);
size_t tg_ufactor_rx_workspace_size(int n, int k);
int tg_u_factor_rx(void *stream, const double *Rx, int ldr, int n, int k, double *U, int ldu,
                   void *ws, size_t ws_bytes);

/* The same U factor (explicit form: m = n - k > k / 16) in column-sharded
 * pieces for one process per GPU (gptq_svd_amd.dist.u_factor_rx_sharded; no
 * reference counterpart: the reference is single-device, quantize.py:180-184).
 * C = R11^-1 R12 (R11 = Rx[:, :k], R12 = Rx[:, k:]):
 *   tg_urx_c:   C[:, c0:c1] into C (k x (c1 - c0), ld ldc);
 *   tg_urx_u11: U[:, :k] = V^-1 from the whole C (k x (n - k), ld ldc);
 *   tg_urx_u12: out (k x ncols, ld ldo) = U[:, :k] C_block.
 * Each entry of C and U12 depends on its own column only, so gathering the
 * ranks' blocks gives tg_u_factor_rx's U bit for bit.  Workspace:
 * tg_ufactor_rx_workspace_size(n, k) for tg_urx_c / tg_urx_u11. */
int tg_urx_c(void *stream, const double *Rx, int ldr, int n, int k, int c0, int c1, double *C,
             int ldc, void *ws, size_t ws_bytes);
int tg_urx_u11(void *stream, const double *Rx, int ldr, int n, int k, const double *C, int ldc,
               double *U, int ldu, void *ws, size_t ws_bytes);
int tg_urx_u12(void *stream, const double *U, int ldu, int k, const double *C, int ldc, int ncols,
               double *out, int ldo);

/* ---- A6: relative prediction error (log_quantization_error,
 * gptq_utils.py:275-291) ---------------------------------------------------
 * out[0] = ||W[:, perm] R^T||_F^2, out[1] = ||(W - Wq)[:, perm] R^T||_F^2
 * (device, 2 doubles) with R = R_x (k x n, ld ldr) rounded to float32, the
 * reference's `R_x.to(float32)`.  W, Wq: m x n float32 (ld ldw), original
 * column order; perm: n int64.  The products are FP32 MFMA (TF32 off in the
 * reference), the sums of squares FP64; the caller takes sqrt(out[1] / out[0]). */
size_t tg_pred_error_workspace_size(int m, int n, int k);
int tg_pred_error(void *stream, const float *W, const float *Wq, int m, int n, int ldw,
                  const double *Rx, int k, int ldr, const int64_t *perm, double *out, void *ws,
                  size_t ws_bytes);

/* ---- A7: Quantizer.find_params (gptq_utils.py:249-266) --------------------
 * W (m x n f32, ld ldw) -> scale, zero (m x n/g f32, ld n/g); g = group or n. */
int tg_group_params(void *stream, const float *W, int m, int n, int ldw, int group, int w_bits,
                    int sym, float *scale, float *zero);

/* ---- A9: triton_process_block (gptq_utils.py:393-453, kernel :298-386) ----
 * One block: w, s, z (m x B f32, ld ldw/lds/ldz), R (B x B f32, ld ldr).
 * Outputs q (dequantised) and e (raw error), m x B, ld ldq / lde. */
size_t tg_process_block_workspace_size(int B);
int tg_process_block(void *stream, const float *w, int ldw, const float *s, int lds,
                     const float *z, int ldz, const float *R, int ldr, int m, int B, int minq,
                     int maxq, float *q, int ldq, float *e, int lde, void *ws, size_t ws_bytes);

/* ---- A8-A12: gptq_fwrd(use_triton=True) (gptq_utils.py:459-565) ---------
 * W (m x n f32, original column order), U (k x n f32, ld ldu), perm (n
 * int64), scale/zero from tg_group_params.  Writes Wq (m x n f32,
 * dequantised, original order) and codes (m x n uint8, original order,
 * stored +2^(b-1) when sym).  `block` is the reference's block_size. */
size_t tg_quantize_workspace_size(int m, int n, int block);
int tg_gptq_quantize(void *stream, const float *W, int m, int n, const float *U, int k, int ldu,
                     const int64_t *perm, const float *scale, const float *zero, int group,
                     int w_bits, int sym, int block, float *Wq, uint8_t *codes, void *ws,
                     size_t ws_bytes);

/* ---- §8(f) GPTQ comparator: gptq_fwrd(use_triton=False)
 * (gptq_utils.py:516-534 column loop, :544 cross-block GEMM) ---------------
 * Same arguments as tg_gptq_quantize; U is the comparator's H_inv_sqrt
 * (tg_hinv_chol).  Per column: q = clamp(round-half-even(w/s + z)),
 * err = (w - (q - z) s) / U[c, c], later block columns w_j -= err * U[c, j];
 * cross-block W[:, i2:] -= Err @ U[i1:i2, i2:] (k-ordered fmaf chain). */
int tg_gptq_quantize_loop(void *stream, const float *W, int m, int n, const float *U, int k,
                          int ldu, const int64_t *perm, const float *scale, const float *zero,
                          int group, int w_bits, int sym, int block, float *Wq, uint8_t *codes,
                          void *ws, size_t ws_bytes);

/* ---- §8(f) GPTQ comparator: process_hessian (gptq_utils.py:129-165) ------
 * R (n x n f64, ld ldr) = upper Cholesky factor of inv(H_p + damp I),
 * H_p = H[perm][:, perm] (perm may be NULL = identity; actorder's perm is
 * computed by the caller), damp = 10^e * damp_percent * mean(diag(H)) for
 * e = 0 .. max_tries-1 until H_p + damp I is positive definite (the
 * reference's ladder, :148-160).  *tries_used (host) = the rung e that
 * succeeded, or max_tries when every rung failed, in which case R = I (the
 * reference's intended fallback, :162-164).  Synchronises the stream once
 * per rung (the reference's try/except is a host round trip too). */
size_t tg_hinv_chol_workspace_size(int n);
int tg_hinv_chol(void *stream, const double *H, int n, int ldh, const int64_t *perm,
                 double damp_percent, int max_tries, double *R, int ldr, int *tries_used,
                 void *ws, size_t ws_bytes);

/* ---- A13: packing (absent in the reference; README.md:133) ----------------
 * codes (m x n uint8, offset form) -> qweight (n*b/32 x m int32, bit stream
 * along in_features; AutoGPTQ layout for b in {2,3,4,8}); zero (m x G f32)
 * -> qzeros (G x m*b/32 int32, stored zero + 2^(b-1) when sym). */
int tg_pack_codes(void *stream, const uint8_t *codes, int m, int n, int w_bits, int32_t *qweight);
int tg_pack_zeros(void *stream, const float *zero, int m, int G, int w_bits, int sym,
                  int32_t *qzeros);

#ifdef __cplusplus
}
#endif
#endif /* TRUNCGPTQ_H */
