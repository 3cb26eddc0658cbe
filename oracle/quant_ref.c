/* CPU oracle for the TruncGPTQ quantize/propagate loop -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain C restatement of gptq_fwrd(use_triton=True)
 * (/root/reference/src/TruncGPTQ/gptq_utils.py:459-565) operating on
 * already-permuted W/S/Z (gptq_utils.py:493-495) and the float32 U:
 *
 *   block loop          gptq_utils.py:499-545
 *   intra-block kernel  gptq_utils.py:345-386  (Triton-interpreter semantics:
 *                       IEEE f32 division, multiply then subtract, no FMA)
 *   cross-block update  gptq_utils.py:537-545  (reduction order defined as the
 *                       k-ordered fmaf chain from +0; the HIP MFMA kernel
 *                       computes exactly this chain)
 *   truncated tail RTN  gptq_utils.py:547-553  (half-to-even rounding)
 *
 * GPTQ-comparator loop (use_triton=False, gptq_utils.py:516-534, :544):
 * qref_gptq_fwrd_loop -- round-half-even, err = (w - qv) / U[c][c],
 * w_j -= err * U[c][j] (raw row), cross-block Err @ U[i1:i2, i2:] (same
 * fmaf-chain definition).
 *
 * Compiled with -ffp-contract=off so the compiler never fuses mul+sub.
 * Used by tests/ and by bench.py's cpu_baseline leg only.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline float clampf(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

/* One block of `bw` columns for rows [r0, r1): W (ld = n) is updated in place
 * inside the block only (the kernel never writes W back, but the values are
 * dead after the block except through E). */
static void block_rows_loop(int r, int n, int c0, int bw, float *Wp, const float *S,
                            const float *Z, const float *U, int ldu, float minq, float maxq,
                            float *Q, float *E, int32_t *codes) {
  float *w = Wp + (size_t)r * n + c0;
  const float *s = S + (size_t)r * n + c0;
  const float *z = Z + (size_t)r * n + c0;
  float *e = E + (size_t)r * bw;
  for (int c = 0; c < bw; ++c) {
    float wc = w[c];
    float t = wc / s[c];
    t = t + z[c];
    float q = clampf(nearbyintf(t), minq, maxq);   /* torch.round: half-to-even */
    float qv = (q - z[c]) * s[c];
    const float *urow = U + (size_t)(c0 + c) * ldu + c0;
    float err = (wc - qv) / urow[c];
    Q[(size_t)r * n + c0 + c] = qv;
    codes[(size_t)r * n + c0 + c] = (int32_t)q;
    e[c] = err;
    for (int j = c + 1; j < bw; ++j) {
      float d = err * urow[j];
      w[j] = w[j] - d;
    }
  }
}

static void block_rows(int r0, int r1, int n, int c0, int bw, float *Wp, const float *S,
                       const float *Z, const float *U, int ldu, float minq, float maxq,
                       float *Q, float *E /* (m, bw) */, int32_t *codes, float *inv_diag) {
  for (int r = r0; r < r1; ++r) {
    float *w = Wp + (size_t)r * n + c0;
    const float *s = S + (size_t)r * n + c0;
    const float *z = Z + (size_t)r * n + c0;
    float *e = E + (size_t)r * bw;
    for (int c = 0; c < bw; ++c) {
      float wc = w[c];
      float t = wc / s[c];
      t = t + z[c];
      t = t + 0.5f;
      float q = clampf(floorf(t), minq, maxq);
      float qv = (q - z[c]) * s[c];
      float err = wc - qv;
      Q[(size_t)r * n + c0 + c] = qv;
      codes[(size_t)r * n + c0 + c] = (int32_t)q;
      e[c] = err;
      const float *urow = U + (size_t)(c0 + c) * ldu + c0;
      float inv = inv_diag[c];
      for (int j = c + 1; j < bw; ++j) {
        float corr = urow[j] * inv;
        float d = err * corr;
        w[j] = w[j] - d;
      }
    }
  }
}

/* One block of the loop (gptq_utils.py:345-386) for all m rows, OpenMP over
 * rows: W block (ld n, in place), Q/codes (ld n), E (m x bw). */
int qref_block(int m, int n, int c0, int bw, float *Wp, const float *S, const float *Z,
               const float *U, int ldu, int minq_i, int maxq_i, float *Q, int32_t *codes, float *E,
               int nthreads) {
  float *inv_diag = (float *)malloc(sizeof(float) * (size_t)bw);
  if (!inv_diag) return -2;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  for (int c = 0; c < bw; ++c) inv_diag[c] = 1.0f / U[(size_t)(c0 + c) * ldu + c0 + c];
#pragma omp parallel for schedule(static)
  for (int r = 0; r < m; ++r)
    block_rows(r, r + 1, n, c0, bw, Wp, S, Z, U, ldu, (float)minq_i, (float)maxq_i, Q, E, codes,
               inv_diag);
  free(inv_diag);
  return 0;
}

static int gptq_fwrd_impl(int loop, int m, int n, int k, int block, float *Wp, const float *S,
                          const float *Z, const float *U, int ldu, int minq_i, int maxq_i,
                          float *Q, int32_t *codes, int nthreads) {
  if (m <= 0 || n <= 0 || k <= 0 || k > n || block <= 0) return -1;
  const float minq = (float)minq_i, maxq = (float)maxq_i;
  float *E = (float *)malloc(sizeof(float) * (size_t)m * (size_t)block);
  float *inv_diag = (float *)malloc(sizeof(float) * (size_t)block);
  float *smat = (float *)malloc(sizeof(float) * (size_t)block * (size_t)n);
  if (!E || !inv_diag || !smat) { free(E); free(inv_diag); free(smat); return -2; }
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  for (int i1 = 0; i1 < k; i1 += block) {
    int i2 = i1 + block < k ? i1 + block : k;
    int bw = i2 - i1;
    for (int c = 0; c < bw; ++c) inv_diag[c] = 1.0f / U[(size_t)(i1 + c) * ldu + i1 + c];
#pragma omp parallel for schedule(static)
    for (int r = 0; r < m; ++r) {
      if (loop) block_rows_loop(r, n, i1, bw, Wp, S, Z, U, ldu, minq, maxq, Q, E, codes);
      else block_rows(r, r + 1, n, i1, bw, Wp, S, Z, U, ldu, minq, maxq, Q, E, codes, inv_diag);
    }
    if (i2 < n) {
      int nc = n - i2;
      /* Scale_mat = U[i1:i2, i2:] / diag[:, None]  (true f32 division);
       * loop mode: the raw rows U[i1:i2, i2:] (:544) */
      for (int c = 0; c < bw; ++c) {
        float d = U[(size_t)(i1 + c) * ldu + i1 + c];
        for (int j = 0; j < nc; ++j)
          smat[(size_t)c * nc + j] = loop ? U[(size_t)(i1 + c) * ldu + i2 + j]
                                          : U[(size_t)(i1 + c) * ldu + i2 + j] / d;
      }
#pragma omp parallel for schedule(static)
      for (int r = 0; r < m; ++r) {
        const float *e = E + (size_t)r * bw;
        float *w = Wp + (size_t)r * n + i2;
        for (int j = 0; j < nc; ++j) {
          float acc = 0.0f;
          for (int c = 0; c < bw; ++c) acc = fmaf(e[c], smat[(size_t)c * nc + j], acc);
          w[j] = w[j] - acc;
        }
      }
    }
  }
  /* truncated tail: plain RTN with half-to-even (torch.round) */
  if (k < n) {
#pragma omp parallel for schedule(static)
    for (int r = 0; r < m; ++r)
      for (int c = k; c < n; ++c) {
        size_t o = (size_t)r * n + c;
        float t = Wp[o] / S[o];
        t = t + Z[o];
        float q = clampf(nearbyintf(t), minq, maxq);
        Q[o] = (q - Z[o]) * S[o];
        codes[o] = (int32_t)q;
      }
  }
  free(E); free(inv_diag); free(smat);
  return 0;
}

int qref_gptq_fwrd(int m, int n, int k, int block, float *Wp, const float *S, const float *Z,
                   const float *U, int ldu, int minq_i, int maxq_i, float *Q, int32_t *codes,
                   int nthreads) {
  return gptq_fwrd_impl(0, m, n, k, block, Wp, S, Z, U, ldu, minq_i, maxq_i, Q, codes, nthreads);
}

int qref_gptq_fwrd_loop(int m, int n, int k, int block, float *Wp, const float *S,
                        const float *Z, const float *U, int ldu, int minq_i, int maxq_i,
                        float *Q, int32_t *codes, int nthreads) {
  return gptq_fwrd_impl(1, m, n, k, block, Wp, S, Z, U, ldu, minq_i, maxq_i, Q, codes, nthreads);
}
