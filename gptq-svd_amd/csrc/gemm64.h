// Internal FP64 MFMA GEMM (gemm64.hip), shared by the factorisation stages.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tg {
// C = alpha * op(A) op(B) + beta * C, row-major; op(A) is M x K, op(B) is K x N.
// C = alpha A B + beta C, A (M x K) upper triangular row-major (zeros below
// the diagonal are not read); own FP64 MFMA kernel.
hipError_t dgemm_upper_a(hipStream_t st, int M, int N, int K, double alpha, const double *A,
                         int64_t lda, const double *B, int64_t ldb, double beta, double *C,
                         int64_t ldc);
hipError_t dgemm(hipStream_t st, bool transA, bool transB, int M, int N, int K, double alpha,
                 const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                 double *C, int64_t ldc);
// Split-K variant for small M*N with long K; scratch >= dgemm_splitk_scratch(M, N, splits).
size_t dgemm_splitk_scratch(int M, int N, int splits);
hipError_t dgemm_splitk(hipStream_t st, bool transA, bool transB, int M, int N, int K,
                        double alpha, const double *A, int64_t lda, const double *B, int64_t ldb,
                        double beta, double *C, int64_t ldc, int splits, double *scratch);
// C = alpha * sum_z P_z + beta * C, P_z = P + z * M * N (M x N, ld N).
hipError_t sum_partials(hipStream_t st, const double *P, int nz, int M, int N, double alpha,
                        double beta, double *C, int64_t ldc);
// Symmetric rank-K updates (lower tiles computed, mirrored to the upper triangle).
hipError_t dsyrk_tn(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc);  // C = a X^T X + b C, X: K x n
// C = a X^T X + b C for an upper-triangular X (n x n, strict lower triangle zero)
hipError_t dsyrk_tn_upper(hipStream_t st, int n, double alpha, const double *X, int64_t ldx,
                          double beta, double *C, int64_t ldc);
hipError_t dsyrk_tn_lower(hipStream_t st, int n, int K, double alpha, const double *X,
                          int64_t ldx, double beta, double *C,
                          int64_t ldc);  // lower tiles of C only, no mirror
hipError_t dsyrk_nt(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc);  // C = a X X^T + b C, X: n x K
// Chunked (grouped) GEMM over z = 0..nc-1.  Chunk z covers rows
// [kb, ke) of a length-m axis: kb = z*c, ke = (z == nc-1) ? m : kb + c.
// Per z:  C_z = alpha * op(A_z) op(B_z) + beta * C_z  with
//   X_z = X + kb * x_kb + z * x_z  (X in {A, B, C}),
//   M/N/K = fixed value, or (when < 0) the chunk length ke - kb.
struct ChunkSpec {
  int c, nc, m;
  int64_t a_kb, a_z, b_kb, b_z, c_kb, c_z;
  int M, N, K;
};
// tri = 1: every chunk's A is upper triangular, 2: every chunk's B (the
// zero triangle is skipped per tile; no transposes then).
hipError_t dgemm_chunked(hipStream_t st, bool transA, bool transB, const ChunkSpec &cs,
                         double alpha, const double *A, int64_t lda, const double *B,
                         int64_t ldb, double beta, double *C, int64_t ldc, int tri = 0);
}  // namespace tg
