// Internal FP64 MFMA GEMM (gemm64.hip), shared by the factorisation stages.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tg {
// C = alpha * op(A) op(B) + beta * C, row-major; op(A) is M x K, op(B) is K x N.
hipError_t dgemm(hipStream_t st, bool transA, bool transB, int M, int N, int K, double alpha,
                 const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                 double *C, int64_t ldc);
// Split-K variant for small M*N with long K; scratch >= dgemm_splitk_scratch(M, N, splits).
size_t dgemm_splitk_scratch(int M, int N, int splits);
hipError_t dgemm_splitk(hipStream_t st, bool transA, bool transB, int M, int N, int K,
                        double alpha, const double *A, int64_t lda, const double *B, int64_t ldb,
                        double beta, double *C, int64_t ldc, int splits, double *scratch);
// Symmetric rank-K updates (lower tiles computed, mirrored to the upper triangle).
hipError_t dsyrk_tn(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc);  // C = a X^T X + b C, X: K x n
hipError_t dsyrk_nt(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc);  // C = a X X^T + b C, X: n x K
}  // namespace tg
