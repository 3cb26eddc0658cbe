// FP64 MFMA GEMM for gfx950 (v_mfma_f64_16x16x4_f64) and the Hessian SYRK.
//
//   C = alpha * op(A) * op(B) + beta * C     (row-major everything)
//
// Used by: Hessian accumulation (A1, gptq_utils.py:222 `H.addmm_(x.T, x)`,
// SYRK mode: lower tiles only, mirrored), the tridiagonalisation's trailing
// rank-2k updates, the eigenvector back-transformation and the factor stages.
//
// Tile BM x BN per 256-thread workgroup, 4 waves as 2x2, each wave a
// (BM/2) x (BN/2) grid of 16x16 MFMA tiles; K staged through LDS in chunks of
// 16 (k-major images so fragment reads are 16 consecutive doubles).
// f64 MFMA C/D layout (differs from f32!): col = lane & 15,
// row = (lane >> 4) + 4 * reg  (MI355X guide §3).
#include <algorithm>
#include <cstdlib>
#include <unordered_map>

#include "../../include/truncgptq.h"
#include "common.h"
#include "gemm64.h"

namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ inline double to_f64(T v) { return double(v); }
template <>
__device__ inline double to_f64<__half>(__half v) { return double(__half2float(v)); }
template <>
__device__ inline double to_f64<__hip_bfloat16>(__hip_bfloat16 v) { return double(__bfloat162float(v)); }

constexpr int KC = 16;
constexpr int PAD = 16;  // row pitch = 32 banks mod 64: the two 16-lane row groups of a
                         // ds_read_b64 half-wave hit disjoint banks

// Staging of an op(X) tile into a k-major LDS image S[KC][W + PAD] covering
// rows r0..r0+W of op(X) (op(X) is R x K) and k0..k0+KC, split into a
// global->register load (issued one K-slab ahead) and a register->LDS store.
//  TRANS == false: X stored R x K (ld), element (r, k) at X[r*ld + k]
//  TRANS == true : X stored K x R (ld), element (r, k) at X[k*ld + r]
template <class T, int W, bool TRANS>
struct Stg {
  static constexpr int PER = W * KC / 256;  // elements per thread
  double v[PER];
  __device__ inline void load(const T *__restrict__ X, int64_t ld, int R, int K, int r0, int k0) {
    const int tid = threadIdx.x;
    if (!TRANS) {  // one row, PER consecutive k
      constexpr int TPR = KC / PER;
      const int r = tid / TPR, kb = (tid % TPR) * PER;
      const int gr = r0 + r;
      const int grc = min(gr, R - 1);
#pragma unroll
      for (int t = 0; t < PER; ++t) v[t] = to_f64(X[int64_t(grc) * ld + min(k0 + kb + t, K - 1)]);
#pragma unroll
      for (int t = 0; t < PER; ++t) v[t] = (gr < R && k0 + kb + t < K) ? v[t] : 0.0;
    } else {  // one k, PER rows strided by TPK (lanes of one k cover consecutive rows:
              // coalesced loads and conflict-free LDS stores)
      constexpr int TPK = W / PER;
      const int k = tid / TPK, rb = tid % TPK;
      const int gk = k0 + k;
      const int gkc = min(gk, K - 1);
#pragma unroll
      for (int t = 0; t < PER; ++t)
        v[t] = to_f64(X[int64_t(gkc) * ld + min(r0 + rb + t * TPK, R - 1)]);
#pragma unroll
      for (int t = 0; t < PER; ++t) v[t] = (gk < K && r0 + rb + t * TPK < R) ? v[t] : 0.0;
    }
  }
  __device__ inline void store(double (*S)[W + PAD]) const {
    const int tid = threadIdx.x;
    if (!TRANS) {
      constexpr int TPR = KC / PER;
      const int r = tid / TPR, kb = (tid % TPR) * PER;
#pragma unroll
      for (int t = 0; t < PER; ++t) S[kb + t][r] = v[t];
    } else {
      constexpr int TPK = W / PER;
      const int k = tid / TPK, rb = tid % TPK;
#pragma unroll
      for (int t = 0; t < PER; ++t) S[k][rb + t * TPK] = v[t];
    }
  }
};

// acc += op(A)[tm:tm+BM, kb:ke] op(B)[kb:ke, tn:tn+BN], 4 waves as 2x2.
// Double-buffered LDS, one barrier per K slab: slab s is read from buffer
// s & 1 while the registers holding slab s+1 go to the other buffer (last
// read in slab s-1, released by the previous barrier) and slab s+2's global
// loads are in flight.
template <class TA_, class TB_, int BM, int BN, bool TA, bool TB>
__device__ inline void mainloop(const TA_ *__restrict__ A, int64_t lda,
                                const TB_ *__restrict__ B, int64_t ldb, int M, int N, int kb,
                                int ke, int tm, int tn, double (*As)[KC][BM + PAD],
                                double (*Bs)[KC][BN + PAD],
                                doublex4 (&acc)[BM / 32][BN / 32]) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  Stg<TA_, BM, TA> sa;
  Stg<TB_, BN, !TB> sb;  // op(B) staged as op(B)^T (N x K)
  if (kb >= ke) return;
  sa.load(A, lda, M, ke, tm, kb);
  sb.load(B, ldb, N, ke, tn, kb);
  sa.store(As[0]);
  sb.store(Bs[0]);
  if (kb + KC < ke) {
    sa.load(A, lda, M, ke, tm, kb + KC);
    sb.load(B, ldb, N, ke, tn, kb + KC);
  }
  __syncthreads();
  int cur = 0;
  for (int k0 = kb; k0 < ke; k0 += KC) {
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      double af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = As[cur][kk + (lane >> 4)][wm * WM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = Bs[cur][kk + (lane >> 4)][wn * WN + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (k0 + KC < ke) {
      sa.store(As[cur ^ 1]);
      sb.store(Bs[cur ^ 1]);
      if (k0 + 2 * KC < ke) {
        sa.load(A, lda, M, ke, tm, k0 + 2 * KC);
        sb.load(B, ldb, N, ke, tn, k0 + 2 * KC);
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}

// C = alpha acc + beta C for the 4-wave tile, one 16-row fragment row at a
// time: its FN x 4 beta != 0 reads are issued together (clamped addresses)
// so they overlap, and at most FN x 4 of them are live -- the whole tile's
// worth (FM x FN x 4 doubles on top of the accumulators) set the kernel's
// register count to one wave per SIMD.
template <int BM, int BN, bool SYRK, bool MIRROR = true>
__device__ inline void epilogue(const doublex4 (&acc)[BM / 32][BN / 32], double alpha, double beta,
                                double *__restrict__ C, int64_t ldc, int M, int N, int tm,
                                int tn) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    double cv[FN][4];
    if (beta != 0.0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = min(tm + wm * WM + i * 16 + (lane >> 4) + 4 * r, M - 1);
          const int gj = min(tn + wn * WN + j * 16 + (lane & 15), N - 1);
          cv[j][r] = C[int64_t(gi) * ldc + gj];
        }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = tm + wm * WM + i * 16 + (lane >> 4) + 4 * r;
        const int gj = tn + wn * WN + j * 16 + (lane & 15);
        if (gi < M && gj < N) {
          const double v = beta == 0.0 ? alpha * acc[i][j][r] : alpha * acc[i][j][r] + beta * cv[j][r];
          C[int64_t(gi) * ldc + gj] = v;
          if (SYRK && MIRROR && tm != tn) C[int64_t(gj) * ldc + gi] = v;
        }
      }
  }
}

// 128 x 128 tiles: two workgroups per CU (LDS 2 x 74 KB) need <= 256
// registers per lane (128 accumulators + the loop's operands and staging)
// UPA: op(A) = A is upper triangular (row-major, A[i][c] = 0 for c < i), so
// the tile of rows tm.. only needs K from tm (rounded down to the slab).
template <class TA_, class TB_, int BM, int BN, bool TA, bool TB, bool SYRK, bool MIRROR = true,
          bool UPA = false>
__global__ __launch_bounds__(256, BM >= 128 ? 2 : 3) void dgemm_kernel(int M, int N, int K, double alpha,
                                                    const TA_ *__restrict__ A, int64_t lda,
                                                    const TB_ *__restrict__ B, int64_t ldb,
                                                    double beta, double *__restrict__ C,
                                                    int64_t ldc, int kchunk, int64_t zstride) {
  __shared__ double As[2][KC][BM + PAD];
  __shared__ double Bs[2][KC][BN + PAD];
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  int tm, tn;
  if (SYRK) {  // blockIdx.x enumerates lower-triangle tiles (I >= J)
    const int b = blockIdx.x;
    int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= b) ++I;
    while (I * (I + 1) / 2 > b) --I;
    const int J = b - I * (I + 1) / 2;
    tm = I * BM;
    tn = J * BN;
  } else {
    tm = blockIdx.y * BM;
    tn = blockIdx.x * BN;
  }
  doublex4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};

  // split-K: workgroup z covers k in [kb, ke) and writes C + z * zstride
  int kb = blockIdx.z * kchunk;
  const int ke = min(K, kb + kchunk);
  if (UPA) kb = max(kb, (tm / KC) * KC);
  C += int64_t(blockIdx.z) * zstride;
  mainloop<TA_, TB_, BM, BN, TA, TB>(A, lda, B, ldb, M, N, kb, ke, tm, tn, As, Bs, acc);
  epilogue<BM, BN, SYRK, MIRROR>(acc, alpha, beta, C, ldc, M, N, tm, tn);
}

// Chunked variant: blockIdx.z = chunk; offsets/dims from ChunkSpec.
// TRI = 1: each chunk's A is upper triangular (K from the tile's first row);
// TRI = 2: each chunk's B is upper triangular (K up to the tile's last column).
template <int BM, int BN, bool TA, bool TB, int TRI = 0>
__global__ __launch_bounds__(256) void dgemm_chunked_kernel(tg::ChunkSpec cs, double alpha,
                                                            const double *__restrict__ A,
                                                            int64_t lda,
                                                            const double *__restrict__ B,
                                                            int64_t ldb, double beta,
                                                            double *__restrict__ C,
                                                            int64_t ldc) {
  __shared__ double As[2][KC][BM + PAD];
  __shared__ double Bs[2][KC][BN + PAD];
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  const int z = blockIdx.z;
  const int kb = z * cs.c;
  const int ke = (z == cs.nc - 1) ? cs.m : kb + cs.c;
  const int h = ke - kb;
  const int M = cs.M < 0 ? h : cs.M, N = cs.N < 0 ? h : cs.N, K = cs.K < 0 ? h : cs.K;
  const int tm = blockIdx.y * BM, tn = blockIdx.x * BN;
  if (tm >= M || tn >= N) return;
  A += int64_t(kb) * cs.a_kb + int64_t(z) * cs.a_z;
  B += int64_t(kb) * cs.b_kb + int64_t(z) * cs.b_z;
  C += int64_t(kb) * cs.c_kb + int64_t(z) * cs.c_z;
  doublex4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  const int k0 = TRI == 1 ? (tm / KC) * KC : 0, k1 = TRI == 2 ? min(K, tn + BN) : K;
  mainloop<double, double, BM, BN, TA, TB>(A, lda, B, ldb, M, N, k0, k1, tm, tn, As, Bs, acc);
  epilogue<BM, BN, false>(acc, alpha, beta, C, ldc, M, N, tm, tn);
}

// ---------------------------------------------------------------------------
// 8-wave FP64 GEMM: 128 x 128 tiles, 512 threads as 2 x 4 waves of 64 x 32
// (4 x 2 MFMA blocks, 64 accumulator registers), two workgroups per CU, so
// four waves per SIMD keep the f64 MFMA pipe fed (one wave alone issues an
// f64 MFMA only every ~128 cycles, two reach 97-99% of peak:
// tools/mfma64_peak.hip).  K in slabs of 16 through a double-buffered k-major
// LDS image (one barrier per slab), 16-byte global loads when the operand
// is 16-byte aligned with an even leading dimension (VEC), 8-byte otherwise.
// SYRK: blockIdx.x enumerates the lower tiles, the result is mirrored.
// ---------------------------------------------------------------------------
constexpr int G8_T = 128, G8_KC = 16, G8_P = G8_T + 16, G8_NT = 512;

// Two doubles of X at [row, idx], [row, idx + 1] (X row-major, ld), zero
// outside rows < R, idx < L; one 16-byte load when both are inside and VEC.
template <bool VEC>
__device__ inline void ld2(const double *__restrict__ X, int64_t ld, int row, int R, int idx, int L,
                           double &v0, double &v1) {
  const bool rok = row < R;
  if (VEC && rok && idx + 1 < L) {
    const double2 v = *reinterpret_cast<const double2 *>(X + int64_t(row) * ld + idx);
    v0 = v.x;
    v1 = v.y;
    return;
  }
  const int rc = rok ? row : 0;
  const double a = X[int64_t(rc) * ld + min(idx, L - 1)];
  const double b = X[int64_t(rc) * ld + min(idx + 1, L - 1)];
  v0 = (rok && idx < L) ? a : 0.0;
  v1 = (rok && idx + 1 < L) ? b : 0.0;
}

// Staging of op(X)[r0 .. r0 + 128) x [k0 .. k0 + 16) (op(X) is R x K) into
// the k-major image S[k][r], four doubles per thread in two pairs.
//  KCONT (op(X)[r][k] = X[r * ld + k]): pair p holds k = 2 (t >> 7) + 8p, +1
//    of row r = t & 127 (16 consecutive rows per 16-lane group: the two
//    8-byte LDS stores per pair are conflict-free);
//  else (op(X)[r][k] = X[k * ld + r]): pair p holds rows 2 (t & 63), +1 of
//    k = (t >> 6) + 8p (one 16-byte LDS store, a wave writes 1 KB contiguous).
template <bool KCONT, bool VEC>
struct Stg8 {
  double v[4];
  __device__ inline void load(const double *__restrict__ X, int64_t ld, int R, int K, int r0,
                              int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (KCONT) {
        const int r = t & 127, k = 2 * (t >> 7) + 8 * p;
        ld2<VEC>(X, ld, r0 + r, R, k0 + k, K, v[2 * p], v[2 * p + 1]);
      } else {
        const int r = 2 * (t & 63), k = (t >> 6) + 8 * p;
        ld2<VEC>(X, ld, k0 + k, K, r0 + r, R, v[2 * p], v[2 * p + 1]);
      }
    }
  }
  __device__ inline void store(double (*S)[G8_P]) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (KCONT) {
        const int r = t & 127, k = 2 * (t >> 7) + 8 * p;
        S[k][r] = v[2 * p];
        S[k + 1][r] = v[2 * p + 1];
      } else {
        const int r = 2 * (t & 63), k = (t >> 6) + 8 * p;
        *reinterpret_cast<double2 *>(&S[k][r]) = double2{v[2 * p], v[2 * p + 1]};
      }
    }
  }
};

// swz (plain GEMM, 1-D grid): block b runs on XCD b % 8 under round-robin
// dispatch (speed only), so the tiles are dealt to the XCDs in contiguous
// ranges, walked 8 tile rows at a time: the workgroups one L2 serves at a
// time cover an 8 x 8 block of tiles and share their row and column panels.
template <bool TA, bool TB, bool VA, bool VB, bool SYRK>
__global__ __launch_bounds__(G8_NT, 4) void dgemm8_kernel(int M, int N, int K, double alpha,
                                                          const double *__restrict__ A, int64_t lda,
                                                          const double *__restrict__ B, int64_t ldb,
                                                          double beta, double *__restrict__ C,
                                                          int64_t ldc, int swz) {
  __shared__ __attribute__((aligned(16))) double As[2][G8_KC][G8_P];
  __shared__ __attribute__((aligned(16))) double Bs[2][G8_KC][G8_P];
  int tm, tn;
  if (SYRK) {
    // swz = 1 in SYRK mode: op(A) = X^T with X upper triangular (K x M), so
    // the lower tile (tm, tn) only sums k < tn + 128; heaviest tiles first
    const int b = swz ? int(gridDim.x) - 1 - int(blockIdx.x) : int(blockIdx.x);
    int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= b) ++I;
    while (I * (I + 1) / 2 > b) --I;
    tm = I * G8_T;
    tn = (b - I * (I + 1) / 2) * G8_T;
    if (swz) K = min(K, tn + G8_T);
  } else if (swz) {
    const int tmn = tg::cdiv(M, G8_T), tnn = tg::cdiv(N, G8_T), nb = tmn * tnn;
    const int per = tg::cdiv(nb, 8);
    const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (L >= nb) return;
    const int GM = 8, gsz = GM * tnn, grp = L / gsz, r = L - grp * gsz;
    const int rows = min(GM, tmn - grp * GM);
    tm = (grp * GM + r % rows) * G8_T;
    tn = (r / rows) * G8_T;
  } else {
    tm = blockIdx.y * G8_T;
    tn = blockIdx.x * G8_T;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;
  doublex4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  // op(A) = A (M x K, k contiguous) or A^T (A is K x M); op(B) is K x N and
  // is staged as op(B)^T (N x K): k contiguous iff B is stored transposed
  Stg8<!TA, VA> sa;
  Stg8<TB, VB> sb;
  if (K > 0) {
    sa.load(A, lda, M, K, tm, 0);
    sb.load(B, ldb, N, K, tn, 0);
    sa.store(As[0]);
    sb.store(Bs[0]);
    if (G8_KC < K) {
      sa.load(A, lda, M, K, tm, G8_KC);
      sb.load(B, ldb, N, K, tn, G8_KC);
    }
    __syncthreads();
    int cur = 0;
    for (int k0 = 0; k0 < K; k0 += G8_KC) {
#pragma unroll
      for (int kk = 0; kk < G8_KC; kk += 4) {
        double af[4], bf[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = As[cur][kk + (lane >> 4)][wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = Bs[cur][kk + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      if (k0 + G8_KC < K) {
        sa.store(As[cur ^ 1]);
        sb.store(Bs[cur ^ 1]);
        if (k0 + 2 * G8_KC < K) {
          sa.load(A, lda, M, K, tm, k0 + 2 * G8_KC);
          sb.load(B, ldb, N, K, tn, k0 + 2 * G8_KC);
        }
      }
      __syncthreads();
      cur ^= 1;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = tm + wm * 64 + i * 16 + (lane >> 4) + 4 * r;
        const int gj = tn + wn * 32 + j * 16 + (lane & 15);
        if (gi < M && gj < N) {
          double *pc = C + int64_t(gi) * ldc + gj;
          const double v = beta == 0.0 ? alpha * acc[i][j][r] : alpha * acc[i][j][r] + beta * *pc;
          *pc = v;
          if (SYRK && tm != tn) C[int64_t(gj) * ldc + gi] = v;
        }
      }
}

inline bool vec_ok(const double *X, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (ld & 1) == 0;
}

template <bool TA, bool TB, bool SYRK>
hipError_t launch8_v(hipStream_t st, dim3 grid, bool va, bool vb, int M, int N, int K,
                     double alpha, const double *A, int64_t lda, const double *B, int64_t ldb,
                     double beta, double *C, int64_t ldc, int swz = 0) {
#define TG_L8(VA_, VB_)                                                                      \
  hipLaunchKernelGGL((dgemm8_kernel<TA, TB, VA_, VB_, SYRK>), grid, dim3(G8_NT), 0, st, M, N, K, \
                     alpha, A, lda, B, ldb, beta, C, ldc, swz)
  if (va && vb) TG_L8(true, true);
  else if (va) TG_L8(true, false);
  else if (vb) TG_L8(false, true);
  else TG_L8(false, false);
#undef TG_L8
  return hipGetLastError();
}

hipError_t launch8(hipStream_t st, bool ta, bool tb, int M, int N, int K, double alpha,
                   const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                   double *C, int64_t ldc) {
  // TG_GEMM_SWZ=0 keeps the 2-D grid (development switch, read per call)
  const char *e = getenv("TG_GEMM_SWZ");
  const int swz = (e && e[0] == '0') ? 0 : 1;
  const int nb = tg::cdiv(N, G8_T) * tg::cdiv(M, G8_T);
  const dim3 grid = swz ? dim3(8 * tg::cdiv(nb, 8)) : dim3(tg::cdiv(N, G8_T), tg::cdiv(M, G8_T));
  const bool va = vec_ok(A, lda), vb = vec_ok(B, ldb);
  if (!ta && !tb) return launch8_v<false, false, false>(st, grid, va, vb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, swz);
  if (!ta && tb) return launch8_v<false, true, false>(st, grid, va, vb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, swz);
  if (ta && !tb) return launch8_v<true, false, false>(st, grid, va, vb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, swz);
  return launch8_v<true, true, false>(st, grid, va, vb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, swz);
}

template <class TA_, class TB_, int BM, int BN, bool TA, bool TB, bool UPA = false>
hipError_t launch(hipStream_t st, int M, int N, int K, double alpha, const TA_ *A, int64_t lda,
                  const TB_ *B, int64_t ldb, double beta, double *C, int64_t ldc, int splits,
                  int64_t zstride) {
  const int kchunk = splits > 1 ? ((tg::cdiv(K, splits) + KC - 1) / KC) * KC : (K > 0 ? K : 1);
  const int nz = splits > 1 ? tg::cdiv(K, kchunk) : 1;
  dim3 grid(tg::cdiv(N, BN), tg::cdiv(M, BM), nz);
  hipLaunchKernelGGL((dgemm_kernel<TA_, TB_, BM, BN, TA, TB, false, true, UPA>), grid, dim3(256), 0,
                     st, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, kchunk, zstride);
  return hipGetLastError();
}

template <class TA_, class TB_, int BM, int BN>
hipError_t dispatch_t(hipStream_t st, bool ta, bool tb, int M, int N, int K, double alpha,
                      const TA_ *A, int64_t lda, const TB_ *B, int64_t ldb, double beta,
                      double *C, int64_t ldc, int splits = 1, int64_t zs = 0) {
  if (!ta && !tb) return launch<TA_, TB_, BM, BN, false, false>(st, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, splits, zs);
  if (!ta && tb) return launch<TA_, TB_, BM, BN, false, true>(st, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, splits, zs);
  if (ta && !tb) return launch<TA_, TB_, BM, BN, true, false>(st, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, splits, zs);
  return launch<TA_, TB_, BM, BN, true, true>(st, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, splits, zs);
}

// C = alpha * sum_z P_z + beta * C
__global__ void splitk_reduce_kernel(const double *__restrict__ P, int nz, int64_t zstride, int M,
                                     int N, double alpha, double beta, double *__restrict__ C,
                                     int64_t ldc) {
  const int64_t total = int64_t(M) * N;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int r = int(idx / N), c = int(idx % N);
    double s = 0.0;
    for (int z = 0; z < nz; ++z) s += P[z * zstride + idx];
    double *p = C + int64_t(r) * ldc + c;
    *p = beta == 0.0 ? alpha * s : alpha * s + beta * *p;
  }
}

template <class T>
hipError_t syrk_t(hipStream_t st, const T *X, int64_t rows, int n, int64_t ldx, double *H,
                  int64_t ldh) {
  constexpr int BT = 64;
  const int nt = tg::cdiv(n, BT);
  const int tiles = nt * (nt + 1) / 2;
  // H += X^T X : op(A) = X^T (A = X stored rows x n -> TA), op(B) = X (K x N, no trans)
  hipLaunchKernelGGL((dgemm_kernel<T, T, BT, BT, true, false, true>), dim3(tiles), dim3(256), 0,
                     st, n, n, int(rows), 1.0, X, ldx, X, ldx, 1.0, H, ldh, int(rows), int64_t(0));
  return hipGetLastError();
}

}  // namespace

namespace tg {
// Tile of the own DGEMM: TG_GEMM_TILE=128|12864|64 forces one (development
// switch, read per call).  Otherwise 128 x 128 (two workgroups per CU, the
// most MFMA work per staged byte) when its tiles fill at least 85% of their
// last round on the chip, else 64 x 64 (three per CU): at M = N = 3058 the
// 576 big tiles run as 512 + 64 (40 TF/s) where 2304 small ones make three
// full rounds (51 TF/s); at 4096^2 the big tiles make two (57 vs 53 TF/s).
static int gemm_tile(int M, int N) {
  if (const char *t = getenv("TG_GEMM_TILE")) return atoi(t);
  static const int slots128 = 2 * [] {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
    return std::max(1, ncu);
  }();
  const int64_t t = int64_t(cdiv(M, 128)) * cdiv(N, 128);
  if (t < slots128 / 2) return 64;
  const int64_t rounds = (t + slots128 - 1) / slots128;
  return double(t) >= 0.85 * double(rounds * slots128) ? 128 : 64;
}

// Which kernel runs the large tiles: TG_GEMM_IMPL=own8 (default: the 8-wave
// kernel) or own (the 4-wave 128 x 128 kernel); read per call (development
// switch).  No vendor BLAS is linked: tools/gemm_bench.py times both against
// torch's hipBLASLt on the solver's shapes.
static int gemm_impl() {
  const char *e = getenv("TG_GEMM_IMPL");
  if (!e) return 2;
  return (e[0] == 'o' && e[1] == 'w' && e[2] == 'n' && e[3] == '8') ? 2 : 1;
}

hipError_t dgemm(hipStream_t st, bool ta, bool tb, int M, int N, int K, double alpha,
                 const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                 double *C, int64_t ldc) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int impl = gemm_impl();
  if (K <= 0) {
    // C = beta * C (alpha * 0): run with K = 0 -> the kernel writes beta*C
  }
  const int tile = gemm_tile(M, N);
  if (tile == 128 && impl == 2 && C != A && C != B)
    return launch8(st, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  if (tile == 128)
    return dispatch_t<double, double, 128, 128>(st, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta,
                                                C, ldc);
  if (tile == 12864)
    return dispatch_t<double, double, 128, 64>(st, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta,
                                               C, ldc);
  return dispatch_t<double, double, 64, 64>(st, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C,
                                            ldc);
}
// C = alpha A B + beta C with A (M x K, M <= K) upper triangular: the
// triangle's zeros are skipped per tile (half the flops of a square A).  The
// tiles' work then falls with the row, so the grid is ordered with the
// heaviest rows first (blockIdx.y = 0 is the top tile row).
hipError_t dgemm_upper_a(hipStream_t st, int M, int N, int K, double alpha, const double *A,
                         int64_t lda, const double *B, int64_t ldb, double beta, double *C,
                         int64_t ldc) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (gemm_tile(M, N) == 128)
    return launch<double, double, 128, 128, false, false, true>(st, M, N, K, alpha, A, lda, B, ldb,
                                                                beta, C, ldc, 1, 0);
  return launch<double, double, 64, 64, false, false, true>(st, M, N, K, alpha, A, lda, B, ldb,
                                                            beta, C, ldc, 1, 0);
}

hipError_t dgemm_chunked(hipStream_t st, bool ta, bool tb, const ChunkSpec &cs, double alpha,
                         const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                         double *C, int64_t ldc, int tri) {
  if (cs.nc <= 0) return hipSuccess;
  if (tri != 0) {  // triangular A (1) or B (2), no transposes
    const int hmax = std::max(cs.c, cs.m - (cs.nc - 1) * cs.c);
    const int M = cs.M < 0 ? hmax : cs.M, N = cs.N < 0 ? hmax : cs.N;
    if (M <= 0 || N <= 0 || ta || tb) return hipErrorInvalidValue;
    const bool big = int64_t(cdiv(M, 128)) * cdiv(N, 128) * cs.nc >= 256 && N > 64;
#define TG_CHT(BM_, TRI_)                                                                        \
  hipLaunchKernelGGL((dgemm_chunked_kernel<BM_, BM_, false, false, TRI_>),                      \
                     dim3(cdiv(N, BM_), cdiv(M, BM_), cs.nc), dim3(256), 0, st, cs, alpha, A,    \
                     lda, B, ldb, beta, C, ldc)
    if (big) {
      if (tri == 1) TG_CHT(128, 1);
      else TG_CHT(128, 2);
    } else {
      if (tri == 1) TG_CHT(64, 1);
      else TG_CHT(64, 2);
    }
#undef TG_CHT
    return hipGetLastError();
  }
  const int hmax = std::max(cs.c, cs.m - (cs.nc - 1) * cs.c);
  const int M = cs.M < 0 ? hmax : cs.M, N = cs.N < 0 ? hmax : cs.N;
  if (M <= 0 || N <= 0) return hipSuccess;
  const bool big = int64_t(cdiv(M, 128)) * cdiv(N, 128) * cs.nc >= 256 && N > 64;
  const bool narrow = N <= 32;
#define TG_CH2(BM_, BN_, TA_, TB_)                                                             \
  hipLaunchKernelGGL((dgemm_chunked_kernel<BM_, BN_, TA_, TB_>),                              \
                     dim3(cdiv(N, BN_), cdiv(M, BM_), cs.nc), dim3(256), 0, st, cs, alpha, A, \
                     lda, B, ldb, beta, C, ldc)
#define TG_CH(BM_, TA_, TB_)                                                                   \
  hipLaunchKernelGGL((dgemm_chunked_kernel<BM_, BM_, TA_, TB_>),                              \
                     dim3(cdiv(N, BM_), cdiv(M, BM_), cs.nc), dim3(256), 0, st, cs, alpha, A, \
                     lda, B, ldb, beta, C, ldc)
#ifndef TG_XG_BM
#define TG_XG_BM 64
#endif
  if (narrow) {
    if (!ta && !tb) TG_CH2(TG_XG_BM, 32, false, false);
    else if (!ta && tb) TG_CH2(TG_XG_BM, 32, false, true);
    else if (ta && !tb) TG_CH2(TG_XG_BM, 32, true, false);
    else TG_CH2(TG_XG_BM, 32, true, true);
  } else if (big) {
    if (!ta && !tb) TG_CH(128, false, false);
    else if (!ta && tb) TG_CH(128, false, true);
    else if (ta && !tb) TG_CH(128, true, false);
    else TG_CH(128, true, true);
  } else {
    if (!ta && !tb) TG_CH(64, false, false);
    else if (!ta && tb) TG_CH(64, false, true);
    else if (ta && !tb) TG_CH(64, true, false);
    else TG_CH(64, true, true);
  }
#undef TG_CH
#undef TG_CH2
  return hipGetLastError();
}

size_t dgemm_splitk_scratch(int M, int N, int splits) {
  return sizeof(double) * size_t(M) * size_t(N) * size_t(splits);
}

hipError_t dgemm_splitk(hipStream_t st, bool ta, bool tb, int M, int N, int K, double alpha,
                        const double *A, int64_t lda, const double *B, int64_t ldb, double beta,
                        double *C, int64_t ldc, int splits, double *scratch) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (splits <= 1 || K < 2 * KC * splits)
    return dgemm(st, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  const int64_t zs = int64_t(M) * N;
  const int kchunk = ((cdiv(K, splits) + KC - 1) / KC) * KC;
  const int nz = cdiv(K, kchunk);
  hipError_t e = dispatch_t<double, double, 64, 64>(st, ta, tb, M, N, K, 1.0, A, lda, B, ldb, 0.0,
                                                    scratch, N, splits, zs);
  if (e != hipSuccess) return e;
  const int blocks = int(std::min<int64_t>(4096, (zs + 255) / 256));
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, scratch, nz, zs, M, N,
                     alpha, beta, C, ldc);
  return hipGetLastError();
}

hipError_t sum_partials(hipStream_t st, const double *P, int nz, int M, int N, double alpha,
                        double beta, double *C, int64_t ldc) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int64_t zs = int64_t(M) * N;
  const int blocks = int(std::min<int64_t>(4096, (zs + 255) / 256));
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, P, nz, zs, M, N, alpha,
                     beta, C, ldc);
  return hipGetLastError();
}

// C = alpha * X^T X + beta * C for an UPPER TRIANGULAR X (n x n, ld ldx;
// its strict lower triangle must hold zeros): lower tiles, mirrored, each
// summing only the rows above its column block (a third of the flops).
hipError_t dsyrk_tn_upper(hipStream_t st, int n, double alpha, const double *X, int64_t ldx,
                          double beta, double *C, int64_t ldc) {
  if (n <= 0) return hipSuccess;
  const int n128 = cdiv(n, 128);
  if (gemm_impl() != 2 || C == X) return dsyrk_tn(st, n, n, alpha, X, ldx, beta, C, ldc);
  const dim3 grid(n128 * (n128 + 1) / 2);
  const bool v = vec_ok(X, ldx);
  return launch8_v<true, false, true>(st, grid, v, v, n, n, n, alpha, X, ldx, X, ldx, beta, C,
                                      ldc, 1);
}

// C = alpha * X^T X + beta * C on lower tiles, mirrored (X is K x n, ld ldx).
// 128 x 128 tiles (two workgroups per CU, the most work per staged byte)
// once there are enough of them for several full rounds.
hipError_t dsyrk_tn(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc) {
  if (n <= 0) return hipSuccess;
  const int n128 = cdiv(n, 128);
  if (n128 * (n128 + 1) / 2 >= 1024 && gemm_impl() == 2 && C != X) {
    const dim3 grid(n128 * (n128 + 1) / 2);
    return vec_ok(X, ldx)
        ? launch8_v<true, false, true>(st, grid, true, true, n, n, K, alpha, X, ldx, X, ldx, beta, C, ldc)
        : launch8_v<true, false, true>(st, grid, false, false, n, n, K, alpha, X, ldx, X, ldx, beta, C, ldc);
  }
  if (n128 * (n128 + 1) / 2 >= 1024) {
    hipLaunchKernelGGL((dgemm_kernel<double, double, 128, 128, true, false, true>),
                       dim3(n128 * (n128 + 1) / 2), dim3(256), 0, st, n, n, K, alpha, X, ldx, X,
                       ldx, beta, C, ldc, K > 0 ? K : 1, int64_t(0));
    return hipGetLastError();
  }
  constexpr int BT = 64;
  const int nt = cdiv(n, BT);
  hipLaunchKernelGGL((dgemm_kernel<double, double, BT, BT, true, false, true>),
                     dim3(nt * (nt + 1) / 2), dim3(256), 0, st, n, n, K, alpha, X, ldx, X, ldx,
                     beta, C, ldc, K > 0 ? K : 1, int64_t(0));
  return hipGetLastError();
}

// As dsyrk_tn, lower tiles only and not mirrored: the strict upper triangle
// outside the diagonal tiles is left stale (readers index (max, min)).
hipError_t dsyrk_tn_lower(hipStream_t st, int n, int K, double alpha, const double *X,
                          int64_t ldx, double beta, double *C, int64_t ldc) {
  if (n <= 0) return hipSuccess;
  constexpr int BT = 64;
  const int nt = cdiv(n, BT);
  hipLaunchKernelGGL((dgemm_kernel<double, double, BT, BT, true, false, true, false>),
                     dim3(nt * (nt + 1) / 2), dim3(256), 0, st, n, n, K, alpha, X, ldx, X, ldx,
                     beta, C, ldc, K > 0 ? K : 1, int64_t(0));
  return hipGetLastError();
}

// C = alpha * X X^T + beta * C on lower tiles, mirrored (X is n x K, ld ldx).
hipError_t dsyrk_nt(hipStream_t st, int n, int K, double alpha, const double *X, int64_t ldx,
                    double beta, double *C, int64_t ldc) {
  if (n <= 0) return hipSuccess;
  constexpr int BT = 64;
  const int nt = cdiv(n, BT);
  hipLaunchKernelGGL((dgemm_kernel<double, double, BT, BT, false, true, true>),
                     dim3(nt * (nt + 1) / 2), dim3(256), 0, st, n, n, K, alpha, X, ldx, X, ldx,
                     beta, C, ldc, K > 0 ? K : 1, int64_t(0));
  return hipGetLastError();
}
}  // namespace tg

extern "C" int tg_dgemm(void *stream, int transA, int transB, int M, int N, int K, double alpha,
                        const double *A, int lda, const double *B, int ldb, double beta,
                        double *C, int ldc) {
  TG_ARG(M >= 0 && N >= 0 && K >= 0, 4, "negative size");
  TG_ARG(A && B && C, 8, "null pointer");
  TG_HIP(tg::dgemm((hipStream_t)stream, transA != 0, transB != 0, M, N, K, alpha, A, lda, B, ldb,
                   beta, C, ldc));
  return 0;
}

extern "C" int tg_syrk_accum(void *stream, const void *X, int x_dtype, int64_t rows, int n,
                             int64_t ldx, double *H, int ldh) {
  TG_ARG(X, 2, "null X");
  TG_ARG(x_dtype >= TG_F16 && x_dtype <= TG_F64, 3, "unsupported dtype");
  TG_ARG(rows >= 0 && rows <= INT32_MAX, 4, "rows out of range");
  TG_ARG(n > 0, 5, "n <= 0");
  TG_ARG(ldx >= n, 6, "ldx < n");
  TG_ARG(H, 7, "null H");
  TG_ARG(ldh >= n, 8, "ldh < n");
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (x_dtype) {
    case TG_F16: e = syrk_t(st, (const __half *)X, rows, n, ldx, H, ldh); break;
    case TG_BF16: e = syrk_t(st, (const __hip_bfloat16 *)X, rows, n, ldx, H, ldh); break;
    case TG_F32: e = syrk_t(st, (const float *)X, rows, n, ldx, H, ldh); break;
    default: e = syrk_t(st, (const double *)X, rows, n, ldx, H, ldh); break;
  }
  TG_HIP(e);
  return 0;
}
