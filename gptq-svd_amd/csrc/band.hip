// Stage 1 of the two-stage eigensolver: dense symmetric -> band (sy2sb).
//
// Replaces the first half of the reduction inside `torch.linalg.eigh`
// (/root/reference/src/TruncGPTQ/gptq_utils.py:92).  The one-stage dlatrd
// reduction (eigh.hip) streams the trailing matrix once per column with two
// grid-wide reductions each; here every panel of SB_B = 32 columns is
// factorised once and applied with GEMM-shaped FP64 MFMA work:
//
//   panel P = A[r0:, p:p+32]  (m = n - r0 rows)
//   TSQR:  level 0 = Householder QR of each leaf of SB_C rows (one workgroup
//          per leaf, the leaf in LDS), level l+1 = QR of the stacked R factors
//          of level l, until one R remains.  Q = D_0 E_1 E_2 ... with D_0
//          block-diagonal over the leaves and E_l embedded on the rows that
//          carry level l's stacked R's.
//   A22 <- Q^T A22 Q, one level at a time, each as the compact-WY two-sided
//          update  X = A22 Y T,  W = X - 1/2 Y T^T Y^T X,  A22 -= Y W^T + W Y^T
//          with Y block-diagonal (chunked grouped GEMMs, gemm64.hip) and the
//          rank-64-per-tile symmetric update on lower tiles, mirrored, so A22
//          stays bitwise symmetric.
//   A[r0:, p:p+32] <- [R; 0]  (and its transpose).
//
// The reflectors (Y, T of every level of every panel) stay in the workspace
// for the back-transformation Z <- Q1 Z of the eigenvectors.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "band.h"
#include "gemm64.h"
#include "reduce.h"
#include "spin.h"

namespace tg {

SbPlan::SbPlan(int n) {
  ncmax = std::max(1, n / SB_C);
  const char *e = getenv("TG_SB_TSQR");
  single = !(e && e[0] == '1') && pqr_rows_per_thread(n) > 0;
  int p = 0;
  while (p + SB_B < n - 1) {
    SbPanel P{};
    P.p = p;
    P.r0 = p + SB_B;
    P.m = n - P.r0;
    if (single) {
      P.L[0] = SbLevel{P.m, 1, ytotal, ttotal};
      ytotal += size_t(P.m) * SB_B;
      ttotal += size_t(SB_B) * SB_B;
      P.nl = 1;
      panels.push_back(P);
      p += SB_B;
      continue;
    }
    int rows = P.m, l = 0;
    while (true) {
      SbLevel &L = P.L[l];
      L.rows = rows;
      L.nc = std::max(1, rows / SB_C);
      L.yoff = ytotal;
      L.toff = ttotal;
      ytotal += size_t(rows) * SB_B;
      ttotal += size_t(L.nc) * SB_B * SB_B;
      ++l;
      if (L.nc == 1) break;
      rows = L.nc * SB_B;
    }
    P.nl = l;
    panels.push_back(P);
    p += SB_B;
  }
}

}  // namespace tg

namespace {

using tg::SB_B;
using tg::SB_C;

typedef double doublex4 __attribute__((ext_vector_type(4)));

// Row map of TSQR level lv: stacked row s of level lv -> row of level 0.
struct RowMap {
  int lv;
  int nc[tg::SB_LV];  // chunks of each level
  __device__ int fwd(int s) const {
    for (int l = lv; l >= 1; --l) s = (s / SB_B) * SB_C + s % SB_B;
    return s;
  }
  __device__ int inv(int r) const {  // -1 if level-0 row r is not in the level's set
    for (int l = 1; l <= lv; ++l) {
      const int I = r / SB_C, o = r % SB_C;
      if (o >= SB_B || I >= nc[l - 1]) return -1;
      r = I * SB_B + o;
    }
    return r;
  }
};

// Cross-lane exchange without the LDS crossbar: partner value of `x` for
// the pairings lane^32, lane^16 (v_permlane{32,16}_swap), lane^15 (DPP
// row_mirror), lane^7 (row_half_mirror), lane^3, lane^1 (quad_perm).
// Each pairing flips a new bit (32, 16, 8 via 15, 4 via 7, 2 via 3, 1), so a
// butterfly over them in this order is a full reduction / reduce-scatter.
// Half-wave sums without selects: v_permlane{32,16}_swap(x, x) leaves the
// lower half's x in one register and the upper half's in the other, lane
// aligned, so their sum is x[l] + x[l ^ 32] (x[l] + x[l ^ 16]) in every lane.
__device__ inline double hsum32(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
__device__ inline double hsum16(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
template <int CTRL>
__device__ inline double xdpp(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
constexpr int DPP_MIRROR = 0x140, DPP_HALF_MIRROR = 0x141, DPP_XOR3 = 0x1B, DPP_XOR1 = 0xB1;

__device__ inline double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}

__device__ inline double wave_allsum(double s) {
  s = hsum32(s);
  s = hsum16(s);
  s += xdpp<DPP_MIRROR>(s);
  s += xdpp<DPP_HALF_MIRROR>(s);
  s += xdpp<DPP_XOR3>(s);
  s += xdpp<DPP_XOR1>(s);
  return s;
}

// Reduce-scatter of the 32 products v * r[l] over the wave: lane ends with
// the sum of column rs_col(lane) (bits 5..1 of the lane id pick the half kept
// at each step).
__device__ inline int rs_col(int lane) {
  return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
         ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
}
// q_l = v0 r0[l] + v1 r1[l], formed inside the first step.
// Swap-based reduce-scatter step: v_permlane{32,16}_swap(a, b) exchanges the
// upper half of `a` with the lower half of `b` (lanes 32-63 / odd 16-lane
// rows), so afterwards one register holds both halves' `a` values and the
// other both halves' `b` values, lane-aligned: their sum is the pairwise
// sum of `a` in the lower half and of `b` in the upper half -- no selects.
__device__ inline double rs_swap32(double a, double b) {
  const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
__device__ inline double rs_swap16(double a, double b) {
  const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}

__device__ inline double reduce_scatter32(const double (&r0)[32], const double (&r1)[32],
                                          double v0, double v1, int lane) {
  auto qf = [&](int l) { return v0 * r0[l] + v1 * r1[l]; };
  double p[16];
  // lanes 0-31 keep column k, lanes 32-63 column k + 16
#pragma unroll
  for (int k = 0; k < 16; ++k) p[k] = rs_swap32(qf(k), qf(k + 16));
  // even 16-lane rows keep p[k], odd rows p[k + 8]
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = rs_swap16(p[k], p[k + 8]);
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double recv = xdpp<DPP_MIRROR>(up ? p[k] : p[k + 4]);
      p[k] = (up ? p[k + 4] : p[k]) + recv;
    }
  }
  {
    const bool up = (lane & 4) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double recv = xdpp<DPP_HALF_MIRROR>(up ? p[k] : p[k + 2]);
      p[k] = (up ? p[k + 2] : p[k]) + recv;
    }
  }
  {
    const bool up = (lane & 2) != 0;
    const double recv = xdpp<DPP_XOR3>(up ? p[0] : p[1]);
    p[0] = (up ? p[1] : p[0]) + recv;
  }
  return p[0] + xdpp<DPP_XOR1>(p[0]);
}

// Uniform-index access to a register array: a switch on the (scalar) index
// keeps every access static, so the array stays in VGPRs.
#define TG_CASES32(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) \
  X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) \
  X(28) X(29) X(30) X(31)
__device__ inline void ugets(const double (&a)[32], const double (&b)[32], int j, double &x,
                             double &y) {
  switch (j) {
#define TG_GET(k)  \
  case k:          \
    x = a[k];      \
    y = b[k];      \
    break;
    TG_CASES32(TG_GET)
#undef TG_GET
    default: x = y = 0.0;
  }
}
__device__ inline void usets(double (&a)[32], double (&b)[32], int j, double x, double y) {
  switch (j) {
#define TG_SET(k)  \
  case k:          \
    a[k] = x;      \
    b[k] = y;      \
    break;
    TG_CASES32(TG_SET)
#undef TG_SET
    default: break;
  }
}

// Householder QR of one leaf (chunk z of `m` rows, rows kb..ke of src, 32
// columns, row stride ld).  Thread t holds rows t and t + 256 in registers
// (rows >= h are zero, so every leaf runs exactly 32 steps: a zero
// subcolumn gives tau = 0).  Outputs (chunk layout, row-major, stride 32):
// Y rows kb..ke (unit lower trapezoid), YT = Y T, T[z] (dlarft
// forward/columnwise: H_0 H_1 ... = I - Y T Y^T), R[z] (32x32 upper).
// Per column one scalar and one 32-wide reduction; the latter gives both
// w = v^T P (trailing columns) and Y^T v (the new T column), and thread a of
// wave 0 extends row a of T in registers: T[a][j] = -tau_j sum_c T[a][c] q_c.
constexpr int QT = 256;
// STATS: per-phase s_memrealtime stamps (TG_QR_STATS); off in production, the
// stamps wait on lgkmcnt and lengthen the serial column chain.
template <bool STATS>
__global__ __launch_bounds__(QT) void tsqr_qr_kernel(const double *__restrict__ src, int64_t ld,
                                                     int c, int nc, int m,
                                                     double *__restrict__ Yo,
                                                     double *__restrict__ To,
                                                     double *__restrict__ Ro,
                                                     double *__restrict__ YTo,
                                                     unsigned long long *__restrict__ qst) {
  __shared__ double prow[SB_B];
  uint64_t ph[5] = {0, 0, 0, 0, 0};
  __shared__ double red[QT / 64][SB_B];
  __shared__ double qw[SB_B], taus[SB_B];
  __shared__ double Ts[SB_B][SB_B + 1];
  __shared__ double Gs[SB_B][SB_B + 1];
  const int z = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kb = z * c, ke = (z == nc - 1) ? m : kb + c, h = ke - kb;
  double r0[SB_B], r1[SB_B];
  auto load_row = [&](int i, double(&r)[SB_B]) {
    if (i < h) {
      const double *p = src + int64_t(kb + i) * ld;
#pragma unroll
      for (int l = 0; l < SB_B; ++l) r[l] = p[l];
    } else {
#pragma unroll
      for (int l = 0; l < SB_B; ++l) r[l] = 0.0;
    }
  };
  load_row(tid, r0);
  load_row(tid + QT, r1);
  for (int idx = tid; idx < SB_B * (SB_B + 1); idx += QT) (&Ts[0][0])[idx] = 0.0;
  const int mycol = rs_col(lane);
  // One reduction per column: with the raw column x as weights,
  // d_l = sum_{i>j} x_i P[i][l] gives both the squared norm (l = j) and,
  // since v = (x_i scal)_{i>j} with v_j = 1, every v^T P[:, l] =
  // P[j][l] + scal d_l (l > j: the update, l < j: the T recurrence input).
  auto step = [&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const uint64_t p0 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    const double x0 = r0[j], x1 = r1[j];
    if (tid == j) {
#pragma unroll
      for (int l = 0; l < SB_B; ++l) prow[l] = r0[l];
    }
    const double d = reduce_scatter32(r0, r1, (tid > j) ? x0 : 0.0, x1, lane);
    const uint64_t p1 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if ((lane & 1) == 0) red[wid][mycol] = d;
    __syncthreads();
    const uint64_t p2 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    const double s = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
    const double alpha = prow[j];
    double tau = 0.0, scal = 0.0, beta = alpha;
    if (s != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + s), alpha);
      // reciprocals by v_rcp_f64 + two Newton steps (~1 ulp): the two IEEE
      // division sequences sit on the serial column chain
      tau = (beta - alpha) * rcp_nr(beta);
      scal = rcp_nr(alpha - beta);
    }
    const uint64_t p3 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if (tid < SB_B) {
      const double dl = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
      const double a = prow[tid] + scal * dl;
      qw[tid] = a;
      Gs[tid][j] = tid < j ? a : 0.0;  // (Y^T v_j)_tid, the T recurrence input
    }
    if (tid == 0) taus[j] = tau;
    __syncthreads();
    const uint64_t p4 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    const double v0 = (tid > j) ? x0 * scal : (tid == j ? 1.0 : 0.0);
    const double v1 = x1 * scal;
    const double tv0 = tau * v0, tv1 = tau * v1;
#pragma unroll
    for (int l = j + 1; l < SB_B; ++l) {
      const double w = qw[l];
      r0[l] -= tv0 * w;
      r1[l] -= tv1 * w;
    }
    r0[j] = (tid > j) ? v0 : (tid == j ? beta : x0);
    r1[j] = v1;
    const uint64_t p5 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if constexpr (STATS) {
      ph[0] += p1 - p0; ph[1] += p2 - p1; ph[2] += p3 - p2; ph[3] += p4 - p3; ph[4] += p5 - p4;
    }
  };
  [&]<int... J>(std::integer_sequence<int, J...>) {
    (step(std::integral_constant<int, J>{}), ...);
  }(std::make_integer_sequence<int, SB_B>{});
  if (STATS && qst && tid == 0) {
    for (int k = 0; k < 5; ++k) atomicAdd(qst + k, (unsigned long long)ph[k]);
    atomicAdd(qst + 5, 1ull);
  }
  // T (dlarft, forward columnwise): row a is independent of the other rows:
  // T[a][j] = -tau_j sum_{c<j} T[a][c] G[c][j], T[a][a] = tau_a, T[a][c<a] = 0.
  __syncthreads();
  if (tid < SB_B) {
    double trow[SB_B];
#pragma unroll
    for (int c2 = 0; c2 < SB_B; ++c2) trow[c2] = 0.0;
#pragma unroll
    for (int j = 0; j < SB_B; ++j) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
      for (int c2 = 0; c2 < j; c2 += 4) {
        a0 += trow[c2] * Gs[c2][j];
        if (c2 + 1 < j) a1 += trow[c2 + 1] * Gs[c2 + 1][j];
        if (c2 + 2 < j) a2 += trow[c2 + 2] * Gs[c2 + 2][j];
        if (c2 + 3 < j) a3 += trow[c2 + 3] * Gs[c2 + 3][j];
      }
      const double tj = taus[j];
      trow[j] = (tid < j) ? -tj * ((a0 + a1) + (a2 + a3)) : (tid == j ? tj : 0.0);
    }
#pragma unroll
    for (int c2 = 0; c2 < SB_B; ++c2) Ts[tid][c2] = trow[c2];
  }
  if (tid < SB_B) {
    double *ro = Ro + size_t(z) * SB_B * SB_B + tid * SB_B;
#pragma unroll
    for (int l = 0; l < SB_B; ++l) ro[l] = (l >= tid) ? r0[l] : 0.0;
  }
  __syncthreads();
  auto emit = [&](int i, double(&r)[SB_B]) {
    if (i >= h) return;
#pragma unroll
    for (int l = 0; l < SB_B; ++l) r[l] = (i == l) ? 1.0 : (i > l ? r[l] : 0.0);  // Y row
    double *yo = Yo + int64_t(kb + i) * SB_B;
    double *yt = YTo + int64_t(kb + i) * SB_B;
#pragma unroll
    for (int l = 0; l < SB_B; ++l) yo[l] = r[l];
#pragma unroll
    for (int l = 0; l < SB_B; ++l) {
      double a = 0.0;
#pragma unroll
      for (int a2 = 0; a2 <= l; ++a2) a += r[a2] * Ts[a2][l];
      yt[l] = a;
    }
  };
  emit(tid, r0);
  emit(tid + QT, r1);
  for (int idx = tid; idx < SB_B * SB_B; idx += QT)
    To[size_t(z) * SB_B * SB_B + idx] = Ts[idx >> 5][idx & 31];
}

hipError_t launch_qr(hipStream_t st, const double *src, int64_t ld, int nc, int m, double *Y,
                     double *T, double *R, double *YT) {
  const int hmax = (nc == 1) ? m : std::max(SB_C, m - (nc - 1) * SB_C);
  if (hmax > 2 * QT) return hipErrorInvalidValue;
  // Householder QR of the nc leaves: ~2 h b^2 flops per leaf
  auto tok = tg::prof_begin(st, tg::PROF_TSQR, 16.0 * m * SB_B, 2.0 * m * SB_B * SB_B);
  static unsigned long long *qst = nullptr;
  static bool want = getenv("TG_QR_STATS") != nullptr;
  if (want && !qst) {
    (void)hipMalloc(&qst, 8 * sizeof(unsigned long long));
    (void)hipMemset(qst, 0, 8 * sizeof(unsigned long long));
    atexit([] {
      unsigned long long h[8];
      (void)hipMemcpy(h, qst, sizeof(h), hipMemcpyDeviceToHost);
      fprintf(stderr, "qr per column (us): rs %.2f  red+bar %.2f  scal %.2f  qv+bar %.2f  upd %.2f (WGs %llu)\n",
              h[0] / 100.0 / h[5] / 32, h[1] / 100.0 / h[5] / 32, h[2] / 100.0 / h[5] / 32,
              h[3] / 100.0 / h[5] / 32, h[4] / 100.0 / h[5] / 32, h[5]);
    });
  }
  if (qst)
    hipLaunchKernelGGL(tsqr_qr_kernel<true>, dim3(nc), dim3(QT), 0, st, src, ld, SB_C, nc, m, Y, T,
                       R, YT, qst);
  else
    hipLaunchKernelGGL(tsqr_qr_kernel<false>, dim3(nc), dim3(QT), 0, st, src, ld, SB_C, nc, m, Y, T,
                       R, YT, nullptr);
  tg::prof_end(st, tok);
  return hipGetLastError();
}

// Per (column block J of 32, chunk I): P = Y_I^T Z[chunk rows, J cols]
// (32 x 32) on FP64 MFMA, then
//   MODE 0: M[I-block rows, J-block cols] = T_I^T P            (two-sided update)
//   MODE 1: Z[chunk rows, J cols] -= Y_I (T_I P)                (back-transform Q Z)
// 8 waves, wave w owns chunk rows 64w..64w+63 (chunks hold < 512 rows) as
// eight 16x16 C-layout fragments; since the f64 MFMA C/D layout (lane l,
// reg q -> row (l>>4)+4q, col l&15) equals the B-operand layout for four
// consecutive K-steps, the same registers are the B operand of P = Y^T Z and
// the accumulator of Z -= Y (T P).  GATHER: stacked row s lives at Z row
// map(s) (TSQR levels >= 1).
template <int MODE, bool GATHER>
__global__ __launch_bounds__(512) void ytz_kernel(const double *__restrict__ Y,
                                                  const double *__restrict__ T,
                                                  double *__restrict__ Z, int64_t ldz, int ncols,
                                                  int c, int nc, int rows, RowMap mp,
                                                  double *__restrict__ M, int64_t ldm) {
  __shared__ double red[8][SB_B][SB_B + 1];
  __shared__ double Ps[SB_B][SB_B + 1];
  __shared__ double Ms[SB_B][SB_B + 1];
  const int J = blockIdx.x, I = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kb = I * c, ke = (I == nc - 1) ? rows : kb + c;
  const int h = ke - kb;
  const int c0 = J * SB_B;
  const int lr = lane >> 4, lc = lane & 15;
  doublex4 F[4][2];
  // load the wave's 64 x 32 slab of Z (zeros outside the chunk / columns)
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
      const int rc = min(rl, h - 1);
      const int zr = GATHER ? mp.fwd(kb + rc) : kb + rc;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        F[rb][cb][q] = Z[int64_t(zr) * ldz + min(c0 + cb * 16 + lc, ncols - 1)];
    }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        F[rb][cb][q] = (rl < h && c0 + cb * 16 + lc < ncols) ? F[rb][cb][q] : 0.0;
    }
  // P_w = Y_w^T Z_w
  doublex4 Pa[2][2];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + 4 * q + lr;
      double ya[2];
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
        ya[ia] = Y[int64_t(kb + min(rl, h - 1)) * SB_B + ia * 16 + lc];
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) ya[ia] = rl < h ? ya[ia] : 0.0;
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[ia], F[rb][cb][q], Pa[ia][cb], 0, 0, 0);
    }
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[wid][ia * 16 + lr + 4 * q][cb * 16 + lc] = Pa[ia][cb][q];
  __syncthreads();
  for (int idx = tid; idx < SB_B * SB_B; idx += 512) {
    const int a = idx >> 5, cc = idx & 31;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w][a][cc];
    Ps[a][cc] = v;
  }
  __syncthreads();
  for (int idx = tid; idx < SB_B * SB_B; idx += 512)
    Ms[idx >> 5][idx & 31] = T[size_t(I) * SB_B * SB_B + idx];
  __syncthreads();
  double mval[2];
  for (int idx = tid, t = 0; idx < SB_B * SB_B; idx += 512, ++t) {
    const int a = idx >> 5, cc = idx & 31;
    double v = 0.0;
    if (MODE == 0) {
      for (int e = 0; e <= a; ++e) v += Ms[e][a] * Ps[e][cc];
      if (c0 + cc < ldm) M[int64_t(I * SB_B + a) * ldm + c0 + cc] = v;
    } else {
      for (int e = a; e < SB_B; ++e) v += Ms[a][e] * Ps[e][cc];
      mval[t] = v;
    }
  }
  if (MODE == 0) return;
  __syncthreads();  // T no longer read: Ms <- T P
  for (int idx = tid, t = 0; idx < SB_B * SB_B; idx += 512, ++t) Ms[idx >> 5][idx & 31] = mval[t];
  __syncthreads();
  // Z_w -= Y_w Ms
#pragma unroll
  for (int k0 = 0; k0 < SB_B; k0 += 4) {
    double bm[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) bm[cb] = Ms[k0 + lr][cb * 16 + lc];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int rl = wid * 64 + rb * 16 + lc;
      const double yl = Y[int64_t(kb + min(rl, h - 1)) * SB_B + k0 + lr];
      const double ya = rl < h ? -yl : 0.0;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        F[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, bm[cb], F[rb][cb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
      if (rl >= h) continue;
      const int zr = GATHER ? mp.fwd(kb + rl) : kb + rl;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col = c0 + cb * 16 + lc;
        if (col < ncols) Z[int64_t(zr) * ldz + col] = F[rb][cb][q];
      }
    }
}

// A22 -= Yd X^T + X Yd^T - Yd S Yd^T,  S = (M + M^T)/2  (== Yd W^T + W Yd^T
// with W = X - Yd M / 2).  Yd block-diagonal over chunks of c rows:
//   (Yd X^T)[r][c'] = sum_l Y[r][l] X[c'][I(r)*32 + l]
//   (X Yd^T)[r][c'] = sum_l X[r][J(c')*32 + l] Y[c'][l]
//   (Yd S Yd^T)[r][c'] = (Y[r] S_{I(r)J(c')}) . Y[c']
// 64x64 lower tiles (c is a multiple of 64: a tile lies in one chunk),
// K = 96 in three segments, mirrored: A22 stays bitwise symmetric.
constexpr int S2T = 64, S2K = 16, S2P = 4;
__global__ __launch_bounds__(256) void syr2k_bs_kernel(double *__restrict__ A, int64_t lda, int m,
                                                       int c, int nc,
                                                       const double *__restrict__ Y,
                                                       const double *__restrict__ X,
                                                       int64_t ldx,
                                                       const double *__restrict__ M,
                                                       int64_t ldm) {
  // one LDS block: As, Bs, YS during the K loop, then the 64 x 65 tile for the
  // coalesced mirror stores
  constexpr int SMN = (2 * S2K + SB_B) * (S2T + S2P);
  static_assert(SMN >= S2T * (S2T + 1), "mirror tile must fit");
  __shared__ double sm[SMN];
  double(*As)[S2T + S2P] = reinterpret_cast<double(*)[S2T + S2P]>(sm);
  double(*Bs)[S2T + S2P] = reinterpret_cast<double(*)[S2T + S2P]>(sm + S2K * (S2T + S2P));
  double(*YS)[S2T + S2P] = reinterpret_cast<double(*)[S2T + S2P]>(sm + 2 * S2K * (S2T + S2P));  // -(Y_rows S_IJ)^T, k-major
  __shared__ double Ss[SB_B][SB_B + 1];
  const int b = blockIdx.x;
  int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  const int J = b - I * (I + 1) / 2;
  const int tm = I * S2T, tn = J * S2T;
  const int ci = min(tm / c, nc - 1), cj = min(tn / c, nc - 1);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // the tile's old values first (clamped addresses): their HBM latency
  // overlaps the S / YS set-up and the K loop instead of following it
  double old[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = min(tm + wm * 32 + i * 16 + (lane >> 4) + 4 * r, m - 1);
        const int gj = min(tn + wn * 32 + j * 16 + (lane & 15), m - 1);
        old[i][j][r] = A[int64_t(gi) * lda + gj];
      }
  // S_IJ and YS = -(Y_rows S_IJ)
  for (int idx = tid; idx < SB_B * SB_B; idx += 256) {
    const int x = idx >> 5, y = idx & 31;
    Ss[x][y] = 0.5 * (M[int64_t(ci * SB_B + x) * ldm + cj * SB_B + y] +
                      M[int64_t(cj * SB_B + y) * ldm + ci * SB_B + x]);
  }
  __syncthreads();
  {
    const int i = tid >> 2, b0 = (tid & 3) * 8;  // row i, columns b0..b0+7
    const int gr = tm + i;
    double yr[SB_B];
#pragma unroll
    for (int l = 0; l < SB_B; ++l) yr[l] = gr < m ? Y[int64_t(gr) * SB_B + l] : 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      double v = 0.0;
#pragma unroll
      for (int l = 0; l < SB_B; ++l) v += yr[l] * Ss[l][b0 + q];
      YS[b0 + q][i] = -v;
    }
  }
  doublex4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  const int sr = tid >> 2, sk = (tid & 3) * 4;
  for (int k0 = 0; k0 < 3 * SB_B; k0 += S2K) {
    const int seg = k0 / SB_B;
    const int kl = (k0 & 31) + sk;
    double va[4], vb[4];
    {
      const int gr = tm + sr, grc = min(gr, m - 1);
      const double *src = seg ? X + int64_t(grc) * ldx + cj * SB_B + kl : Y + int64_t(grc) * SB_B + kl;
#pragma unroll
      for (int t = 0; t < 4; ++t) va[t] = src[t];
    }
    {
      const int gr = tn + sr, grc = min(gr, m - 1);
      const double *src = seg == 0 ? X + int64_t(grc) * ldx + ci * SB_B + kl : Y + int64_t(grc) * SB_B + kl;
#pragma unroll
      for (int t = 0; t < 4; ++t) vb[t] = src[t];
    }
    if (seg < 2) {
#pragma unroll
      for (int t = 0; t < 4; ++t) As[sk + t][sr] = tm + sr < m ? va[t] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) Bs[sk + t][sr] = tn + sr < m ? vb[t] : 0.0;
    __syncthreads();
    double(*Ap)[S2T + S2P] = seg < 2 ? As : YS + (k0 & 31);
#pragma unroll
    for (int kq = 0; kq < S2K; kq += 4) {
      double af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = Ap[kq + (lane >> 4)][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bs[kq + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // the lower tile written and, for an off-diagonal tile, its transpose
  // written row-contiguous from LDS
  double(*Tt)[S2T + 1] = reinterpret_cast<double(*)[S2T + 1]>(sm);  // K loop done (barrier)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wm * 32 + i * 16 + (lane >> 4) + 4 * r, lj = wn * 32 + j * 16 + (lane & 15);
        const int gi = tm + li, gj = tn + lj;
        if (gi < m && gj < m && gi >= gj) {
          const double v = old[i][j][r] - acc[i][j][r];
          A[int64_t(gi) * lda + gj] = v;
          if (tm != tn) Tt[li][lj] = v;
          else if (gi != gj) A[int64_t(gj) * lda + gi] = v;
        }
      }
  if (tm != tn) {
    __syncthreads();
    for (int idx = tid; idx < S2T * S2T; idx += 256) {
      const int lc = idx >> 6, lr = idx & 63;  // row tn + lc, column tm + lr
      if (tn + lc < m && tm + lr < m) A[int64_t(tn + lc) * lda + tm + lr] = Tt[lr][lc];
    }
  }
}

// Single-level panels: X = A22 YT (m x 32, K = m) by row blocks, with the
// 32 x 32 products Y_zᵀ X_z of the blocks reduced on the way to
// M = Tᵀ (Yᵀ X) -- replaces the split-K GEMM over 256-row blocks of A22ᵀ,
// its partial sum and the separate M reduction (three launches).
// One workgroup per XR rows of X, XW waves splitting K (interleaved steps),
// each accumulating a 16 x 32 tile on FP64 MFMA with DA steps of loads in
// flight; the XW tiles are summed in wave order.  Yᵀ X partials: per
// workgroup, then per group of XG workgroups by its last arriver, then (more
// than one group) over the groups by the last group -- fixed orders, so the
// sums are bit-reproducible; the last arriver forms M.  Tickets: tick[0 ..
// groups) and tick[groups], zero before the launch, reset by their last
// arrivers.
constexpr int XR = 16, XW = 8, XG = 32;
struct XmArgs {
  const double *A;  // A22, lda
  int64_t lda;
  int m;
  const double *YT, *Y, *T;
  double *X, *part, *gpart, *M;
  unsigned *tick;
  int asm_loads;  // K loop with the hand-written loads and waits (TG_XM_ASM, default 1)
  // panel pairs (NBC = 2 only): panel a's deferred factors Ya = Y_a', Wa =
  // W_a' (rows of this panel's A22, ld 32) -> the corrections' products
  // P = Wa^T YT, Q = Ya^T YT, E1 = Y^T Ya, E2 = Y^T Wa ride on the block
  // partials and the last arriver writes PQ = {P, Q, T^T (E1 P + E2 Q)}
  // (what pair_part_kernel + pair_fin_kernel form otherwise); null: none
  const double *Ya, *Wa;
  double *PQ;
  // fused W (no pair products; every workgroup resident): after M, every
  // workgroup turns its rows of X into W = X - Y M / 2 in place (what
  // w_update_kernel does, same operations): the last arriver publishes M
  // write-through and raises *mflag to epoch, the others wait for it
  int fuse_w;
  unsigned *mflag, epoch;
  unsigned *stall;  // timeout flag of the wait (the band reduction's, pq_ctl[0])
  unsigned long long timeout;
  // K split: S workgroups per column block, each over kc rows of A22 (a
  // multiple of 32); their partial X blocks meet in xpart (write-through) and
  // the last of the S (ticket cbt[cb], reset by it) sums them in split order
  // and goes on as the block's workgroup.  S = 1: no split.
  int S, kc;
  double *xpart;
  unsigned *cbt;
};
// doubles of one block's partials: Y^T X, + the four pair products
__host__ __device__ inline int xm_np(const XmArgs &g) { return g.Ya ? 5 : 1; }
// The product is formed transposed, Xᵀ[:, j-block] = YTᵀ · A22[:, j-block]
// (A22 symmetric): the MFMA B operand is then 4 rows x 16 consecutive
// columns of A22, so lane l reads A22[k + l/16][j0 + l%16] and every load
// instruction covers four whole 128-B lines (the row-block form, A operand =
// 16 rows x 4 k, touched sixteen half-used lines per instruction and
// streamed at ~8 GB/s per CU).  The A operand is YTᵀ: lane l reads
// YT[k + l/16][16 i + l%16], 128 B of an L2-resident row.  All workgroups
// sweep K in the same order, so at any moment they read neighbouring strips
// of the same rows of A22.
// NBC 16-column blocks per workgroup (XR = 16 NBC rows of X): the YT
// fragments of a step feed all NBC blocks, so YT's L2 -> CU traffic is
// 16 m^2 / NBC bytes per panel against A22's 8 m^2.  NBC = 2 once the grid
// still covers the chip (m >= XM_WIDE).
constexpr int XM_WIDE = 6144;
// TG_XM_PACK (build-time, NBC = 2): a lane's two A22 values are adjacent
// columns (r0 + 2j, r0 + 2j + 1) and its two YT values adjacent YT columns
// (2j, 2j + 1), one 16-byte load each -- two load instructions per step
// instead of four, the same bytes.  MFMA block c then holds the columns of
// parity c and block i the YT columns of parity i; the products, their k
// order and so every X entry are unchanged, only where they land in the
// accumulators (the reduction's LDS image is written accordingly).
#ifndef TG_XM_PACK
#define TG_XM_PACK 1
#endif
#ifndef TG_XM_DA2
#define TG_XM_DA2 6
#endif
#ifndef TG_XM_MINW2
#define TG_XM_MINW2 4
#endif
// NBC = 1: TG_XM_PACK1 packs the two YT values (the single A22 value stays
// one 8-byte load), TG_XM_DA1 steps in flight
#ifndef TG_XM_PACK1
#define TG_XM_PACK1 0
#endif
#ifndef TG_XM_DA1
#define TG_XM_DA1 8
#endif
template <int NBC>
constexpr bool xm_pack() { return NBC == 2 && TG_XM_PACK; }
template <int NBC>
constexpr bool xm_pack_yt() { return NBC == 2 ? TG_XM_PACK : TG_XM_PACK1; }
typedef double xm_d2 __attribute__((ext_vector_type(2)));
template <int NBC>
struct XmStep {
  double b[NBC];
  xm_d2 ap;  // YT values (a[0], a[1])
};
template <>
struct XmStep<2> {
  xm_d2 bp, ap;  // packed: (b[0], b[1]), (a[0], a[1]) -- or unpacked, element-wise
};
template <int NBC>
__device__ __forceinline__ double xm_b(const XmStep<NBC> &f, int c) { return f.b[c]; }
template <>
__device__ __forceinline__ double xm_b<2>(const XmStep<2> &f, int c) { return f.bp[c]; }
template <int NBC>
__device__ __forceinline__ double xm_a(const XmStep<NBC> &f, int i) { return f.ap[i]; }
template <int NBC>
__device__ __forceinline__ void xm_load(const XmArgs &g, const int (&col)[NBC], int k0,
                                        XmStep<NBC> &f) {
  const int lane = threadIdx.x & 63;
  const int k = min(k0 + (lane >> 4), g.m - 1);
  if constexpr (xm_pack<NBC>()) {  // col[0] = the pair's first column
    f.bp = *reinterpret_cast<const xm_d2 *>(g.A + int64_t(k) * g.lda + col[0]);
    f.ap = *reinterpret_cast<const xm_d2 *>(g.YT + int64_t(k) * SB_B + 2 * (lane & 15));
  } else if constexpr (NBC == 2) {
    f.bp[0] = g.A[int64_t(k) * g.lda + col[0]];
    f.bp[1] = g.A[int64_t(k) * g.lda + col[1]];
    f.ap[0] = g.YT[int64_t(k) * SB_B + (lane & 15)];
    f.ap[1] = g.YT[int64_t(k) * SB_B + 16 + (lane & 15)];
  } else {
#pragma unroll
    for (int c = 0; c < NBC; ++c) f.b[c] = g.A[int64_t(k) * g.lda + col[c]];
    if constexpr (xm_pack_yt<NBC>()) {
      f.ap = *reinterpret_cast<const xm_d2 *>(g.YT + int64_t(k) * SB_B + 2 * (lane & 15));
    } else {
      f.ap[0] = g.YT[int64_t(k) * SB_B + (lane & 15)];
      f.ap[1] = g.YT[int64_t(k) * SB_B + 16 + (lane & 15)];
    }
  }
}
// The same loads as inline asm, with the waits written out (TG_XM_ASM, the
// default): with the compiler's loads the K loop's back edge carried DA
// steps of pending loads and the compiler waited for ALL of them at the loop
// header (s_waitcnt vmcnt(0) once per DA steps), so each wave had between 0
// and DA steps in flight.  Here step u's slot waits only for its own loads
// (vmcnt = the loads of the DA - 1 younger steps), so DA - 1 steps stay in
// flight across the back edge.  The waits tie the slot's registers ("+v"), so
// nothing that reads them is scheduled above the wait, and the loop exit
// drains every slot before the registers are reused.
__device__ __forceinline__ double xm_gload(const double *p) {
  double v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
__device__ __forceinline__ xm_d2 xm_gload2(const double *p) {
  xm_d2 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
template <int NBC>
__device__ __forceinline__ void xm_load_asm(const XmArgs &g, const int (&col)[NBC], int k0,
                                            XmStep<NBC> &f) {
  const int lane = threadIdx.x & 63;
  const int k = min(k0 + (lane >> 4), g.m - 1);
  if constexpr (xm_pack<NBC>()) {
    f.bp = xm_gload2(g.A + int64_t(k) * g.lda + col[0]);
    f.ap = xm_gload2(g.YT + int64_t(k) * SB_B + 2 * (lane & 15));
  } else if constexpr (NBC == 2) {
    f.bp[0] = xm_gload(g.A + int64_t(k) * g.lda + col[0]);
    f.bp[1] = xm_gload(g.A + int64_t(k) * g.lda + col[1]);
    const double *yt = g.YT + int64_t(k) * SB_B + (lane & 15);
    f.ap[0] = xm_gload(yt);
    f.ap[1] = xm_gload(yt + 16);
  } else {
#pragma unroll
    for (int c = 0; c < NBC; ++c) f.b[c] = xm_gload(g.A + int64_t(k) * g.lda + col[c]);
    if constexpr (xm_pack_yt<NBC>()) {
      f.ap = xm_gload2(g.YT + int64_t(k) * SB_B + 2 * (lane & 15));
    } else {
      const double *yt = g.YT + int64_t(k) * SB_B + (lane & 15);
      f.ap[0] = xm_gload(yt);
      f.ap[1] = xm_gload(yt + 16);
    }
  }
}
// load instructions per step slot
template <int NBC>
constexpr int xm_lps() { return xm_pack<NBC>() ? 2 : NBC + (xm_pack_yt<NBC>() ? 1 : 2); }
// wait until step slot f's loads are in: the DA - 1 younger steps' loads
// may stay outstanding
template <int NBC, int DA>
__device__ __forceinline__ void xm_wait_slot(XmStep<NBC> &f) {
  constexpr int W = (DA - 1) * xm_lps<NBC>();
  static_assert(W <= 63, "xm wait count exceeds the vmcnt field");
  if constexpr (NBC == 2) {
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(f.bp[0]), "+v"(f.bp[1]), "+v"(f.ap[0]), "+v"(f.ap[1])
                 : "n"(W));
  } else {
    asm volatile("s_waitcnt vmcnt(%3)" : "+v"(f.b[0]), "+v"(f.ap[0]), "+v"(f.ap[1]) : "n"(W));
  }
}
template <int NBC>
__device__ __forceinline__ void xm_drain_slot(XmStep<NBC> &f) {
  if constexpr (NBC == 2) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(f.bp[0]), "+v"(f.bp[1]), "+v"(f.ap[0]), "+v"(f.ap[1]));
  } else {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(f.b[0]), "+v"(f.ap[0]), "+v"(f.ap[1]));
  }
}
// sh (packed loads only): the lane's pair starts at column m - 1 (m odd), so
// its 16-byte load was moved one column left, (m - 2, m - 1), and column
// m - 1's value is the load's second element
template <int NBC>
__device__ __forceinline__ void xm_mma(const XmStep<NBC> &f, const bool (&cok)[NBC], bool sh,
                                       int k0, doublex4 (&acc)[NBC][2], int kend) {
  const bool kok = k0 + ((threadIdx.x & 63) >> 4) < kend;  // rows of this workgroup's K range
#pragma unroll
  for (int c = 0; c < NBC; ++c) {
    double v = xm_b<NBC>(f, c);
    if constexpr (xm_pack<NBC>())
      if (c == 0) v = sh ? xm_b<NBC>(f, 1) : v;
    const double b = (cok[c] && kok) ? v : 0.0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      acc[c][i] = __builtin_amdgcn_mfma_f64_16x16x4f64(xm_a<NBC>(f, i), b, acc[c][i], 0, 0, 0);
  }
}
// sum over z in [z0, z1) of p[z * 1024 + e], in z order, with the L1-
// bypassing loads of a batch all in flight before the first add
__device__ __forceinline__ double xm_sum(const double *p, int z0, int z1, int e,
                                         int stride = 1024) {
  constexpr int NB = 8;
  double s = 0.0;
  for (int zb = z0; zb < z1; zb += NB) {
    double v[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      v[u] = tg::load_partial(&p[size_t(min(zb + u, z1 - 1)) * stride + e]);
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (zb + u < z1) s += v[u];
  }
  return s;
}

// Fused W (XmArgs::fuse_w): wait until M is published, stage it, and turn
// this block's rows of X into W = X - Y M / 2 in place -- per entry the fma
// chain of w_update_kernel (l ascending from 0.0, then x - v / 2), so the
// result is the same.  xs / ys: the block's X / Y rows in LDS; ms: 1024
// doubles of LDS scratch.
template <int NBC>
__device__ __forceinline__ void xm_fused_w(const XmArgs &g, int r0, const double (*xs)[SB_B + 1],
                                        const double (*ys)[SB_B + 1], double *ms) {
  constexpr int RB = XR * NBC;
  const int tid = threadIdx.x;
  if (tid < 64) tg::spin_geq(g.mflag, g.epoch, g.stall, g.timeout);
  __syncthreads();
  for (int e = tid; e < SB_B * SB_B; e += 64 * XW)
    ms[e] = __hip_atomic_load(&g.M[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  for (int e = tid; e < RB * SB_B; e += 64 * XW) {
    const int rr = e >> 5, c = e & 31;
    double v = 0.0;
#pragma unroll
    for (int l = 0; l < SB_B; ++l) v = fma(ys[rr][l], ms[l * SB_B + c], v);
    if (r0 + rr < g.m) g.X[int64_t(r0 + rr) * SB_B + c] = fma(-0.5, v, xs[rr][c]);
  }
}

// NBC = 2 (m >= XM_WIDE, the HBM-resident trailing matrices): two
// workgroups per CU -- 6 K steps in flight per wave (<= 128 registers) and
// the Y / X rows of the block staged in the reduction buffer once it is free
// (<= 80 KB of LDS), so one workgroup's reductions and ramp-up overlap the
// other's stream; at 1 per CU the stream paused through both.
template <int NBC>
constexpr int xm_depth() { return NBC == 2 ? TG_XM_DA2 : TG_XM_DA1; }
template <int NBC>
__global__ __launch_bounds__(64 * XW, NBC == 2 ? TG_XM_MINW2 : 1) void xm_kernel(XmArgs g) {
  constexpr int RB = XR * NBC;                // rows of X per workgroup
  constexpr int DA = xm_depth<NBC>();
  __shared__ double red[XW][RB][SB_B + 1];   // the last workgroup reuses it for C, T
  // the block's X and Y rows in the last two slices (kept through the last
  // arrivers' C / T / pair work in the first ones, for the fused W)
  static_assert(XW >= 8, "xs and ys are red[XW - 2] and red[XW - 1]");
  double(*xs)[SB_B + 1] = red[XW - 2];
  double(*ys)[SB_B + 1] = red[XW - 1];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: uniform K loop
  // column block cb, K split ks (the S splits of a block are adjacent)
  const int cb = int(blockIdx.x) / g.S, ks = int(blockIdx.x) - cb * g.S;
  const int r0 = cb * RB;
  const int G = int(gridDim.x) / g.S, NG = (G + XG - 1) / XG;
  const int kbeg = ks * g.kc, kend = min(g.m, kbeg + g.kc);
  constexpr int YPT = RB * SB_B / (64 * XW);  // Y values per thread
  double yv[YPT];
#pragma unroll
  for (int u = 0; u < YPT; ++u) {
    const int e = tid + u * 64 * XW, rr = e >> 5, c = e & 31, row = r0 + rr;
    yv[u] = row < g.m ? g.Y[int64_t(row) * SB_B + c] : 0.0;
  }
  // wave w takes the K steps w, w + XW, ... (4 rows of A22 each) of the range
  const int KS = 4 * XW, kb = kbeg + 4 * wid;
  int colc[NBC];
  bool cok[NBC];
  // packed pair (m - 1, m) of an odd m: loaded as (m - 2, m - 1), see xm_mma
  const bool csh = xm_pack<NBC>() && r0 + 2 * (lane & 15) > g.m - 2;
#pragma unroll
  for (int c = 0; c < NBC; ++c) {
    if constexpr (xm_pack<NBC>()) {  // columns r0 + 2j + c; colc[0]: the pair, inside A22
      const int col = r0 + 2 * (lane & 15) + c;
      cok[c] = col < g.m;
      colc[c] = min(r0 + 2 * (lane & 15), g.m - 2);
    } else {
      const int col = r0 + 16 * c + (lane & 15);
      cok[c] = col < g.m;
      colc[c] = min(col, g.m - 1);
    }
  }
  doublex4 acc[NBC][2];
#pragma unroll
  for (int c = 0; c < NBC; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[c][i] = doublex4{0.0, 0.0, 0.0, 0.0};
  if (kb < kend && g.asm_loads) {
    const int nit = (kend - kb + KS - 1) / KS;
    XmStep<NBC> f[DA];
#pragma unroll
    for (int u = 0; u < DA; ++u) xm_load_asm<NBC>(g, colc, kb + KS * u, f[u]);
    for (int it = 0; it < nit; it += DA) {
#pragma unroll
      for (int u = 0; u < DA; ++u) {
        const int k0 = kb + KS * (it + u);
        xm_wait_slot<NBC, DA>(f[u]);
        xm_mma<NBC>(f[u], cok, csh, k0, acc, kend);
        xm_load_asm<NBC>(g, colc, k0 + KS * DA, f[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < DA; ++u) xm_drain_slot<NBC>(f[u]);
  } else if (kb < kend) {
    const int nit = (kend - kb + KS - 1) / KS;
    XmStep<NBC> f[DA];
#pragma unroll
    for (int u = 0; u < DA; ++u) xm_load<NBC>(g, colc, kb + KS * u, f[u]);
    // (the compiler drains vmcnt to 0 at the loop header -- the slots are
    // loop-carried -- and waits only for the slot in use inside the body;
    // unrolling 4 or 8 rounds per iteration measured no faster)
    for (int it = 0; it < nit; it += DA) {
#pragma unroll
      for (int u = 0; u < DA; ++u) {
        // scheduling barriers keep the issue order (MFMAs on step it + u,
        // then the load of step it + u + DA into the freed slot): the
        // machine scheduler otherwise sinks prefetches next to their uses
        const int k0 = kb + KS * (it + u);
        xm_mma<NBC>(f[u], cok, csh, k0, acc, kend);
        __builtin_amdgcn_sched_barrier(0);
        xm_load<NBC>(g, colc, k0 + KS * DA, f[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // acc[c][i][q] = Xᵀ[16 i + lane / 16 + 4 q][r0 + 16 c + lane % 16]
#pragma unroll
  for (int c = 0; c < NBC; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if constexpr (xm_pack<NBC>())
          red[wid][2 * (lane & 15) + c][2 * ((lane >> 4) + 4 * q) + i] = acc[c][i][q];
        else if constexpr (xm_pack_yt<NBC>())
          red[wid][16 * c + (lane & 15)][2 * ((lane >> 4) + 4 * q) + i] = acc[c][i][q];
        else
          red[wid][16 * c + (lane & 15)][16 * i + (lane >> 4) + 4 * q] = acc[c][i][q];
  __syncthreads();
  double xv[YPT];
#pragma unroll
  for (int u = 0; u < YPT; ++u) {
    const int e = tid + u * 64 * XW, rr = e >> 5, c = e & 31;
    double x = 0.0;
#pragma unroll
    for (int w = 0; w < XW; ++w) x += red[w][rr][c];
    xv[u] = x;
  }
  if (g.S > 1) {
    // this split's partial X block, write-through; the last of the block's
    // S splits sums them in split order and goes on
    double *mine = g.xpart + (size_t(cb) * g.S + ks) * (RB * SB_B);
#pragma unroll
    for (int u = 0; u < YPT; ++u)
      __hip_atomic_store(&mine[tid + u * 64 * XW], xv[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      s_last = __hip_atomic_fetch_add(&g.cbt[cb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               unsigned(g.S - 1);
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) tg::ctl_reset(&g.cbt[cb]);
    const double *blk = g.xpart + size_t(cb) * g.S * (RB * SB_B);
#pragma unroll
    for (int u = 0; u < YPT; ++u) {
      const int e = tid + u * 64 * XW;
      double x = 0.0;
      for (int z = 0; z < g.S; ++z)
        x += __hip_atomic_load(&blk[size_t(z) * (RB * SB_B) + e], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      xv[u] = x;
    }
  }
#pragma unroll
  for (int u = 0; u < YPT; ++u) {
    const int e = tid + u * 64 * XW, rr = e >> 5, c = e & 31;
    if (r0 + rr < g.m) g.X[int64_t(r0 + rr) * SB_B + c] = xv[u];
    xv[u] = r0 + rr < g.m ? xv[u] : 0.0;
  }
  __syncthreads();  // red is free: its first two slices take the block's X and Y rows
#pragma unroll
  for (int u = 0; u < YPT; ++u) {
    const int e = tid + u * 64 * XW, rr = e >> 5, c = e & 31;
    xs[rr][c] = xv[u];
    ys[rr][c] = yv[u];
  }
  // panel pairs: the block's rows of Ya, Wa and YT in the next three slices
  const bool pp = NBC == 2 && g.Ya != nullptr;  // uniform
  const int NP = pp ? 5 : 1;
  if constexpr (NBC == 2) {
    if (pp) {
#pragma unroll
      for (int u = 0; u < YPT; ++u) {
        const int e = tid + u * 64 * XW, rr = e >> 5, c = e & 31, row = r0 + rr;
        const bool ok = row < g.m;
        const int64_t o = int64_t(ok ? row : 0) * SB_B + c;
        red[2][rr][c] = ok ? g.Ya[o] : 0.0;
        red[3][rr][c] = ok ? g.Wa[o] : 0.0;
        red[4][rr][c] = ok ? g.YT[o] : 0.0;
      }
    }
  }
  __syncthreads();
  // this block's Y_zᵀ X_z (and the pair products), write-through, then the group ticket
  double *mypart = g.part + size_t(cb) * NP * 1024;
  for (int e = tid; e < SB_B * SB_B; e += 64 * XW) {
    const int a = e >> 5, c = e & 31;
    double p = 0.0;
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) p = fma(ys[rr][a], xs[rr][c], p);
    __hip_atomic_store(&mypart[e], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (NBC == 2) {
    if (pp) {
      // k = 0: P = Wa^T YT, 1: Q = Ya^T YT, 2: E1 = Y^T Ya, 3: E2 = Y^T Wa
      for (int e = tid; e < 4 * SB_B * SB_B; e += 64 * XW) {
        const int k = e >> 10, a = (e >> 5) & 31, c = e & 31;
        const double(*L)[SB_B + 1] = k == 0 ? red[3] : k == 1 ? red[2] : ys;
        const double(*R)[SB_B + 1] = k <= 1 ? red[4] : k == 2 ? red[2] : red[3];
        double p = 0.0;
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) p = fma(L[rr][a], R[rr][c], p);
        __hip_atomic_store(&mypart[1024 + e], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int grp = cb / XG, z0 = grp * XG, z1 = min(G, z0 + XG);
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(&g.tick[grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             unsigned(z1 - z0 - 1);
  __syncthreads();
  if (!s_last) {
    if constexpr (NBC == 1)
      if (g.fuse_w) xm_fused_w<NBC>(g, r0, xs, ys, &red[XW - 4][0][0]);
    return;
  }
  // Cs = C (Y^T X), then the pair sums P, Q, E1, E2 (pp); Ts = T
  double *Cs = &red[0][0][0], *Ts = Cs + 5 * SB_B * SB_B;
  static_assert(XW * XR * (SB_B + 1) >= 2 * SB_B * SB_B, "C and T fit in red");
  static_assert(NBC == 1 || XW * XR * NBC * (SB_B + 1) >= 6 * SB_B * SB_B,
                "C, the pair sums and T fit in red");
  if (!pp) Ts = Cs + SB_B * SB_B;
  const int ne = NP * SB_B * SB_B;
  for (int e = tid; e < ne; e += 64 * XW) {
    const double s = xm_sum(g.part, z0, z1, e, NP * 1024);
    if (NG == 1)
      Cs[e] = s;  // one group: its last arriver forms M (no second hand-off)
    else
      __hip_atomic_store(&g.gpart[size_t(grp) * NP * 1024 + e], s, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int e = tid; e < SB_B * SB_B; e += 64 * XW) Ts[e] = g.T[e];
  if (NG > 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      tg::ctl_reset(&g.tick[grp]);
      s_last = __hip_atomic_fetch_add(&g.tick[NG], 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == unsigned(NG - 1);
    }
    __syncthreads();
    if (!s_last) {
      if constexpr (NBC == 1)
        if (g.fuse_w) xm_fused_w<NBC>(g, r0, xs, ys, &red[XW - 4][0][0]);
      return;
    }
    for (int e = tid; e < ne; e += 64 * XW) Cs[e] = xm_sum(g.gpart, 0, NG, e, NP * 1024);
  }
  __syncthreads();
  for (int e = tid; e < SB_B * SB_B; e += 64 * XW) {
    const int a = e >> 5, c = e & 31;
    double v = 0.0;
    for (int k = 0; k <= a; ++k) v = fma(Ts[k * SB_B + a], Cs[k * SB_B + c], v);
    if (NBC == 1 && g.fuse_w)
      __hip_atomic_store(&g.M[e], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
    else
      g.M[e] = v;
  }
  if (NBC == 1 && g.fuse_w) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's M stores drained
    __syncthreads();
    if (tid == 0) {
      tg::ctl_reset(&g.tick[grp]);
      if (NG > 1) tg::ctl_reset(&g.tick[NG]);
      __hip_atomic_store(g.mflag, g.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (NBC == 1) xm_fused_w<NBC>(g, r0, xs, ys, &red[XW - 4][0][0]);
    return;
  }
  if (pp) {
    // PQ[0 .. 2047] = {P, Q}; D = E1 P + E2 Q into C's slot (M is out);
    // PQ[2048 ..] = T^T D
    const double *Ps = Cs + 1024, *Qs = Cs + 2048, *E1 = Cs + 3072, *E2 = Cs + 4096;
    for (int e = tid; e < 2048; e += 64 * XW) g.PQ[e] = Cs[1024 + e];
    __syncthreads();
    for (int e = tid; e < SB_B * SB_B; e += 64 * XW) {
      const int a = e >> 5, c = e & 31;
      double v = 0.0;
#pragma unroll 8
      for (int k = 0; k < SB_B; ++k) v = fma(E1[a * SB_B + k], Ps[k * SB_B + c], v);
#pragma unroll 8
      for (int k = 0; k < SB_B; ++k) v = fma(E2[a * SB_B + k], Qs[k * SB_B + c], v);
      Cs[e] = v;
    }
    __syncthreads();
    for (int e = tid; e < SB_B * SB_B; e += 64 * XW) {
      const int a = e >> 5, c = e & 31;
      double v = 0.0;
      for (int k = 0; k <= a; ++k) v = fma(Ts[k * SB_B + a], Cs[k * SB_B + c], v);
      g.PQ[2048 + e] = v;
    }
  }
  if (tid == 0) {
    tg::ctl_reset(&g.tick[grp]);
    if (NG > 1) tg::ctl_reset(&g.tick[NG]);
  }
}

// Single-level panels: W = X - 1/2 Y M in place over X (m x 32 each, M 32 x
// 32), so the trailing update is the rank-64 A22 -= Y W^T + W Y^T (K = 64
// instead of the K = 96 form above, which folds Y S Y^T into the tiles).
// One workgroup per 16 rows (m / 16 workgroups: the latency of one row's
// loads, not a queue of rows, sets the time): M in LDS, the thread's Y row
// and X pair straight from L2, two outputs per thread.
constexpr int WU_R = 16;
__global__ __launch_bounds__(256) void w_update_kernel(const double *__restrict__ Y,
                                                       double *__restrict__ X, int m,
                                                       const double *__restrict__ M) {
  __shared__ double2 Ms[SB_B][SB_B / 2];
  const int tid = threadIdx.x;
  const int r = blockIdx.x * WU_R + (tid >> 4), c2 = tid & 15;  // row r, columns 2c2, 2c2 + 1
  const int rc = min(r, m - 1);
  double2 y[SB_B / 2];
#pragma unroll
  for (int h = 0; h < SB_B / 2; ++h) y[h] = reinterpret_cast<const double2 *>(Y + int64_t(rc) * SB_B)[h];
  const double2 x = reinterpret_cast<const double2 *>(X + int64_t(rc) * SB_B)[c2];
  for (int e = tid; e < SB_B * SB_B / 2; e += 256)
    Ms[e >> 4][e & 15] = reinterpret_cast<const double2 *>(M)[e];
  __syncthreads();
  double v0 = 0.0, v1 = 0.0;
#pragma unroll
  for (int h = 0; h < SB_B / 2; ++h) {
    const double2 a = Ms[2 * h][c2], b = Ms[2 * h + 1][c2];
    v0 = fma(y[h].x, a.x, v0);
    v1 = fma(y[h].x, a.y, v1);
    v0 = fma(y[h].y, b.x, v0);
    v1 = fma(y[h].y, b.y, v1);
  }
  if (r < m)
    reinterpret_cast<double2 *>(X + int64_t(r) * SB_B)[c2] =
        make_double2(fma(-0.5, v0, x.x), fma(-0.5, v1, x.y));
}

// A22 -= Y W^T + W Y^T on 64 x 64 lower tiles, mirrored (A22 stays bitwise
// symmetric).  The whole K = 64 of both operands is staged at once -- A side
// [Y_rows | W_rows], B side [W_cols | Y_cols], k-major -- behind ONE barrier,
// with the tile's old values already in flight: the K = 96 kernel above
// waits out an L2 round trip per 16-deep slab.  Two workgroups per CU.
constexpr int WT = 64, WK = 2 * SB_B, WP = 4;
// NP (Y, W) pairs: A22 -= sum_p Y_p W_p^T + W_p Y_p^T (NP = 2: two panels'
// updates deferred into one pass over A22, K = 128 staged 64 at a time).
struct YW2 {
  const double *Y[2], *W[2];  // m x 32 each, leading dimension SB_B
};
template <int NP>
__global__ __launch_bounds__(256, 2) void syr2k_w_kernel(double *__restrict__ A, int64_t lda, int m,
                                                         YW2 yw) {
  __shared__ double Aop[WK][WT + WP];
  __shared__ double Bop[WK][WT + WP];
  const int b = blockIdx.x;
  int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  const int J = b - I * (I + 1) / 2;
  const int tm = I * WT, tn = J * WT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  double old[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = min(tm + wm * 32 + i * 16 + (lane >> 4) + 4 * r, m - 1);
        const int gj = min(tn + wn * 32 + j * 16 + (lane & 15), m - 1);
        old[i][j][r] = A[int64_t(gi) * lda + gj];
      }
  doublex4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    if (pp > 0) __syncthreads();  // the previous pair's operand images are consumed
    const double *Y = yw.Y[pp], *W = yw.W[pp];
    {
      // thread: row tid / 4 of the tile, 8 consecutive k (two 16-B loads) of
      // each of Y_r, W_r, W_c, Y_c
      const int rl = tid >> 2, k0 = (tid & 3) * 8;
      const int gr = min(tm + rl, m - 1), gc = min(tn + rl, m - 1);
      const bool okr = tm + rl < m, okc = tn + rl < m;
      double2 v[4][4];
      const double *src[4] = {Y + int64_t(gr) * SB_B + k0, W + int64_t(gr) * SB_B + k0,
                              W + int64_t(gc) * SB_B + k0, Y + int64_t(gc) * SB_B + k0};
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int h = 0; h < 4; ++h) v[o][h] = reinterpret_cast<const double2 *>(src[o])[h];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int k = k0 + 2 * h;
        Aop[k][rl] = okr ? v[0][h].x : 0.0;
        Aop[k + 1][rl] = okr ? v[0][h].y : 0.0;
        Aop[SB_B + k][rl] = okr ? v[1][h].x : 0.0;
        Aop[SB_B + k + 1][rl] = okr ? v[1][h].y : 0.0;
        Bop[k][rl] = okc ? v[2][h].x : 0.0;
        Bop[k + 1][rl] = okc ? v[2][h].y : 0.0;
        Bop[SB_B + k][rl] = okc ? v[3][h].x : 0.0;
        Bop[SB_B + k + 1][rl] = okc ? v[3][h].y : 0.0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kq = 0; kq < WK; kq += 4) {
      double af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = Aop[kq + (lane >> 4)][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bop[kq + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // operand images dead: Aop becomes the mirror tile
  double(*Tt)[WT + 1] = reinterpret_cast<double(*)[WT + 1]>(&Aop[0][0]);
  static_assert(WK * (WT + WP) >= WT * (WT + 1), "mirror tile must fit");
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wm * 32 + i * 16 + (lane >> 4) + 4 * r, lj = wn * 32 + j * 16 + (lane & 15);
        const int gi = tm + li, gj = tn + lj;
        if (gi < m && gj < m && gi >= gj) {
          const double v = old[i][j][r] - acc[i][j][r];
          A[int64_t(gi) * lda + gj] = v;
          if (tm != tn) Tt[li][lj] = v;
          else if (gi != gj) A[int64_t(gj) * lda + gi] = v;
        }
      }
  if (tm != tn) {
    __syncthreads();
    for (int idx = tid; idx < WT * WT; idx += 256) {
      const int lc = idx >> 6, lr = idx & 63;  // row tn + lc, column tm + lr
      if (tn + lc < m && tm + lr < m) A[int64_t(tn + lc) * lda + tm + lr] = Tt[lr][lc];
    }
  }
}

// Persistent form of syr2k_w_kernel<NP> (the default): two workgroups per CU
// loop over the lower tiles; while a tile's operands are staged, multiplied
// and written back, the NEXT tile's old values are already loading (issued
// after this tile's operand loads, so waiting for those leaves them in
// flight).  The one-tile-per-workgroup form left the memory pipe idle
// through every workgroup's MFMA, epilogue and dispatch: 3.7 TB/s on the
// HBM-resident trailing matrices of n >= 12,288.
__device__ __forceinline__ void syr2k_tile(int b, int &tm, int &tn) {
  int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  tm = I * WT;
  tn = (b - I * (I + 1) / 2) * WT;
}
template <int NP>
__global__ __launch_bounds__(256, 2) void syr2k_wp_kernel(double *__restrict__ A, int64_t lda,
                                                          int m, YW2 yw, int ntiles) {
  __shared__ double Aop[WK][WT + WP];
  __shared__ double Bop[WK][WT + WP];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int b = blockIdx.x;
  if (b >= ntiles) return;
  auto load_old = [&](int tb, double (&o)[2][2][4]) __attribute__((always_inline)) {
    int tm, tn;
    syr2k_tile(tb, tm, tn);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = min(tm + wm * 32 + i * 16 + (lane >> 4) + 4 * r, m - 1);
          const int gj = min(tn + wn * 32 + j * 16 + (lane & 15), m - 1);
          o[i][j][r] = A[int64_t(gi) * lda + gj];
        }
  };
  double old[2][2][4], nold[2][2][4];
  load_old(b, old);
  for (; b < ntiles; b += gridDim.x) {
    int tm, tn;
    syr2k_tile(b, tm, tn);
    const int rl = tid >> 2, k0 = (tid & 3) * 8;
    const int gr = min(tm + rl, m - 1), gc = min(tn + rl, m - 1);
    const bool okr = tm + rl < m, okc = tn + rl < m;
    doublex4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      // the previous tile's mirror reads / the previous pair's MFMA reads of Aop are done
      __syncthreads();
      const double *Y = yw.Y[pp], *W = yw.W[pp];
      double2 v[4][4];
      {
        const double *src[4] = {Y + int64_t(gr) * SB_B + k0, W + int64_t(gr) * SB_B + k0,
                                W + int64_t(gc) * SB_B + k0, Y + int64_t(gc) * SB_B + k0};
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
          for (int h = 0; h < 4; ++h) v[o][h] = reinterpret_cast<const double2 *>(src[o])[h];
      }
      if (pp == 0) {
        __builtin_amdgcn_sched_barrier(0);
        const int bn = b + int(gridDim.x);
        if (bn < ntiles) load_old(bn, nold);  // in flight through this tile
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int k = k0 + 2 * h;
        Aop[k][rl] = okr ? v[0][h].x : 0.0;
        Aop[k + 1][rl] = okr ? v[0][h].y : 0.0;
        Aop[SB_B + k][rl] = okr ? v[1][h].x : 0.0;
        Aop[SB_B + k + 1][rl] = okr ? v[1][h].y : 0.0;
        Bop[k][rl] = okc ? v[2][h].x : 0.0;
        Bop[k + 1][rl] = okc ? v[2][h].y : 0.0;
        Bop[SB_B + k][rl] = okc ? v[3][h].x : 0.0;
        Bop[SB_B + k + 1][rl] = okc ? v[3][h].y : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int kq = 0; kq < WK; kq += 4) {
        double af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = Aop[kq + (lane >> 4)][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = Bop[kq + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // operand images dead: Aop becomes the mirror tile
    double(*Tt)[WT + 1] = reinterpret_cast<double(*)[WT + 1]>(&Aop[0][0]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int li = wm * 32 + i * 16 + (lane >> 4) + 4 * r, lj = wn * 32 + j * 16 + (lane & 15);
          const int gi = tm + li, gj = tn + lj;
          if (gi < m && gj < m && gi >= gj) {
            const double val = old[i][j][r] - acc[i][j][r];
            A[int64_t(gi) * lda + gj] = val;
            if (tm != tn) Tt[li][lj] = val;
            else if (gi != gj) A[int64_t(gj) * lda + gi] = val;
          }
        }
    if (tm != tn) {  // uniform per workgroup
      __syncthreads();
      for (int idx = tid; idx < WT * WT; idx += 256) {
        const int lc = idx >> 6, lr = idx & 63;  // row tn + lc, column tm + lr
        if (tn + lc < m && tm + lr < m) A[int64_t(tn + lc) * lda + tm + lr] = Tt[lr][lc];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) old[i][j][r] = nold[i][j][r];
  }
}

// ---------------------------------------------------------------------------
// Panel pairs (single-level plans): the two-sided update of panel a is
// deferred and merged with panel b's (the next 32 columns) into one rank-128
// pass over the trailing matrix.
//  1. after W_a: panel b's columns (every row of A22_a, the 32 columns at its
//     left edge, lower part + mirror) get panel a's update now (they are
//     panel b's QR input and its band diagonal block);
//  2. panel b's X is formed from the NOT yet updated trailing matrix,
//     X_raw = A_cur YT_b, and corrected:  X_b = X_raw - Y_a' P - W_a' Q,
//     P = W_a'^T YT_b, Q = Y_a'^T YT_b (a' = panel a's rows below panel b's
//     columns); M_b = M_raw - T_b^T (E1 P + E2 Q), E1 = Y_b^T Y_a',
//     E2 = Y_b^T W_a';
//  3. one syr2k over A22_b with (Y_a', W_a') and (Y_b, W_b).
// Per pair the trailing matrix is streamed 3x (two X passes, one update of
// 1.5x the bytes) instead of 4x.
// ---------------------------------------------------------------------------
// 1: A22[i][j] -= sum_l Y[i][l] W[j][l] + W[i][l] Y[j][l] for j < 32,
// i >= j, mirrored to A22[j][i]; 32 rows x 32 columns per workgroup.
__global__ __launch_bounds__(256) void panel_upd_kernel(double *__restrict__ A, int64_t lda, int m,
                                                        const double *__restrict__ Y,
                                                        const double *__restrict__ W) {
  __shared__ double yc[SB_B][SB_B + 1], wc[SB_B][SB_B + 1];  // rows 0..31: the columns' factors
  __shared__ double yr[SB_B][SB_B + 1], wr[SB_B][SB_B + 1];  // this block's 32 rows
  const int tid = threadIdx.x, i0 = blockIdx.x * SB_B;
  for (int e = tid; e < SB_B * SB_B; e += 256) {
    const int r = e >> 5, c = e & 31;
    yc[r][c] = Y[r * SB_B + c];
    wc[r][c] = W[r * SB_B + c];
    const int gi = min(i0 + r, m - 1);
    yr[r][c] = Y[int64_t(gi) * SB_B + c];
    wr[r][c] = W[int64_t(gi) * SB_B + c];
  }
  __syncthreads();
  const int j = tid & 31;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int il = (tid >> 5) + 8 * q, i = i0 + il;
    if (i >= m || i < j) continue;
    double v = 0.0;
#pragma unroll
    for (int l = 0; l < SB_B; ++l) v = fma(yr[il][l], wc[j][l], v);
#pragma unroll
    for (int l = 0; l < SB_B; ++l) v = fma(wr[il][l], yc[j][l], v);
    const double a = A[int64_t(i) * lda + j] - v;
    A[int64_t(i) * lda + j] = a;
    if (i != j) A[int64_t(j) * lda + i] = a;
  }
}

// 2a: per block of PR rows r of panel b's trailing rows (Ya = Y_a', Wa =
// W_a', Yb = Y_b, YTb = YT_b, m rows each, ld 32): partial sums of the four
// 32 x 32 products P = Wa^T YTb, Q = Ya^T YTb, E1 = Yb^T Ya, E2 = Yb^T Wa,
// to part[blk * 4096 + {0, 1024, 2048, 3072} + 32 l + c].
constexpr int PR = 128;
__global__ __launch_bounds__(256) void pair_part_kernel(const double *__restrict__ Ya,
                                                        const double *__restrict__ Wa,
                                                        const double *__restrict__ Yb,
                                                        const double *__restrict__ YTb, int m,
                                                        double *__restrict__ part) {
  __shared__ double sa[32][SB_B + 1], sw[32][SB_B + 1], sb[32][SB_B + 1], st[32][SB_B + 1];
  const int tid = threadIdx.x, r0 = blockIdx.x * PR;
  // thread: 16 outputs = product pr (tid >> 6), row l (tid & 31), columns c0 .. c0 + 15
  const int pr = tid >> 6, l = tid & 31, c0 = ((tid >> 5) & 1) * 16;
  double acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = 0.0;
  for (int rb = r0; rb < min(m, r0 + PR); rb += 32) {
    __syncthreads();
    for (int e = tid; e < 32 * SB_B; e += 256) {
      const int r = e >> 5, c = e & 31, gr = rb + r;
      const bool ok = gr < m;
      const int64_t o = int64_t(ok ? gr : 0) * SB_B + c;
      sa[r][c] = ok ? Ya[o] : 0.0;
      sw[r][c] = ok ? Wa[o] : 0.0;
      sb[r][c] = ok ? Yb[o] : 0.0;
      st[r][c] = ok ? YTb[o] : 0.0;
    }
    __syncthreads();
    // left factor column l, right factor columns c0..: sum over the 32 rows
    const double(*L)[SB_B + 1] = pr == 0 ? sw : pr == 1 ? sa : sb;
    const double(*R)[SB_B + 1] = pr <= 1 ? st : pr == 2 ? sa : sw;
    for (int r = 0; r < 32; ++r) {
      const double a = L[r][l];
#pragma unroll
      for (int c = 0; c < 16; ++c) acc[c] = fma(a, R[r][c0 + c], acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) part[size_t(blockIdx.x) * 4096 + pr * 1024 + l * 32 + c0 + c] = acc[c];
}

// 2b: one workgroup: the four products summed over the blocks in block order
// -> PQ[0..2047] = {P, Q}, PQ[2048..3071] = T^T (E1 P + E2 Q) (subtracted
// from M_raw by w_update2_kernel).
__global__ __launch_bounds__(1024) void pair_fin_kernel(const double *__restrict__ part, int nblk,
                                                        const double *__restrict__ T,
                                                        double *__restrict__ PQ) {
  __shared__ double S[4][SB_B][SB_B + 1], D[SB_B][SB_B + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < 4096; e += 1024) {
    double v = 0.0;
    for (int z = 0; z < nblk; ++z) v += part[size_t(z) * 4096 + e];
    S[e >> 10][(e >> 5) & 31][e & 31] = v;
    if (e < 2048) PQ[e] = v;
  }
  __syncthreads();
  {  // D = E1 P + E2 Q
    const int a = tid >> 5, c = tid & 31;
    double v = 0.0;
#pragma unroll 8
    for (int k = 0; k < SB_B; ++k) v = fma(S[2][a][k], S[0][k][c], v);
#pragma unroll 8
    for (int k = 0; k < SB_B; ++k) v = fma(S[3][a][k], S[1][k][c], v);
    D[a][c] = v;
  }
  __syncthreads();
  {  // T^T D (T upper triangular: column a of T has rows k <= a)
    const int a = tid >> 5, c = tid & 31;
    double v = 0.0;
    for (int k = 0; k <= a; ++k) v = fma(T[k * SB_B + a], D[k][c], v);
    PQ[2048 + a * SB_B + c] = v;
  }
}

// 2c: W_b = X_raw - Ya P - Wa Q - 1/2 Yb M_b in place over X (as
// w_update_kernel, two more 32-term products).
__global__ __launch_bounds__(256) void w_update2_kernel(const double *__restrict__ Yb,
                                                        double *__restrict__ X, int m,
                                                        const double *__restrict__ M,
                                                        const double *__restrict__ Ya,
                                                        const double *__restrict__ Wa,
                                                        const double *__restrict__ PQ) {
  __shared__ double2 Ms[SB_B][SB_B / 2], Ps[SB_B][SB_B / 2], Qs[SB_B][SB_B / 2];
  const int tid = threadIdx.x;
  const int r = blockIdx.x * WU_R + (tid >> 4), c2 = tid & 15;
  const int rc = min(r, m - 1);
  for (int e = tid; e < SB_B * SB_B / 2; e += 256) {
    const double2 mr = reinterpret_cast<const double2 *>(M)[e];
    const double2 td = reinterpret_cast<const double2 *>(PQ + 2048)[e];
    Ms[e >> 4][e & 15] = make_double2(mr.x - td.x, mr.y - td.y);  // M_b = M_raw - T^T D
    Ps[e >> 4][e & 15] = reinterpret_cast<const double2 *>(PQ)[e];
    Qs[e >> 4][e & 15] = reinterpret_cast<const double2 *>(PQ + 1024)[e];
  }
  const double2 x = reinterpret_cast<const double2 *>(X + int64_t(rc) * SB_B)[c2];
  __syncthreads();
  double v0 = 0.0, v1 = 0.0, u0 = 0.0, u1 = 0.0;
  for (int h = 0; h < SB_B; ++h) {
    const double yb = Yb[int64_t(rc) * SB_B + h], ya = Ya[int64_t(rc) * SB_B + h],
                 wa = Wa[int64_t(rc) * SB_B + h];
    const double2 mm = Ms[h][c2], pp = Ps[h][c2], qq = Qs[h][c2];
    v0 = fma(yb, mm.x, v0);
    v1 = fma(yb, mm.y, v1);
    u0 = fma(ya, pp.x, u0);
    u1 = fma(ya, pp.y, u1);
    u0 = fma(wa, qq.x, u0);
    u1 = fma(wa, qq.y, u1);
  }
  if (r < m)
    reinterpret_cast<double2 *>(X + int64_t(r) * SB_B)[c2] =
        make_double2((x.x - u0) - 0.5 * v0, (x.y - u1) - 0.5 * v1);
}

// dst[s][:] = src[map(s)][:]
// Both passes of sym_scatter_kernel in one launch: blockIdx.z = pass, each
// with its own (x, y) extent; the passes write disjoint entries.
__global__ void sym_scatter2_kernel(double *__restrict__ A, int64_t lda, int m, int nS, RowMap mp,
                                    const double *__restrict__ U, int gx0, int gx1, int gy1) {
  if (blockIdx.z == 0) {
    const int s = blockIdx.y;
    if (s >= nS || int(blockIdx.x) >= gx0) return;
    const int r = mp.fwd(s);
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < m; c += gx0 * blockDim.x) {
      const int t = mp.inv(c);
      double v = U[int64_t(s) * m + c];
      if (t >= 0) v = v + U[int64_t(t) * m + r];
      A[int64_t(r) * lda + c] -= v;
    }
  } else {
    if (int(blockIdx.x) >= gx1 || int(blockIdx.y) >= gy1) return;
    const int r = blockIdx.x * 64 + (threadIdx.x & 63);
    if (r >= m || mp.inv(r) >= 0) return;
    for (int t = blockIdx.y * 4 + (threadIdx.x >> 6); t < nS; t += gy1 * 4)
      A[int64_t(r) * lda + mp.fwd(t)] -= U[int64_t(t) * m + r];
  }
}

// X[S_s, :] -= 1/2 sum_a Y[s][a] M[z(s) * 32 + a][:]  (z(s) = chunk of level
// row s), in place through the row map: the level >= 1 W = X - Yd M / 2.
__global__ void xs_update_kernel(double *__restrict__ X, int w, int rows, int nc, RowMap mp,
                                 const double *__restrict__ Y, const double *__restrict__ M) {
  const int s = blockIdx.y, col = blockIdx.x * 64 + threadIdx.x;
  if (col >= w) return;
  const int z = min(s / SB_C, nc - 1);
  const double *yr = Y + int64_t(s) * SB_B;
  const double *mc = M + int64_t(z) * SB_B * w + col;
  double acc = 0.0;
#pragma unroll
  for (int a = 0; a < SB_B; ++a) acc += yr[a] * mc[int64_t(a) * w];
  X[int64_t(mp.fwd(s)) * w + col] += -0.5 * acc;
}

__global__ void gather_rows_kernel(const double *__restrict__ src, int64_t lds, int ncols, int nrows,
                                   RowMap mp, double *__restrict__ dst) {
  const int s = blockIdx.y;
  const int r = mp.fwd(s);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < ncols; c += gridDim.x * blockDim.x)
    dst[int64_t(s) * ncols + c] = src[int64_t(r) * lds + c];
}

// dst[map(s)][:] = src[s][:]
__global__ void scatter_rows_kernel(const double *__restrict__ src, int ncols, int nrows, RowMap mp,
                                    double *__restrict__ dst, int64_t ldd) {
  const int s = blockIdx.y;
  const int r = mp.fwd(s);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < ncols; c += gridDim.x * blockDim.x)
    dst[int64_t(r) * ldd + c] = src[int64_t(s) * ncols + c];
}

// A22 -= Ye U^T... in scattered form: U (nS x m) = Y_l W^T.
//   z = 0: rows map(s): A[map(s)][c] -= U[s][c] + (c in set ? U[t(c)][map(s)] : 0)
//   z = 1: rows r not in set, columns map(t): A[r][map(t)] -= U[t][r]
__global__ void sym_scatter_kernel(double *__restrict__ A, int64_t lda, int m, int nS, RowMap mp,
                                   const double *__restrict__ U, int pass) {
  if (pass == 0) {
    const int s = blockIdx.y;
    if (s >= nS) return;
    const int r = mp.fwd(s);
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < m; c += gridDim.x * blockDim.x) {
      const int t = mp.inv(c);
      double v = U[int64_t(s) * m + c];
      if (t >= 0) v = v + U[int64_t(t) * m + r];
      A[int64_t(r) * lda + c] -= v;
    }
  } else {
    // rows r = blockIdx.x * 64 + (tid & 63), columns t = blockIdx.y*4 + (tid >> 6) ...
    const int r = blockIdx.x * 64 + (threadIdx.x & 63);
    if (r >= m || mp.inv(r) >= 0) return;
    for (int t = blockIdx.y * 4 + (threadIdx.x >> 6); t < nS; t += gridDim.y * 4)
      A[int64_t(r) * lda + mp.fwd(t)] -= U[int64_t(t) * m + r];
  }
}

// A[r0+i][p+l] = [R; 0] and the transpose (i < m, l < 32).
__global__ void write_panel_kernel(double *__restrict__ A, int64_t lda, int p, int r0, int m,
                                   const double *__restrict__ R) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * SB_B) return;
  const int i = idx >> 5, l = idx & 31;
  const double v = (i < SB_B) ? R[i * SB_B + l] : 0.0;
  A[int64_t(r0 + i) * lda + p + l] = v;
  A[int64_t(p + l) * lda + r0 + i] = v;
}


}  // namespace

namespace tg {

constexpr int NPQ_STAT = 8;

#define TG_CHK(x)                     \
  do {                                \
    hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return e_;  \
  } while (0)

// Side stream + events for the TSQR levels >= 1 (created once per device).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t ev0[2] = {nullptr, nullptr}, ev1[2] = {nullptr, nullptr}, evj = nullptr;
};
static hipError_t side_stream(SideStream *&out) {
  static SideStream ss[64];
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  SideStream &x = ss[dev & 63];
  if (!x.s) {
    if ((e = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking)) != hipSuccess) return e;
    for (int i = 0; i < 2; ++i) {
      if ((e = hipEventCreateWithFlags(&x.ev0[i], hipEventDisableTiming)) != hipSuccess) return e;
      if ((e = hipEventCreateWithFlags(&x.ev1[i], hipEventDisableTiming)) != hipSuccess) return e;
    }
    if ((e = hipEventCreateWithFlags(&x.evj, hipEventDisableTiming)) != hipSuccess) return e;
  }
  out = &x;
  return hipSuccess;
}

// Fork work onto the side stream after everything queued on st so far, and
// join it back (tg_eigh_vectors_range: the Q2 T factors beside inverse
// iteration)
hipError_t side_fork(hipStream_t st, hipStream_t *side) {
  SideStream *ss = nullptr;
  TG_CHK(side_stream(ss));
  TG_CHK(hipEventRecord(ss->evj, st));
  TG_CHK(hipStreamWaitEvent(ss->s, ss->evj, 0));
  *side = ss->s;
  return hipSuccess;
}
hipError_t side_join(hipStream_t st) {
  SideStream *ss = nullptr;
  TG_CHK(side_stream(ss));
  TG_CHK(hipEventRecord(ss->evj, ss->s));
  TG_CHK(hipStreamWaitEvent(st, ss->evj, 0));
  return hipSuccess;
}

// One compact-WY block per panel (pqr.hip): panel QR, X = A22 YT, M, update.
// (Measured and removed in round 3's clean-up, DESIGN.md §5: a look-ahead
// with the next panel's QR on a side stream, +5 ms -- the QR's workgroups need
// a whole CU's LDS and wait for the trailing update to drain; the same on
// CU-masked streams, update kernels 1.3-2x slower; A22 kept as its lower
// triangle, X 27 -> 35 us for syr2k 38 -> 35 us.  Round 5: the look-ahead
// with the update's workgroups kept off the QR's XCD (b % 8 != 0, dense
// tile index) does overlap the two, but the next panel's column update and
// the cross-stream waits cost what the overlap saves: 59.11 vs 59.11 ms at
// n = 4096, +2 ms at 12,288.)
// X = A22 YT and M = T^T Y^T X in one launch (row blocks of A22)
static int xm_nbc(int m) {
  const char *fx = getenv("TG_XM_NBC");  // development switch (1 | 2), read per call
  return fx ? (atoi(fx) == 2 ? 2 : 1) : (m >= XM_WIDE ? 2 : 1);
}
// X / M workgroups that fit the device at once (occupancy x CUs, cached)
template <int NBC>
static int xm_resident() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cached[dev] == 0) {
    int ncu = 0, occ = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, xm_kernel<NBC>, 64 * XW, 0) !=
        hipSuccess)
      occ = 0;
    cached[dev] = std::max(0, ncu) * std::max(0, occ);
    if (cached[dev] == 0) cached[dev] = -1;
  }
  return std::max(0, cached[dev]);
}
// Ya / Wa (panel pairs, NBC = 2 only): also form the pair products into PQ.
// epoch > 0: fuse W = X - Y M / 2 into the launch when every workgroup fits
// the device at once (they wait for M); returns *fused (false: the caller
// runs w_update_kernel)
// K splits per column block (TG_XM_KSPLIT=s forces s, 1 = none, 0 = the
// default; read per call): the column-block grid alone leaves CUs idle once m / (16 NBC) is
// below the device's workgroup slots, and at m / 32 = 192 .. 384 blocks of
// the HBM-resident NBC = 2 launches it puts two blocks on some CUs and one on
// others.  Splitting K brings the grid to about three rounds of 512
// workgroups (two per CU on 256 CUs) -- a function of m only, so the
// results do not depend on the device.
// Measured (profiles/r06/env_ab_*_ksplit.log): n = 12,288 392.8 -> 389.7 ms
// (the NBC = 2 launches 244 -> 226 us), but n = 4096 56.96 -> 58.30 ms (the
// 16-column launches are MALL-resident and their extra partial hand-off
// costs more than the balance gains), so only the 32-column form splits.
static int xm_ksplit(int m, int G, int nbc) {
  const char *e = getenv("TG_XM_KSPLIT");  // 0 / unset: the default below
  int S = (e && atoi(e) > 0) ? atoi(e) : (nbc == 1 || G >= 1536 ? 1 : cdiv(1536, G));
  S = std::max(1, std::min(8, S));
  while (S > 1 && cdiv(m, S) < 4 * 32) --S;  // at least 128 rows per split
  return S;
}
static hipError_t launch_xm(hipStream_t st, double *A22, int lda, int m, const double *YT,
                            const double *Yp, const double *Tp, double *X, const SbBufs &b,
                            int n, const double *Ya = nullptr, const double *Wa = nullptr,
                            double *PQ = nullptr, unsigned epoch = 0, bool *fused = nullptr) {
  const int nbc = xm_nbc(m);
  if (Ya && nbc != 2) return hipErrorInvalidValue;
  const int G = cdiv(m, XR * nbc), np = Ya ? 5 : 1;
  const int S = xm_ksplit(m, G, nbc), kc = cdiv(cdiv(m, S), 32) * 32;
  unsigned *mflag = b.xm_tick + xm_mflag_off(n);
  const char *xs = getenv("TG_XM_ASM");  // development switch: 0 = compiler-scheduled loads
  const int asm_loads = !(xs && xs[0] == '0');
  // TG_XM_FUSE_W=1 (development switch, per call): W inside the launch.  Measured
  // 57.13 vs 56.82 ms per factorisation at n = 4096 and equal at 12,288
  // (profiles/r06/env_ab_*.log): the wait for M costs what the separate
  // w_update_kernel did, so the default keeps the separate kernel.
  const char *fw = getenv("TG_XM_FUSE_W");
  // (NBC = 1 only: at two workgroups per CU the fused tail spills xm_kernel<2>.
  // Half the resident capacity, so that two processes sharing the device --
  // the multi-rank tests -- can both have every workgroup of a launch
  // resident at once: the waiting workgroups never block the ones that
  // would publish M.)
  const bool fuse = epoch > 0 && !Ya && nbc == 1 && (fw && fw[0] == '1') &&
                    2 * G * S <= xm_resident<1>();
  if (fused) *fused = fuse;
  static const unsigned long long tmo_ticks = spin_timeout_ticks("TG_XM_TIMEOUT_TICKS");
  XmArgs xa{A22, int64_t(lda), m, YT, Yp, Tp, X, b.U, b.U + size_t(G) * np * 1024, b.M,
            b.xm_tick, asm_loads, Ya, Wa, PQ, fuse ? 1 : 0,
            mflag, epoch, b.pq_ctl, tmo_ticks, S, kc, b.xm_xpart, b.xm_tick + xm_cbt_off(n)};
  if (nbc == 2) hipLaunchKernelGGL(xm_kernel<2>, dim3(G * S), dim3(64 * XW), 0, st, xa);
  else hipLaunchKernelGGL(xm_kernel<1>, dim3(G * S), dim3(64 * XW), 0, st, xa);
  return hipGetLastError();
}

// Panel pairs (see panel_upd_kernel) for panels whose partner has at least
// PAIR_MIN trailing rows (TG_SB_PAIR=1: every panel with a partner of >= 256
// rows, 0: none; read per call); the workspace's X holds n x ncmax*32
// doubles, so two m x 32 slabs fit once n >= 2 SB_C.  The merged rank-128
// update streams the HBM-resident trailing matrix once per two panels; the
// pair's correction products run on a side stream beside X_raw.  Measured
// (tools/solve_time.py): n = 12,288 509.5 vs 521.8 ms, n = 28,672 3.18 vs
// 3.47 s, but n = 4096 64.6 vs 61.4 ms (MALL-resident trailing matrices: the
// corrections' reductions cost more than the pass they save), hence the
// 6144-row default.
constexpr int PAIR_MIN_ALL = 256, PAIR_MIN = 6144;

// One compact-WY block per panel (pqr.hip): panel QR, X = A22 YT, M, update.
// (Measured and removed in round 3's clean-up, DESIGN.md §5: a look-ahead
// with the next panel's QR on a side stream, +5 ms -- the QR's workgroups need
// a whole CU's LDS and wait for the trailing update to drain; the same on
// CU-masked streams, update kernels 1.3-2x slower; A22 kept as its lower
// triangle, X 27 -> 35 us for syr2k 38 -> 35 us.  Round 5: the look-ahead
// with the update's workgroups kept off the QR's XCD (b % 8 != 0, dense
// tile index) does overlap the two, but the next panel's column update and
// the cross-stream waits cost what the overlap saves: 59.11 vs 59.11 ms at
// n = 4096, +2 ms at 12,288.)
static hipError_t sy2sb_single(hipStream_t st, double *A, int lda, int n, const SbPlan &pl,
                               const SbBufs &b) {
  TG_CHK(hipMemsetAsync(b.pq_ctl, 0, sizeof(unsigned) * pq_ctl_words(n), st));
  TG_CHK(hipMemsetAsync(b.xm_tick, 0, sizeof(unsigned) * xm_tick_words(n), st));
  const int np = int(pl.panels.size());
  const char *pe = getenv("TG_SB_PAIR");
  const bool pairs = !(pe && pe[0] == '0') && pl.ncmax >= 2;
  const int pair_min = (pe && pe[0] == '1') ? PAIR_MIN_ALL : PAIR_MIN;
  // TG_SYR2K_PERSIST=0: one tile per workgroup (development switch, per call)
  const char *ps = getenv("TG_SYR2K_PERSIST");
  const bool persist = !(ps && ps[0] == '0');
  const XcdInfo xi = xcd_info();
  const int ncu = std::max(1, xi.xcds * xi.cus_per_xcd);
  SideStream *ss = nullptr;
  // TG_SB_PAIR_SIDE=1: the pair products by pair_part / pair_fin on a side
  // stream even where the X / M kernel can form them (development switch)
  const char *psd = getenv("TG_SB_PAIR_SIDE");
  const bool pair_side = psd && psd[0] == '1';
  double *Xa = b.X, *Xb = b.X + size_t(n) * SB_B;
  for (int pi = 0; pi < np; ++pi) {
    const SbPanel &P = pl.panels[pi];
    const int m = P.m, r0 = P.r0;
    double *A22 = A + int64_t(r0) * lda + r0;
    double *Yp = b.Y + P.L[0].yoff, *Tp = b.T + P.L[0].toff;
    TG_CHK(panel_qr(st, A, lda, P.p, P.r0, P.m, Yp, b.YT, Tp, b.pq_part, b.pq_bc,
                    b.pq_ctl + 4 + 4 * pi, b.pq_ctl));
    const bool pair = pairs && pi + 1 < np && pl.panels[pi + 1].m >= pair_min;
    // W = X - Y M / 2 in place: inside the X / M launch where it can be
    // (panel a of a pair needs M only through W as well)
    bool fused = false;
    TG_CHK(launch_xm(st, A22, lda, m, b.YT, Yp, Tp, Xa, b, n, nullptr, nullptr, nullptr,
                     unsigned(pi + 1), &fused));
    if (!fused) {
      hipLaunchKernelGGL(w_update_kernel, dim3(cdiv(m, WU_R)), dim3(256), 0, st, Yp, Xa, m, b.M);
      TG_CHK(hipGetLastError());
    }
    if (!pair) {  // A22 -= Y W^T + W Y^T
      const int nt = cdiv(m, WT), tiles = nt * (nt + 1) / 2;
      auto tok = prof_begin(st, PROF_SBUPD, 12.0 * double(m) * m, 64.0 * double(m) * m);
      if (persist)
        hipLaunchKernelGGL(syr2k_wp_kernel<1>, dim3(std::min(tiles, 2 * ncu)), dim3(256), 0, st,
                           A22, int64_t(lda), m, YW2{{Yp, nullptr}, {Xa, nullptr}}, tiles);
      else
        hipLaunchKernelGGL(syr2k_w_kernel<1>, dim3(tiles), dim3(256), 0, st, A22, int64_t(lda), m,
                           YW2{{Yp, nullptr}, {Xa, nullptr}});
      prof_end(st, tok);
      TG_CHK(hipGetLastError());
      continue;
    }
    // panel b = pi + 1: its columns get panel a's update now
    hipLaunchKernelGGL(panel_upd_kernel, dim3(cdiv(m, SB_B)), dim3(256), 0, st, A22,
                       int64_t(lda), m, Yp, Xa);
    TG_CHK(hipGetLastError());
    ++pi;
    const SbPanel &Q = pl.panels[pi];
    const int mb = Q.m;
    double *A22b = A + int64_t(Q.r0) * lda + Q.r0;
    double *Yb = b.Y + Q.L[0].yoff, *Tb = b.T + Q.L[0].toff;
    const double *Ya = Yp + SB_B * SB_B, *Wa = Xa + SB_B * SB_B;  // panel a's rows >= Q.r0
    TG_CHK(panel_qr(st, A, lda, Q.p, Q.r0, Q.m, Yb, b.YT, Tb, b.pq_part, b.pq_bc,
                    b.pq_ctl + 4 + 4 * pi, b.pq_ctl));
    if (xm_nbc(mb) == 2 && !pair_side) {
      // X_raw, M_raw and the corrections' products in one launch
      TG_CHK(launch_xm(st, A22b, lda, mb, b.YT, Yb, Tb, Xb, b, n, Ya, Wa, b.G));
    } else {
      // the corrections' products depend only on panel b's QR and panel a's
      // Y / W: a side stream forms them while X_raw streams the matrix
      const int nblk = cdiv(mb, PR);
      if (!ss) TG_CHK(side_stream(ss));
      TG_CHK(hipEventRecord(ss->ev0[0], st));
      TG_CHK(hipStreamWaitEvent(ss->s, ss->ev0[0], 0));
      hipLaunchKernelGGL(pair_part_kernel, dim3(nblk), dim3(256), 0, ss->s, Ya, Wa, Yb, b.YT, mb,
                         b.Gr);
      TG_CHK(hipGetLastError());
      hipLaunchKernelGGL(pair_fin_kernel, dim3(1), dim3(1024), 0, ss->s, b.Gr, nblk, Tb, b.G);
      TG_CHK(hipGetLastError());
      TG_CHK(hipEventRecord(ss->ev1[0], ss->s));
      TG_CHK(launch_xm(st, A22b, lda, mb, b.YT, Yb, Tb, Xb, b, n));  // X_raw, M_raw
      TG_CHK(hipStreamWaitEvent(st, ss->ev1[0], 0));
    }
    hipLaunchKernelGGL(w_update2_kernel, dim3(cdiv(mb, WU_R)), dim3(256), 0, st, Yb, Xb, mb, b.M,
                       Ya, Wa, b.G);
    TG_CHK(hipGetLastError());
    const int nt = cdiv(mb, WT);
    auto tok = prof_begin(st, PROF_SBUPD, 12.0 * double(mb) * mb, 128.0 * double(mb) * mb);
    const int tiles = nt * (nt + 1) / 2;
    if (persist)
      hipLaunchKernelGGL(syr2k_wp_kernel<2>, dim3(std::min(tiles, 2 * ncu)), dim3(256), 0, st,
                         A22b, int64_t(lda), mb, YW2{{Ya, Yb}, {Wa, Xb}}, tiles);
    else
      hipLaunchKernelGGL(syr2k_w_kernel<2>, dim3(tiles), dim3(256), 0, st, A22b, int64_t(lda), mb,
                         YW2{{Ya, Yb}, {Wa, Xb}});
    prof_end(st, tok);
    TG_CHK(hipGetLastError());
  }
  return hipSuccess;
}

hipError_t sy2sb_timed_out(hipStream_t st, const SbPlan &pl, const SbBufs &b, bool *tmo) {
  *tmo = false;
  if (!pl.single || pl.panels.empty()) return hipSuccess;
  unsigned h = 0;
  hipError_t e = hipMemcpyAsync(&h, b.pq_ctl, sizeof(unsigned), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  *tmo = h != 0u;
  if (getenv("TG_PQR_STATS")) {
    std::vector<unsigned> c(4 + 4 * pl.panels.size());
    (void)hipMemcpy(c.data(), b.pq_ctl, sizeof(unsigned) * c.size(), hipMemcpyDeviceToHost);
    int hist[4][NPQ_STAT] = {};
    for (size_t i = 0; i < pl.panels.size(); ++i) {
      const unsigned v = c[4 + 4 * i + 1];
      hist[std::min(3u, v / 16)][std::min(unsigned(NPQ_STAT - 1), v % 16)]++;
    }
    fprintf(stderr, "pqr: %zu panels; accept after 2/3/4 passes: %d/%d/%d; fallback: %d\n",
            pl.panels.size(), hist[2][2], hist[2][3], hist[2][4],
            hist[3][0] + hist[3][1] + hist[3][2] + hist[3][3] + hist[3][4]);
  }
  return e;
}

hipError_t sy2sb(hipStream_t st, double *A, int lda, int n, const SbPlan &pl, const SbBufs &b) {
  if (pl.single) return sy2sb_single(st, A, lda, n, pl, b);
  SideStream *ss = nullptr;
  TG_CHK(side_stream(ss));
  int pi = 0;
  for (const SbPanel &P : pl.panels) {
    const int m = P.m, r0 = P.r0;
    double *A22 = A + int64_t(r0) * lda + r0;
    RowMap mp{};
    for (int l = 0; l < P.nl; ++l) mp.nc[l] = P.L[l].nc;
    // level-0 QR on the main stream; levels >= 1 (QR of the stacked R's) on
    // the side stream, overlapping level 0's two-sided update.
    TG_CHK(launch_qr(st, A + int64_t(r0) * lda + P.p, lda, P.L[0].nc, m, b.Y + P.L[0].yoff,
                     b.T + P.L[0].toff, b.R[0], b.YT));
    const int ph = pi & 1;
    if (P.nl > 1) {
      TG_CHK(hipEventRecord(ss->ev0[ph], st));
      TG_CHK(hipStreamWaitEvent(ss->s, ss->ev0[ph], 0));
      for (int l = 1; l < P.nl; ++l) {
        const SbLevel &L = P.L[l];
        TG_CHK(launch_qr(ss->s, b.R[(l - 1) & 1], SB_B, L.nc, L.rows, b.Y + L.yoff, b.T + L.toff,
                         b.R[l & 1], b.YTl[l]));
      }
      TG_CHK(hipEventRecord(ss->ev1[ph], ss->s));
      // R (in R[1] when nl is even) -> the panel's band block, off the main
      // stream's critical path: it writes A outside every later A22 and
      // outside the next panels' columns; joined after the last panel
      if (((P.nl - 1) & 1) == 1) {
        hipLaunchKernelGGL(write_panel_kernel, dim3(cdiv(m * SB_B, 256)), dim3(256), 0, ss->s, A,
                           int64_t(lda), P.p, r0, m, b.R[1]);
        TG_CHK(hipGetLastError());
      }
    }
    for (int l = 0; l < P.nl; ++l) {
      const SbLevel &L = P.L[l];
      double *Yl = b.Y + L.yoff, *Tl = b.T + L.toff;
      const int nc = L.nc, rows = L.rows, w = nc * SB_B;
      mp.lv = l;
      if (l == 0) {
        // X = A22 blockdiag(YT)   (m x w)
        ChunkSpec cx{SB_C, nc, m, 1, 0, SB_B, 0, 0, SB_B, m, SB_B, -1};
        TG_CHK(dgemm_chunked(st, false, false, cx, 1.0, A22, lda, b.YT, SB_B, 0.0, b.X, w));
        // M = Td^T Yd^T X  (w x w)
        hipLaunchKernelGGL((ytz_kernel<0, false>), dim3(nc, nc), dim3(512), 0, st, Yl, Tl, b.X,
                           int64_t(w), w, SB_C, nc, m, mp, b.M, int64_t(w));
        TG_CHK(hipGetLastError());
        const int nt = cdiv(m, S2T);
        // HBM: lower tiles of A22 read, both triangles written (1.5 m^2 doubles)
        auto tok = prof_begin(st, PROF_SBUPD, 12.0 * double(m) * m, 96.0 * double(m) * m);
        hipLaunchKernelGGL(syr2k_bs_kernel, dim3(nt * (nt + 1) / 2), dim3(256), 0, st, A22,
                           int64_t(lda), m, SB_C, nc, Yl, b.X, int64_t(w), b.M, int64_t(w));
        prof_end(st, tok);
        TG_CHK(hipGetLastError());
        if (P.nl > 1) TG_CHK(hipStreamWaitEvent(st, ss->ev1[ph], 0));
      } else {
        double *YTl = b.YTl[l];
        // X = A22[S, :]^T blockdiag(YT)   (m x w)
        if (nc == 1) {
          // one chunk (w = 32): the rows S are 32-row blocks of A22 at a
          // fixed stride, so X = sum_z A22[block z, :]^T YT[32z : 32z + 32, :]
          // is one chunked GEMM straight from A22 (no gather; nz x 64 output
          // tiles instead of m/64) and a sum of the nz partials (scratch: U,
          // which this level fills only later; nz * 32 * m <= ncmax * 32 * n)
          int stride = SB_C;
          for (int q = 1; q < l; ++q) stride *= SB_C / SB_B;
          const int nz = rows / SB_B;
          ChunkSpec cz{SB_B, nz, rows, int64_t(stride / SB_B) * lda, 0, SB_B, 0, 0,
                       int64_t(m) * SB_B, m, SB_B, SB_B};
          TG_CHK(dgemm_chunked(st, true, false, cz, 1.0, A22, lda, YTl, SB_B, 0.0, b.U, SB_B));
          TG_CHK(sum_partials(st, b.U, nz, m, SB_B, 1.0, 0.0, b.X, w));
        } else {
          // Gr = A22[S, :]  (rows x m)
          hipLaunchKernelGGL(gather_rows_kernel, dim3(cdiv(m, 256), rows), dim3(256), 0, st, A22,
                             int64_t(lda), m, rows, mp, b.Gr);
          TG_CHK(hipGetLastError());
          ChunkSpec cx{SB_C, nc, rows, m, 0, SB_B, 0, 0, SB_B, m, SB_B, -1};
          TG_CHK(dgemm_chunked(st, true, false, cx, 1.0, b.Gr, m, YTl, SB_B, 0.0, b.X, w));
        }
        // M = T^T Y^T X[S, :]  (the rows S of X read through the row map)
        hipLaunchKernelGGL((ytz_kernel<0, true>), dim3(nc, nc), dim3(512), 0, st, Yl, Tl, b.X,
                           int64_t(w), w, SB_C, nc, rows, mp, b.M, int64_t(w));
        TG_CHK(hipGetLastError());
        // W = X - 1/2 Yd M on the rows S, in place
        hipLaunchKernelGGL(xs_update_kernel, dim3(cdiv(w, 64), rows), dim3(64), 0, st, b.X, w,
                           rows, nc, mp, Yl, b.M);
        TG_CHK(hipGetLastError());
        // U = Y_l W^T  (rows x m)
        ChunkSpec cu{SB_C, nc, rows, SB_B, 0, 0, SB_B, m, 0, -1, m, SB_B};
        TG_CHK(dgemm_chunked(st, false, true, cu, 1.0, Yl, SB_B, b.X, w, 0.0, b.U, m));
        // A22[S, :] and A22[:, S] -= U, U^T in one launch (disjoint entries)
        {
          const int gx0 = cdiv(m, 256), gx1 = cdiv(m, 64), gy1 = std::min(64, cdiv(rows, 4));
          hipLaunchKernelGGL(sym_scatter2_kernel, dim3(std::max(gx0, gx1), std::max(rows, gy1), 2),
                             dim3(256), 0, st, A22, int64_t(lda), m, rows, mp, b.U, gx0, gx1, gy1);
          TG_CHK(hipGetLastError());
        }
      }
    }
    if (((P.nl - 1) & 1) == 0) {
      hipLaunchKernelGGL(write_panel_kernel, dim3(cdiv(m * SB_B, 256)), dim3(256), 0, st, A,
                         int64_t(lda), P.p, r0, m, b.R[(P.nl - 1) & 1]);
      TG_CHK(hipGetLastError());
    }
    ++pi;
  }
  TG_CHK(hipEventRecord(ss->evj, ss->s));  // side-stream panel writes done
  TG_CHK(hipStreamWaitEvent(st, ss->evj, 0));
  return hipSuccess;
}

hipError_t sb_apply_q1(hipStream_t st, int n, double *Z, int k, const SbPlan &pl,
                       const SbBufs &b) {
  (void)n;
  if (pl.single) {
    // Z[r0:, :] -= Y (T (Y^T Z[r0:, :])) per panel, last panel first
    for (auto it = pl.panels.rbegin(); it != pl.panels.rend(); ++it) {
      const SbPanel &P = *it;
      double *Zs = Z + int64_t(P.r0) * k;
      const double *Yp = b.Y + P.L[0].yoff, *Tp = b.T + P.L[0].toff;
      auto tok = prof_begin(st, PROF_Q1, 24.0 * double(P.m) * k, 4.0 * double(P.m) * SB_B * k);
      const int splits = std::max(1, std::min(pl.ncmax, P.m / SB_C));
      TG_CHK(dgemm_splitk(st, true, false, SB_B, k, P.m, 1.0, Yp, SB_B, Zs, k, 0.0, b.P, k, splits,
                          b.Zg));
      TG_CHK(dgemm(st, false, false, SB_B, k, SB_B, 1.0, Tp, SB_B, b.P, k, 0.0, b.Mz, k));
      TG_CHK(dgemm(st, false, false, P.m, k, SB_B, -1.0, Yp, SB_B, b.Mz, k, 1.0, Zs, k));
      prof_end(st, tok);
    }
    return hipSuccess;
  }
  for (auto it = pl.panels.rbegin(); it != pl.panels.rend(); ++it) {
    const SbPanel &P = *it;
    double *Zs = Z + int64_t(P.r0) * k;
    RowMap mp{};
    for (int l = 0; l < P.nl; ++l) mp.nc[l] = P.L[l].nc;
    for (int l = P.nl - 1; l >= 0; --l) {  // Q = D_0 E_1 E_2 ...: top level first
      const SbLevel &L = P.L[l];
      mp.lv = l;
      // HBM: read + write of the level's rows of Z
      auto tok = prof_begin(st, PROF_Q1, 16.0 * double(L.rows) * k, 4.0 * double(L.rows) * SB_B * k);
      if (l > 0)
        hipLaunchKernelGGL((ytz_kernel<1, true>), dim3(cdiv(k, SB_B), L.nc), dim3(512), 0, st,
                           b.Y + L.yoff, b.T + L.toff, Zs, int64_t(k), k, SB_C, L.nc, L.rows, mp,
                           nullptr, int64_t(0));
      else
        hipLaunchKernelGGL((ytz_kernel<1, false>), dim3(cdiv(k, SB_B), L.nc), dim3(512), 0, st,
                           b.Y + L.yoff, b.T + L.toff, Zs, int64_t(k), k, SB_C, L.nc, L.rows, mp,
                           nullptr, int64_t(0));
      prof_end(st, tok);
      TG_CHK(hipGetLastError());
    }
  }
  return hipSuccess;
}

}  // namespace tg
