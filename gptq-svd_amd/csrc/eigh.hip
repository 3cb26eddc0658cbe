// Symmetric eigensolver for the TruncGPTQ spectral factorisation (A2, A3).
//
// Replaces `L, V = torch.linalg.eigh(H_double)` + the descending flip and the
// rank rule of process_hessian_alt
// (/root/reference/src/TruncGPTQ/gptq_utils.py:92-110), which the reference
// runs through cuSOLVER syevd.  MI355X-native pipeline:
//
//   1. Householder tridiagonalisation A = Q T Q^T, blocked like LAPACK dlatrd
//      (panels of NB columns).  Per column: one row-parallel kernel computes
//      the reflector and y = A v (memory-bound, every CU streams rows of the
//      Infinity-Cache-resident trailing matrix), one kernel finishes the panel
//      column of W and updates the next column.  Cross-workgroup sums use the
//      deterministic last-arriver reduction (reduce.h).  Between panels the
//      trailing matrix takes the rank-2NB update A -= V W^T + W V^T on FP64
//      MFMA (gemm64.hip).
//   2. All eigenvalues of T by Sturm-count multisection: 16 lanes per
//      eigenvalue evaluate 16 shifts per round (interval shrinks 17x/round).
//   3. Eigenvectors of T for the k largest eigenvalues by inverse iteration
//      (tridiagonal LU with partial pivoting, 3 solves from a per-index
//      pseudo-random start); tight clusters are re-orthogonalised (MGS).
//   4. Back-transformation V = Q Z with compact-WY blocks of BT reflectors
//      (dlarft T factors, FP64 MFMA GEMMs, split-K for the V^T Z products).
#include <algorithm>
#include <vector>
#include <cfloat>
#include <cstdlib>
#include <cmath>
#include <type_traits>

#include "../../include/truncgptq.h"
#include "band.h"
#include "common.h"
#include "gemm64.h"
#include "reduce.h"

namespace {

constexpr int NB = 32;    // tridiagonalisation panel width
constexpr int NG = 256;   // workgroups of the symv kernel (16 waves each)
constexpr int SYT = 1024; // symv threads per workgroup
constexpr int BT = 64;    // back-transformation block of reflectors
constexpr int PST = 2 * NB + 2;  // partials stride
#ifndef TG_ML
#define TG_ML 16
#endif
constexpr int ML = TG_ML;  // multisection lanes per eigenvalue
// (ML+1)^ROUNDS > 2^57: the Gershgorin interval shrinks below one ulp
constexpr int ROUNDS = ML == 16 ? 14 : (ML == 32 ? 12 : 10);
static_assert(ML == 16 || ML == 32 || ML == 64, "ML");
// Shared first rounds (ML = 16, n >= GRID_MIN_N): Sturm counts of the first
// unreduced block [0, be[0]) at the 17^4 - 1 points of a uniform grid of the
// Gershgorin interval, computed once for all of that block's eigenvalues
// (each one's first four 17-sections would evaluate points of this grid);
// they then start from their grid cells and run ROUNDS - 4 rounds.  The first
// block is the one that matters: a rank-deficient H gives T = one block of
// about the rank followed by 1 x 1 blocks (n = 4096, k = 3058: [0, 3128) and
// 962 single rows).
constexpr int GRID_ROUNDS = ML == 16 ? 4 : 0;
constexpr int GRID_PTS = ML == 16 ? 17 * 17 * 17 * 17 - 1 : 1;
constexpr int GRID_MIN_N = 1024;
constexpr int SPLITK = 8;

struct Tri {
  double *V;     // n x n reflectors: V[r*n + j] = v_j[r] (0 above j+1, 1 at r = j+1)
  double *PT;    // 3 x NB x n  column-major panel [V^T; W^T; V^T] (coalesced, one K=2NB update)
  double *tau;   // n
  double *d;     // n   diagonal of T
  double *e;     // n   off-diagonal of T (e[i] couples i, i+1)
  double *acol;  // n   current updated column
  double *y;     // n   symv result
  double *part;  // PST x NG partial sums (transposed)
  double *red;   // PST reduced sums: [0] = |x|^2, [1..NB] = V^T v, [1+NB..2NB] = W^T v, [1+2NB] = v^T y
  double *Tf;    // nblk x BT x BT  block-reflector T factors
  double *Z;     // n x n  eigenvectors of T (column j), later of A
  double *lu;    // 3 x n x n  inverse-iteration U factors ([i][thread] layout)
  double *X1;    // BT x n
  double *X2;    // BT x n
  double *skp;   // split-K scratch
  double *scal;  // small scalars (norm of T)
  double *es;    // n   off-diagonal with negligible entries zeroed (block splits)
  double *wraw;  // n   eigenvalue of slot j (block-local order)
  int32_t *bs;   // n   start of the unreduced block containing position j
  int32_t *be;   // n   end (exclusive) of that block
  int32_t *slot; // n   slot of the j-th smallest eigenvalue
  unsigned *cnt; // reduction tickets
  int32_t *gcnt; // GRID_PTS  Sturm counts of T at the bisection grid points
  int32_t *cl;   // 2 + 4n  cluster lists: [0] small count, [1] big count, small (start, len)
                 //         pairs from 2, big pairs from 2 + 2n
};

template <class A>
void tri_layout(A &ar, int n, Tri *t) {
  Tri d{};
  Tri &q = t ? *t : d;
  const size_t nn = size_t(n) * n;
  const int nblk = tg::cdiv(n, BT);
  auto take = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<A, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  take(q.V, nn);
  take(q.PT, size_t(3) * NB * n);
  take(q.tau, n);
  take(q.d, n);
  take(q.e, n);
  take(q.acol, n);
  take(q.y, n);
  take(q.part, size_t(NG) * PST);
  take(q.red, PST);
  take(q.Tf, size_t(nblk) * BT * BT);
  take(q.Z, nn);
  take(q.lu, 3 * nn);
  take(q.X1, size_t(BT) * n);
  take(q.X2, size_t(BT) * n);
  take(q.skp, size_t(SPLITK) * BT * n);
  take(q.scal, 16);
  take(q.cnt, 16);
  take(q.es, n);
  take(q.wraw, n);
  take(q.bs, n);
  take(q.be, n);
  take(q.slot, n);
  take(q.gcnt, GRID_PTS);
  take(q.cl, 2 + 4 * size_t(n));
}

// ---------------------------------------------------------------------------
// 1. tridiagonalisation kernels
// ---------------------------------------------------------------------------

// Panel start at column i (no pending panel corrections): acol = A[i:, i]
// (= row i by symmetry), d[i], and |x|^2 of A[i+2:, i].
__global__ __launch_bounds__(256) void tri_start_kernel(const double *__restrict__ A, int lda,
                                                        int n, int i, Tri w) {
  __shared__ double scratch[8];
  __shared__ double vals[1];
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0;
  for (int r = i + gtid; r < n; r += gridDim.x * blockDim.x) {
    const double a = A[size_t(i) * lda + r];
    w.acol[r] = a;
    if (r == i) w.d[i] = a;
    if (r >= i + 2) s += a * a;
  }
  s = tg::block_sum(s, scratch);
  if (threadIdx.x == 0) vals[0] = s;
  __syncthreads();
  if (tg::publish_partials(vals, 1, w.part, w.cnt)) tg::sum_partials(w.part, 1, w.red, w.cnt);
}

// Reflector for column i + y = A[i+1:, i+1:] v + partial V^T v, W^T v, v^T y.
// One wave per row; lanes stream the row as 16-byte double2 loads, 8 in flight
// per lane.  v lives in LDS (n <= 16384) indexed by absolute column, zero
// below i+1; otherwise v_c = acol[c] * scal is formed on the fly.
template <bool VLDS>
__global__ __launch_bounds__(SYT) void tri_symv_kernel(const double *__restrict__ A, int lda, int n,
                                                       int i, int p, Tri w) {
  extern __shared__ double vsh[];
  __shared__ double wpart[SYT / 64][PST];
  __shared__ double vals[PST];
  const int t = i - p;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const double *VT = w.PT, *WT = w.PT + size_t(NB) * n;
  const int c_lo = (i + 1) & ~1;
  const bool vec = ((lda & 1) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const int len2 = (n - c_lo) >> 1;  // double2 count
  const int TW = gridDim.x * (SYT / 64);
  const int r_first = i + 1 + blockIdx.x * (SYT / 64) + wid;
  // row data does not depend on the reflector: put the first batch in flight now
  double2 pre[8];
  const bool have_pre = VLDS && vec && r_first < n;
  if (have_pre) {
    const double2 *r2 = reinterpret_cast<const double2 *>(A + size_t(r_first) * lda + c_lo);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = lane + u * 64;
      pre[u] = r2[c < len2 ? c : 0];
    }
  }
  // dlarfg (LAPACK): beta = -sign(alpha) * hypot(alpha, |x|), tau = (beta-alpha)/beta,
  // v = [1, x / (alpha - beta)]
  const double xn2 = w.red[0];
  const double alpha = w.acol[i + 1];
  double tau = 0.0, beta = alpha, scal = 0.0;
  if (xn2 > 0.0) {
    beta = -copysign(hypot(alpha, sqrt(xn2)), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
  }
  auto vval = [&](int c) -> double {
    return c < i + 1 ? 0.0 : (c == i + 1 ? 1.0 : w.acol[c] * scal);
  };
  if (VLDS)
    for (int c = c_lo + tid; c < n; c += blockDim.x) vsh[c] = vval(c);
  if (blockIdx.x == 0 && tid == 0) {
    w.tau[i] = tau;
    w.e[i] = beta;
  }
  for (int j = tid; j < (SYT / 64) * PST; j += blockDim.x) (&wpart[0][0])[j] = 0.0;
  __syncthreads();

  const int tail = (n - c_lo) & 1;
  double q1 = 0.0, q2 = 0.0, sv = 0.0;  // per-lane partials (lane l -> panel column l)
  for (int r = r_first; r < n; r += TW) {
    const double *row = A + size_t(r) * lda + c_lo;
    double a0 = 0.0, a1 = 0.0;
    if (VLDS && vec) {
      const double2 *r2 = reinterpret_cast<const double2 *>(row);
      const double2 *v2 = reinterpret_cast<const double2 *>(vsh + c_lo);
      int c = lane;
      if (r == r_first) {  // consume the prefetched batch
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int cc = lane + u * 64;
          if (cc < len2) {
            const double2 vv = v2[cc];
            a0 += pre[u].x * vv.x;
            a1 += pre[u].y * vv.y;
          }
        }
        c = lane + 8 * 64;
      }
      for (; c + 7 * 64 < len2; c += 8 * 64) {
        double2 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = r2[c + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double2 vv = v2[c + u * 64];
          a0 += x[u].x * vv.x;
          a1 += x[u].y * vv.y;
        }
      }
      for (; c < len2; c += 64) {
        const double2 x = r2[c], vv = v2[c];
        a0 += x.x * vv.x;
        a1 += x.y * vv.y;
      }
      if (tail && lane == 0) a0 += row[2 * len2] * vsh[c_lo + 2 * len2];
    } else {
      for (int c = lane; c < n - c_lo; c += 64) {
        const double vc = VLDS ? vsh[c_lo + c] : vval(c_lo + c);
        a0 += row[c] * vc;
      }
    }
    double dot = a0 + a1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
    const double vr = VLDS ? vsh[r] : vval(r);
    if (lane == 0) {
      w.y[r] = dot;
      w.V[size_t(r) * n + i] = vr;
      sv += vr * dot;
    }
    if (lane == 1) w.PT[size_t(t) * n + r] = vr;                   // V^T panel row t
    if (lane == 2) w.PT[size_t(2 * NB + t) * n + r] = vr;          // second copy
    if (lane < t) {
      q1 += VT[size_t(lane) * n + r] * vr;
      q2 += WT[size_t(lane) * n + r] * vr;
    }
  }
  // live values only: [q1 (t) | q2 (t) | v^T y]
  if (lane < t) {
    wpart[wid][lane] = q1;
    wpart[wid][t + lane] = q2;
  }
  if (lane == 0) wpart[wid][2 * t] = sv;
  __syncthreads();
  const int nv = 2 * t + 1;
  for (int j = tid; j < nv; j += blockDim.x) {
    double s = 0.0;
    for (int ww = 0; ww < SYT / 64; ++ww) s += wpart[ww][j];
    vals[j] = s;
  }
  __syncthreads();
  if (tg::publish_partials(vals, nv, w.part, w.cnt)) tg::sum_partials(w.part, nv, w.red + 1, w.cnt);
}

// W[:, t] = tau (y - V (W^T v) - W (V^T v)) + alpha2 v, then (do_next) update
// column i+1 with the panel's t+1 reflectors and reduce its |x|^2.  One thread
// per row; the column-major panel makes every load coalesced.
__global__ __launch_bounds__(64) void tri_fin_kernel(const double *__restrict__ A, int lda, int n,
                                                      int i, int p, int do_next, Tri w) {
  __shared__ double q1[NB], q2[NB], vrow[NB], wrow[NB];
  __shared__ double scratch[8];
  __shared__ double vals[1];
  const int t = i - p, j = i + 1;
  const int tid = threadIdx.x;
  const double *VT = w.PT;
  double *WT = w.PT + size_t(NB) * n;
  // the thread's first row: its panel rows do not depend on the reductions
  const int r_first = j + blockIdx.x * blockDim.x + tid;
  double vr_[NB], wr_[NB];
  {
    const int rr = r_first < n ? r_first : n - 1;
#pragma unroll
    for (int l = 0; l < NB; ++l) {
      vr_[l] = VT[size_t(l) * n + rr];
      wr_[l] = WT[size_t(l) * n + rr];
    }
  }
  const double tau = w.tau[i];
  if (tid < NB) {
    q1[tid] = tid < t ? w.red[1 + tid] : 0.0;
    q2[tid] = tid < t ? w.red[1 + t + tid] : 0.0;
    vrow[tid] = tid <= t ? VT[size_t(tid) * n + j] : 0.0;
    wrow[tid] = tid < t ? WT[size_t(tid) * n + j] : 0.0;
  }
  __syncthreads();
  double dq = 0.0;
  for (int l = 0; l < t; ++l) dq += q1[l] * q2[l];
  const double wtv = tau * (w.red[1 + 2 * t] - 2.0 * dq);
  const double alpha2 = -0.5 * tau * wtv;
  if (tid == 0) {
    double acc = w.y[j];
    for (int l = 0; l < t; ++l) acc -= vrow[l] * q2[l];
    for (int l = 0; l < t; ++l) acc -= wrow[l] * q1[l];
    wrow[t] = tau * acc + alpha2 * vrow[t];
  }
  __syncthreads();
  double s = 0.0;
  for (int r = r_first; r < n; r += gridDim.x * blockDim.x) {
    if (r != r_first) {
#pragma unroll
      for (int l = 0; l < NB; ++l) {
        vr_[l] = VT[size_t(l) * n + r];
        wr_[l] = WT[size_t(l) * n + r];
      }
    }
    double acc = w.y[r];
#pragma unroll
    for (int l = 0; l < NB; ++l) acc -= l < t ? vr_[l] * q2[l] : 0.0;
#pragma unroll
    for (int l = 0; l < NB; ++l) acc -= l < t ? wr_[l] * q1[l] : 0.0;
    double vt = 0.0;
#pragma unroll
    for (int l = 0; l < NB; ++l) vt = l == t ? vr_[l] : vt;
    const double wr = tau * acc + alpha2 * vt;
    WT[size_t(t) * n + r] = wr;
    if (do_next) {
      double a = A[size_t(j) * lda + r];
#pragma unroll
      for (int l = 0; l < NB; ++l) a -= l <= t ? vr_[l] * wrow[l] : 0.0;
#pragma unroll
      for (int l = 0; l < NB; ++l) a -= l < t ? wr_[l] * vrow[l] : 0.0;
      a -= wr * vrow[t];
      w.acol[r] = a;
      if (r == j) w.d[j] = a;
      if (r >= j + 2) s += a * a;
    }
  }
  if (!do_next) return;
  s = tg::block_sum(s, scratch);
  if (tid == 0) vals[0] = s;
  __syncthreads();
  if (tg::publish_partials(vals, 1, w.part, w.cnt)) tg::sum_partials(w.part, 1, w.red, w.cnt);
}

// ---------------------------------------------------------------------------
// 2. eigenvalues of T: Sturm-count multisection
// ---------------------------------------------------------------------------
// a / b with v_rcp_f64 + two Newton steps + one residual correction (the
// sweeps only need a backward-stable quotient, not IEEE rounding)
__device__ inline double fdiv(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  r = fma(fma(-b, r, 1.0), r, r);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}

// msk[lane] ? t : f as two v_cndmask_b32 (no control flow)
__device__ inline double vsel(uint64_t msk, double t, double f) {
  int lo, hi;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(__double2loint(f)), "v"(__double2loint(t)), "s"(msk));
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(__double2hiint(f)), "v"(__double2hiint(t)), "s"(msk));
  return __hiloint2double(hi, lo);
}

// Negative pivots of the LDL^T of T - x I (dlaebz's q recurrence).  The
// division e2/q uses the hardware reciprocal plus one Newton step (relative
// error ~2^-50, the count of a matrix a few ulps away) to keep the serial
// chain short; d and e2 are read 8 ahead of the chain.
__device__ inline int sturm_count(const double *__restrict__ d, const double *__restrict__ e2, int n,
                                  double x, double pivmin) {
  double q = d[0] - x;
  if (fabs(q) <= pivmin) q = -pivmin;
  int c = q < 0.0;
  for (int k0 = 1; k0 < n; k0 += 8) {
    double dv[8], ev[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = min(k0 + u, n - 1);
      dv[u] = d[k] - x;
      ev[u] = e2[k - 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (k0 + u < n) {
        double r = __builtin_amdgcn_rcp(q);
        r = fma(fma(-q, r, 1.0), r, r);
        q = fma(-ev[u], r, dv[u]);
        if (fabs(q) <= pivmin) q = -pivmin;
        c += q < 0.0;
      }
    }
  }
  return c;
}

// One step of the count over an LDS row v = {d[k], e2[k-1]}: the pivot q of
// row k-1 is counted (negative, or clamped to -pivmin when |q| <= pivmin: both
// are q <= pivmin) and replaced by row k's.  The reciprocal of q and its Newton
// step run unconditionally; a tiny q then selects the refined reciprocal of
// -pivmin instead (v_cndmask, no branch), so the clamp is off the serial chain.
__device__ inline void sturm_step(double &q, int &c, double2 v, double x, double pivmin,
                                  double rpivn) {
  const uint64_t tiny = __builtin_amdgcn_fcmp(fabs(q), pivmin, 5);  // OLE
  c += q <= pivmin;
  const double r0 = __builtin_amdgcn_rcp(q);
  const double r = vsel(tiny, rpivn, fma(fma(-q, r0, 1.0), r0, r0));
  q = fma(-v.y, r, v.x - x);
}
__device__ inline double rcp_pivmin(double pivmin) {  // 1/(-pivmin), one Newton step
  const double r = __builtin_amdgcn_rcp(-pivmin);
  return fma(fma(pivmin, r, 1.0), r, r);
}

// sturm_count over LDS rows de[k] = {d[k], e2[k-1]} (one 16-byte read per step).
__device__ inline int sturm_count_rows(const double2 *__restrict__ de, int n, double x,
                                       double pivmin) {
  const double rpivn = rcp_pivmin(pivmin);
  double q = de[0].x - x;
  int c = 0;
  int k0 = 1;
  for (; k0 + 8 <= n; k0 += 8) {
    double2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = de[k0 + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) sturm_step(q, c, v[u], x, pivmin, rpivn);
  }
  for (; k0 < n; ++k0) sturm_step(q, c, de[k0], x, pivmin, rpivn);
  return c + (q <= pivmin);
}

// Gershgorin bounds, ||T||_1 and pivmin: one workgroup.
__global__ void tri_bounds_kernel(const double *__restrict__ d, const double *__restrict__ e, int n,
                                  double *__restrict__ out /* gl gu tnorm pivmin */) {
  __shared__ double s_lo[256], s_hi[256], s_e2[256];
  double lo = INFINITY, hi = -INFINITY, me2 = 0.0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const double el = k > 0 ? fabs(e[k - 1]) : 0.0;
    const double er = k < n - 1 ? fabs(e[k]) : 0.0;
    lo = fmin(lo, d[k] - el - er);
    hi = fmax(hi, d[k] + el + er);
    if (k < n - 1) me2 = fmax(me2, e[k] * e[k]);
  }
  s_lo[threadIdx.x] = lo;
  s_hi[threadIdx.x] = hi;
  s_e2[threadIdx.x] = me2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (int(threadIdx.x) < off) {
      s_lo[threadIdx.x] = fmin(s_lo[threadIdx.x], s_lo[threadIdx.x + off]);
      s_hi[threadIdx.x] = fmax(s_hi[threadIdx.x], s_hi[threadIdx.x + off]);
      s_e2[threadIdx.x] = fmax(s_e2[threadIdx.x], s_e2[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double tnorm = fmax(fabs(s_lo[0]), fabs(s_hi[0]));
    const double pad = 2.0 * DBL_EPSILON * tnorm * n + 1e-300;
    out[0] = s_lo[0] - pad;
    out[1] = s_hi[0] + pad;
    out[2] = tnorm;
    out[3] = DBL_MIN * fmax(1.0, s_e2[0]);
  }
}

// Split T into unreduced blocks at |e_i| <= eps * ||T|| (LAPACK dstebz does the
// same with a relative test); one thread scans (n is small).  es = e with the
// split entries zeroed; bs/be = block of each position.
// One workgroup of 1024 threads: split flags in parallel, block starts by a
// prefix max and block ends by a suffix min over per-thread chunks.
__global__ __launch_bounds__(1024) void tri_split_kernel(const double *__restrict__ e, int n,
                                                         const double *__restrict__ bnd,
                                                         double *__restrict__ es,
                                                         int32_t *__restrict__ bs,
                                                         int32_t *__restrict__ be) {
  __shared__ int cmax[1024], cmin[1024];
  const double tol = DBL_EPSILON * bnd[2];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int ch = (n + nt - 1) / nt, c0 = tid * ch, c1 = min(n, c0 + ch);
  auto split = [&](int i) { return i == n - 1 || fabs(e[i]) <= tol; };
  int lmax = 0, lmin = n;  // last split + 1 in the chunk / first split + 1 in the chunk
  for (int i = c0; i < c1; ++i) {
    const bool sp = split(i);
    es[i] = sp ? 0.0 : e[i];
    if (sp) {
      lmax = i + 1;
      if (lmin == n) lmin = i + 1;
    }
  }
  cmax[tid] = lmax;
  cmin[tid] = lmin;
  __syncthreads();
  // exclusive prefix max / suffix min over chunks (Hillis-Steele, then shift)
  for (int off = 1; off < nt; off <<= 1) {
    const int a = tid >= off ? cmax[tid - off] : 0;
    const int b = tid + off < nt ? cmin[tid + off] : n;
    __syncthreads();
    cmax[tid] = max(cmax[tid], a);
    cmin[tid] = min(cmin[tid], b);
    __syncthreads();
  }
  int start = tid > 0 ? cmax[tid - 1] : 0;
  const int after = tid + 1 < nt ? cmin[tid + 1] : n;
  // ends: walk the chunk backwards
  int end = after;
  for (int i = c1 - 1; i >= c0; --i) {
    if (split(i)) end = i + 1;
    be[i] = end;
  }
  for (int i = c0; i < c1; ++i) {
    bs[i] = start;
    if (split(i)) start = i + 1;
  }
}

// Global ascending order of the block eigenvalues: rank(j) = #{i: v_i < v_j or
// (v_i == v_j and i < j)} -- deterministic, O(n^2) compares; 16 lanes per
// element each count a strided share of i (n/16 workgroups fill the chip).
constexpr int RS_G = 16;
__global__ __launch_bounds__(256) void rank_sort_kernel(const double *__restrict__ v, int n,
                                                        double *__restrict__ w_asc,
                                                        int32_t *__restrict__ slot) {
  extern __shared__ double sv[];
  const int tid = threadIdx.x, g = tid & (RS_G - 1);
  const int j = blockIdx.x * (256 / RS_G) + tid / RS_G;
  const double vj = j < n ? v[j] : 0.0;
  int r = 0;
  for (int c0 = 0; c0 < n; c0 += 2048) {
    const int cn = min(2048, n - c0);
    __syncthreads();
    for (int c = tid; c < cn; c += blockDim.x) sv[c] = v[c0 + c];
    __syncthreads();
    if (j < n)
      for (int c = g; c < cn; c += RS_G) {
        const double vi = sv[c];
        r += (vi < vj) || (vi == vj && c0 + c < j);
      }
  }
#pragma unroll
  for (int off = RS_G / 2; off > 0; off >>= 1) r += __shfl_xor(r, off, RS_G);
  if (j < n && g == 0) {
    w_asc[r] = vj;
    slot[r] = j;
  }
}

// Grid point g of the Gershgorin interval [lo, hi] (g = -1 / GRID_PTS: the ends).
__device__ inline double grid_x(double lo, double hi, int g) {
  return g < 0 ? lo : (g >= GRID_PTS ? hi : lo + (hi - lo) * double(g + 1) / double(GRID_PTS + 1));
}

// Sturm counts of the first block [0, be[0]) at every grid point, one thread
// each; rows staged through LDS.
constexpr int GRID_CH = 2048;
__global__ __launch_bounds__(256) void grid_count_kernel(const double *__restrict__ d,
                                                         const double *__restrict__ e2g, int n,
                                                         const double *__restrict__ bnd,
                                                         const int32_t *__restrict__ bev,
                                                         int32_t *__restrict__ gcnt) {
  __shared__ double2 rows[GRID_CH];
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  n = bev[0];
  const double pivmin = bnd[3], rpivn = rcp_pivmin(pivmin);
  const double x = grid_x(bnd[0], bnd[1], g);
  double q = 0.0;
  int c = 0;
  for (int c0 = 0; c0 < n; c0 += GRID_CH) {
    const int cn = min(GRID_CH, n - c0);
    __syncthreads();
    for (int k = threadIdx.x; k < cn; k += blockDim.x)
      rows[k] = make_double2(d[c0 + k], c0 + k > 0 ? e2g[c0 + k - 1] : 0.0);
    __syncthreads();
    int k0 = 0;
    if (c0 == 0) {
      q = rows[0].x - x;
      k0 = 1;
    }
    for (; k0 + 8 <= cn; k0 += 8) {
      double2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = rows[k0 + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) sturm_step(q, c, v[u], x, pivmin, rpivn);
    }
    for (; k0 < cn; ++k0) sturm_step(q, c, rows[k0], x, pivmin, rpivn);
  }
  if (g < GRID_PTS) gcnt[g] = c + (q <= pivmin);
}

// Starting interval of eigenvalue j of the first block: the grid cell
// [x_{g-1}, x_g) with count(x_{g-1}) <= j < count(x_g) (binary search; the
// ends count 0 and n, so a cell is found even if rounding broke monotonicity).
__device__ inline void grid_start(const int32_t *__restrict__ gcnt, int j, const double *bnd,
                                  double &lo, double &hi) {
  int a = -1, b = GRID_PTS;  // count(a) <= j < count(b)
  while (b - a > 1) {
    const int m = (a + b) >> 1;
    if (gcnt[m] > j) b = m;
    else a = m;
  }
  lo = grid_x(bnd[0], bnd[1], a);
  hi = grid_x(bnd[0], bnd[1], b);
}

// LDS: d and e^2 staged in LDS (n <= 10240); otherwise e2 holds e^2 in global memory.
// gcnt (null: no grid): a wave whose slots are all in the first block starts them from their grid cells.
template <bool LDS>
__global__ __launch_bounds__(256) void bisect_kernel(const double *__restrict__ d,
                                                     const double *__restrict__ e2g, int n,
                                                     const double *__restrict__ bnd,
                                                     const int32_t *__restrict__ bsv,
                                                     const int32_t *__restrict__ bev,
                                                     const int32_t *__restrict__ gcnt,
                                                     double *__restrict__ w_out) {
  extern __shared__ double sh[];
  const double *dd = d, *ee2 = e2g;
  double2 *rows = reinterpret_cast<double2 *>(sh);  // rows[k] = {d[k], e2[k-1]}
  if (LDS) {
    for (int k = threadIdx.x; k < n; k += blockDim.x)
      rows[k] = make_double2(d[k], k > 0 ? e2g[k - 1] : 0.0);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int sub = lane & (ML - 1);
  const int grp_base = lane & ~(ML - 1);
  // slot j = local eigenvalue (j - bs) of the unreduced block [bs, be) holding position j
  const int j = (blockIdx.x * blockDim.x + threadIdx.x) / ML;
  const int b0 = j < n ? bsv[j] : 0, b1 = j < n ? bev[j] : 1;
  const int jl = j - b0;
  const double pivmin = bnd[3];
  double lo = bnd[0], hi = bnd[1];
  // slots of the first block start from their grid cells and need GRID_ROUNDS
  // fewer rounds; the wave runs its longest slot's count, the others idle
  const bool sg = gcnt && j < n && b0 == 0;
  if (sg) grid_start(gcnt, j, bnd, lo, hi);
  const int my_rounds = sg ? ROUNDS - GRID_ROUNDS : ROUNDS;
  const int rounds = __ballot(j < n && !sg) ? ROUNDS : ROUNDS - GRID_ROUNDS;
  for (int round = 0; round < rounds; ++round) {
    const bool act = j < n && round < my_rounds;
    const double x = lo + (hi - lo) * double(sub + 1) / double(ML + 1);
    int c = 0;
    if (act)
      c = LDS ? sturm_count_rows(rows + b0, b1 - b0, x, pivmin)
              : sturm_count(dd + b0, ee2 + b0, b1 - b0, x, pivmin);
    // lanes with count(x) <= jl have x <= lambda_jl
    const unsigned long long m = __ballot(act && c <= jl);
    const unsigned long long gm = ML == 64 ? ~0ull : ((1ull << (ML & 63)) - 1) << grp_base;
    const int a = __popcll(m & gm);
    const double xa1 = __shfl(x, grp_base + (a > 0 ? a - 1 : 0));
    const double xa = __shfl(x, grp_base + (a < ML ? a : ML - 1));
    if (act) {
      lo = a > 0 ? xa1 : lo;
      hi = a < ML ? xa : hi;
    }
  }
  if (j < n && sub == 0) w_out[j] = 0.5 * (lo + hi);
}

// Tridiagonals too long for LDS (n > 10,240): the rows stream through LDS in
// chunks of BIS_CH, staged by the whole workgroup.  The staged block is that of
// the workgroup's first slot; its slots' recurrences walk the same rows in
// lock-step, each carrying its q across the chunks (same arithmetic as the
// LDS-row count).  Slots of other blocks (a workgroup straddling a split:
// in practice the 1 x 1 blocks after the first one) count from global memory.
constexpr int BIS_CH = 2048;
__global__ __launch_bounds__(256) void bisect_chunk_kernel(const double *__restrict__ d,
                                                           const double *__restrict__ e2g, int n,
                                                           const double *__restrict__ bnd,
                                                           const int32_t *__restrict__ bsv,
                                                           const int32_t *__restrict__ bev,
                                                           const int32_t *__restrict__ gcnt,
                                                           double *__restrict__ w_out) {
  __shared__ double2 rows[BIS_CH];
  __shared__ int s_b[2];
  const int lane = threadIdx.x & 63;
  const int sub = lane & (ML - 1);
  const int grp_base = lane & ~(ML - 1);
  const int j = (blockIdx.x * blockDim.x + threadIdx.x) / ML;
  const int b0 = j < n ? bsv[j] : 0, b1 = j < n ? bev[j] : 1;
  const int jl = j - b0;
  const double pivmin = bnd[3];
  const double rpivn = rcp_pivmin(pivmin);
  if (threadIdx.x == 0) {
    const int j0 = blockIdx.x * (blockDim.x / ML);  // < n: the grid covers n slots
    s_b[0] = bsv[j0];
    s_b[1] = bev[j0];
  }
  __syncthreads();
  const int B0 = s_b[0], len = s_b[1] - s_b[0];
  const bool mine = j < n && b0 == B0 && b1 == s_b[1];
  double lo = bnd[0], hi = bnd[1];
  const bool sg = gcnt && j < n && b0 == 0;
  if (sg) grid_start(gcnt, j, bnd, lo, hi);
  const int my_rounds = sg ? ROUNDS - GRID_ROUNDS : ROUNDS;
  // workgroup-uniform trip counts (the chunk loop's barriers)
  const int rounds = __syncthreads_or(j < n && !sg) ? ROUNDS : ROUNDS - GRID_ROUNDS;
  for (int round = 0; round < rounds; ++round) {
    const bool act = j < n && round < my_rounds;
    const double x = lo + (hi - lo) * double(sub + 1) / double(ML + 1);
    int c = 0;
    if (act && !mine) c = sturm_count(d + b0, e2g + b0, b1 - b0, x, pivmin);
    if (__syncthreads_or(act && mine)) {
      const bool run = act && mine;
      double q = 0.0;
      for (int c0 = 0; c0 < len; c0 += BIS_CH) {
        const int cn = min(BIS_CH, len - c0);
        __syncthreads();  // the previous chunk's readers are done
        for (int k = threadIdx.x; k < cn; k += blockDim.x) {
          const int a = B0 + c0 + k;
          rows[k] = make_double2(d[a], c0 + k > 0 ? e2g[a - 1] : 0.0);
        }
        __syncthreads();
        if (run) {
          int k0 = 0;
          if (c0 == 0) {
            q = rows[0].x - x;
            k0 = 1;
          }
          for (; k0 + 8 <= cn; k0 += 8) {
            double2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = rows[k0 + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) sturm_step(q, c, v[u], x, pivmin, rpivn);
          }
          for (; k0 < cn; ++k0) sturm_step(q, c, rows[k0], x, pivmin, rpivn);
        }
      }
      if (run) c += q <= pivmin;
    }
    const unsigned long long m = __ballot(act && c <= jl);
    const unsigned long long gm = ML == 64 ? ~0ull : ((1ull << (ML & 63)) - 1) << grp_base;
    const int a = __popcll(m & gm);
    const double xa1 = __shfl(x, grp_base + (a > 0 ? a - 1 : 0));
    const double xa = __shfl(x, grp_base + (a < ML ? a : ML - 1));
    if (act) {
      lo = a > 0 ? xa1 : lo;
      hi = a < ML ? xa : hi;
    }
  }
  if (j < n && sub == 0) w_out[j] = 0.5 * (lo + hi);
}

// e^2 (e[n-1] = 0 padding)
__global__ void square_kernel(const double *__restrict__ e, int n, double *__restrict__ e2) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) e2[k] = k < n - 1 ? e[k] * e[k] : 0.0;
}

// ---------------------------------------------------------------------------
// A3: truncation rank (gptq_utils.py:94, 97-108), one thread (sequential sums,
// deterministic).
// ---------------------------------------------------------------------------
// LDS: S also staged in LDS (n <= RANK_LDS_N) so the serial passes wait on
// LDS, not on the global round trip of each batch.
constexpr int RANK_LDS_N = 16384;
template <bool LDS>
__global__ void rank_kernel(const double *__restrict__ w_asc, int n, double thr, int rule,
                            double *__restrict__ Sg, int32_t *__restrict__ kout) {
  extern __shared__ double Sl[];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double v = sqrt(fmax(w_asc[n - 1 - i], 1e-12));
    Sg[i] = v;
    if (LDS) Sl[i] = v;
  }
  __syncthreads();
  const double *S = LDS ? Sl : Sg;
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int k = n;
  if (rule == TG_RULE_ENERGY) {
    // sequential sums in the reference's order: the lanes square a chunk of
    // 64 values side by side and the serial adds take them by v_readlane
    auto sq_at = [&](int i0) {
      const double v = i0 + lane < n ? S[i0 + lane] : 0.0;
      return v * v;
    };
    auto rl = [](double x, int u) {
      return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), u),
                              __builtin_amdgcn_readlane(__double2loint(x), u));
    };
    double total = 0.0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const double q = sq_at(i0);
      if (i0 + 64 <= n) {
#pragma unroll
        for (int u = 0; u < 64; ++u) total += rl(q, u);
      } else {
        for (int u = 0; u < n - i0; ++u) total += rl(q, u);
      }
    }
    const double target = (1.0 - thr) * total;
    // the partial sums never decrease (squares >= 0): once one exceeds the
    // target every later one does, so the count stops at that chunk
    double cs = 0.0;
    int cnt = 0;
    for (int i0 = 0; i0 < n && cs <= target; i0 += 64) {
      const double q = sq_at(i0);
      if (i0 + 64 <= n) {
#pragma unroll
        for (int u = 0; u < 64; ++u) {
          cs += rl(q, u);
          cnt += cs <= target;
        }
      } else {
        for (int u = 0; u < n - i0; ++u) {
          cs += rl(q, u);
          cnt += cs <= target;
        }
      }
    }
    k = cnt < n ? cnt + 1 : cnt;
  } else if (rule == TG_RULE_MEAN_TRIMMED) {
    const int ref_k = n < 33 ? n : 33;
    double ref = S[0];
    if (n > 1) {
      double s = 0.0;
      for (int i = 1; i < ref_k; ++i) s += S[i];
      ref = s / double(ref_k - 1);
    }
    int cnt = 0;
    for (int i = lane; i < n; i += 64) cnt += S[i] > thr * ref;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    k = cnt;
  }
  if (lane == 0) *kout = k;
}

// ---------------------------------------------------------------------------
// 3. inverse iteration: one thread per wanted eigenvector (column jj of Z,
// eigenvalue w_asc[n-1-jj]).  LU with partial pivoting of T - lambda I
// (dgttrf pattern), tiny pivots replaced by +-eps*||T|| (dlagts).
// ---------------------------------------------------------------------------
__device__ inline double hash_unit(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return (double(h) + 0.5) / 4294967296.0 - 0.5;
}

constexpr int FCH = 32;  // forward-sweep chunk (elements staged in registers)
constexpr int BCH = 16;  // backward-sweep chunk



__global__ __launch_bounds__(64) void invit_kernel(const double *__restrict__ d,
                                                   const double *__restrict__ e, int n, int k,
                                                   int first,
                                                   const double *__restrict__ w_asc,
                                                   const double *__restrict__ bnd, int iters,
                                                   Tri w) {
  // vector jj (column of Z) is the eigenvector of the (first + jj)-th largest eigenvalue
  const int jj = blockIdx.x * blockDim.x + threadIdx.x;
  if (jj >= k) return;
  const int gi = n - 1 - (first + jj);  // ascending index
  const double lam = w_asc[gi];
  const int sl = w.slot[gi];
  const int b0 = w.bs[sl], b1 = w.be[sl];
  const double tol = fmax(DBL_EPSILON * bnd[2], 1e-300);
  const size_t K = size_t(k);
  const size_t nn = size_t(n) * n;
  // the solve runs on the unreduced block [b0, b1) only; x is zero elsewhere
  double *dd = w.lu + b0 * K, *du = w.lu + nn + b0 * K, *du2 = w.lu + 2 * nn + b0 * K;
  double *x = w.Z + b0 * K;
  d += b0;
  e += b0;
  for (int i = 0; i < b0; ++i) w.Z[size_t(i) * K + jj] = 0.0;
  for (int i = b1; i < n; ++i) w.Z[size_t(i) * K + jj] = 0.0;
  n = b1 - b0;
  auto at = [&](int i) { return size_t(i) * K + jj; };
  auto clampp = [&](double v) { return fabs(v) < tol ? (v < 0.0 ? -tol : tol) : v; };
  for (int i = 0; i < n; ++i) x[at(i)] = hash_unit(uint32_t(b0 + i), uint32_t(first + jj)) + 0.25;
  for (int it = 0; it < iters; ++it) {
    // fused LU (dgttrf pattern) + forward substitution with the row interchanges
    double cur_d = d[0] - lam, cur_u = n > 1 ? e[0] : 0.0, xi = x[at(0)];
    for (int i0 = 0; i0 < n - 1; i0 += FCH) {
      const int cnt = min(FCH, n - 1 - i0);
      double xn[FCH], dn[FCH], en[FCH], enn[FCH];
#pragma unroll
      for (int u = 0; u < FCH; ++u) {  // unconditional (clamped) loads: one batch in flight
        const int i = min(i0 + u, n - 2);
        xn[u] = x[at(i + 1)];
        dn[u] = d[i + 1];
        en[u] = e[i];
        enn[u] = e[min(i + 1, n - 1)];
        if (i + 1 >= n - 1) enn[u] = 0.0;
      }
#pragma unroll
      for (int u = 0; u < FCH; ++u) {
        if (u < cnt) {
          const int i = i0 + u;
          const double sub = en[u], nd = dn[u] - lam, nu = enn[u], xnext = xn[u];
          double xi_next;
          if (fabs(cur_d) >= fabs(sub)) {
            const double piv = clampp(cur_d);
            const double f = fdiv(sub, piv);
            dd[at(i)] = piv;
            du[at(i)] = cur_u;
            du2[at(i)] = 0.0;
            x[at(i)] = xi;
            xi_next = xnext - f * xi;
            cur_d = nd - f * cur_u;
            cur_u = nu;
          } else {
            const double f = fdiv(cur_d, sub);
            dd[at(i)] = sub;
            du[at(i)] = nd;
            du2[at(i)] = nu;
            x[at(i)] = xnext;
            xi_next = xi - f * xnext;
            cur_d = cur_u - f * nd;
            cur_u = -f * nu;
          }
          xi = xi_next;
        }
      }
    }
    dd[at(n - 1)] = clampp(cur_d);
    x[at(n - 1)] = xi;
    // backward substitution with U, in chunks from the end
    double xn1 = 0.0, xn2 = 0.0, amax = 0.0;
    for (int i1 = n; i1 > 0; i1 -= BCH) {
      const int i0 = max(0, i1 - BCH), cnt = i1 - i0;
      double xv[BCH], dv[BCH], uv[BCH], u2v[BCH];
#pragma unroll
      for (int u = 0; u < BCH; ++u) {  // unconditional (clamped) loads: one batch in flight
        const int i = min(i0 + u, n - 1);
        xv[u] = x[at(i)];
        dv[u] = dd[at(i)];
        uv[u] = du[at(i)];
        u2v[u] = du2[at(i)];
        if (i >= n - 1) uv[u] = 0.0;
        if (i >= n - 2) u2v[u] = 0.0;
      }
#pragma unroll
      for (int u = BCH - 1; u >= 0; --u) {
        if (u < cnt) {
          const double v = fdiv(xv[u] - uv[u] * xn1 - u2v[u] * xn2, dv[u]);
          xv[u] = v;
          xn2 = xn1;
          xn1 = v;
          amax = fmax(amax, fabs(v));
        }
      }
#pragma unroll
      for (int u = 0; u < BCH; ++u)
        if (u < cnt) x[at(i0 + u)] = xv[u];
    }
    // rescale (and normalise on the last iteration)
    const double sc = amax > 0.0 ? 1.0 / amax : 1.0;
    double nrm = 0.0;
    for (int i0 = 0; i0 < n; i0 += BCH) {
      double xv[BCH];
#pragma unroll
      for (int u = 0; u < BCH; ++u) xv[u] = x[at(min(i0 + u, n - 1))] * sc;
#pragma unroll
      for (int u = 0; u < BCH; ++u)
        if (i0 + u < n) {
          nrm += xv[u] * xv[u];
          x[at(i0 + u)] = xv[u];
        }
    }
    if (it == iters - 1) {
      const double inv = 1.0 / sqrt(nrm);
      for (int i0 = 0; i0 < n; i0 += BCH) {
        double xv[BCH];
#pragma unroll
        for (int u = 0; u < BCH; ++u) xv[u] = x[at(min(i0 + u, n - 1))];
#pragma unroll
        for (int u = 0; u < BCH; ++u)
          if (i0 + u < n) x[at(i0 + u)] = xv[u] * inv;
      }
    }
  }
}

// Few-vector form of invit_kernel: one wave per vector, its lane 0 runs the
// serial sweeps with x and the LU factors held in LDS, and d, e streamed from
// global one chunk ahead of the chain, so the sweeps wait on neither global
// loads nor stores.  A single lane's LDS instructions cost tens of cycles of
// issue each, so row i keeps {1/pivot, du, du2, x} together (32 bytes) and
// moves as two 16-byte accesses.  The whole wave rescales.  Same dgttrf
// pivoting and substitution order as invit_kernel.
// GR (n > 5120: the rows do not fit the LDS): the same kernel with the rows
// in a per-vector slab of global memory (w.lu), the next chunk's rows
// prefetched through each sweep so the chain still waits on no load.
constexpr int IFCH = 16;
// TG_INVIT_STATS (build-time): s_memrealtime stamps of vector 0's passes
// (start, then per iteration: forward done, backward done, rescaled), printed
// by the host after the launch
#ifndef TG_INVIT_STATS
#define TG_INVIT_STATS 0
#endif
#if TG_INVIT_STATS
__device__ unsigned long long g_invit_stats[16];
#define INVIT_T(slot)                                                              \
  if (jj == 0 && lane == 0) g_invit_stats[slot] = __builtin_amdgcn_s_memrealtime();
#else
#define INVIT_T(slot)
#endif
// Two waves (128 threads; TG_INVIT_ONEWAVE builds: 64, the chain and the
// factor rows on one wave): in a factoring pass wave 0 runs only the pivot
// chain (cur_d, cur_u -> interchange, multiplier f) and hands each chunk's f,
// pivot and cur_u to wave 1 through an LDS ring (workgroup acquire / release),
// which forms the factor rows, the multipliers' copies and the forward
// substitution from them with the same operations -- the chain no longer
// issues them (measured per vector at n = 4096: the factoring pass was 580 us,
// 340 cycles a step, for a dependent chain of ~10 operations).
constexpr int IXS = 4;  // chunk slots of the ring
// TG_INVIT_ONEWAVE=1 (build-time, A/B): the round-6 one-wave kernel (64
// threads, the factoring pass on lane 0 alone); with both forms compiled in,
// the kernel spills (the two waves' blocks and the one-wave step share its
// register budget)
#ifndef TG_INVIT_ONEWAVE
#define TG_INVIT_ONEWAVE 0
#endif
struct InvitXch {
  double2 fd[IXS][IFCH];  // (f, pivot) of each step
  double2 cn[IXS][IFCH];  // (cur_u before the step, d - lambda of the next row)
  double nu[IXS][IFCH];   // e of the next row (0 past the block)
  unsigned msk[IXS];
  unsigned pub, con;  // chunks published by wave 0 / consumed by wave 1
};
__device__ __forceinline__ void ixs_wait(const unsigned *p, unsigned v) {
  // both waves are resident (one workgroup): the other always progresses
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v)
    __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void ixs_put(unsigned *p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool GR>
__global__ __launch_bounds__(128) void invit_lds_kernel(const double *__restrict__ d,
                                                       const double *__restrict__ e, int n, int k,
                                                       int first,
                                                       const double *__restrict__ w_asc,
                                                       const double *__restrict__ bnd, int iters,
                                                       int refac,
                                                       Tri w) {
  extern __shared__ double2 lds_rows[];  // rows[2i] = {1/pivot, du}, rows[2i+1] = {du2, x}
  __shared__ InvitXch xc;
  const int jj = blockIdx.x, lane = threadIdx.x;  // lane < 64: wave 0
  const bool two = !TG_INVIT_ONEWAVE && blockDim.x > 64;
  double2 *rows = GR ? reinterpret_cast<double2 *>(w.lu + size_t(jj) * 4 * size_t(n)) : lds_rows;
  // after the LDS rows (or from the start): the interchange bits of each IFCH-step chunk
  unsigned *swm = reinterpret_cast<unsigned *>(lds_rows + (GR ? 0 : 2 * size_t(n)));
  const int gi = n - 1 - (first + jj);
  const double lam = w_asc[gi];
  const int sl = w.slot[gi];
  const int b0 = w.bs[sl], b1 = w.be[sl], m = b1 - b0;
  const double tol = fmax(DBL_EPSILON * bnd[2], 1e-300);
  const size_t K = size_t(k);
  double *rw = reinterpret_cast<double *>(rows);
  auto X = [&](int i) -> double & { return rw[4 * i + 3]; };
  if (lane < 64)
    for (int i = lane; i < n; i += 64)
      if (i < b0 || i >= b1) w.Z[size_t(i) * K + jj] = 0.0;
  d += b0;
  e += b0;
  double *fz = w.Z + jj;  // multiplier f of block row i at fz[(b0 + i) K] until the last write
  if (lane < 64)
    for (int i = lane; i < m; i += 64) X(i) = hash_unit(uint32_t(b0 + i), uint32_t(first + jj)) + 0.25;
  auto clampp = [&](double v) { return fabs(v) < tol ? (v < 0.0 ? -tol : tol) : v; };
  auto rcp2 = [](double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    return fma(fma(-b, r, 1.0), r, r);
  };
  // e[i] for i in [0, m-1), zero past the block (unconditional load + select)
  auto eat = [&](int i) {
    const double v = e[max(min(i, m - 2), 0)];
    return i < m - 1 ? v : 0.0;
  };
  // a zero the compiler cannot prove uniform: d and e then arrive by vector
  // loads (vmcnt), not scalar ones, so waiting on the chain's LDS traffic
  // (lgkmcnt) does not also wait on the prefetch.  Set afresh (opaque) in each
  // block that fetches, so no block's addresses are hoisted out of the
  // iteration loop and held across the others.
  int vz = 0;
  auto opaque_zero = [&]() { asm volatile("v_mov_b32 %0, 0" : "=v"(vz)); };
  // chunk c covers steps i0..i0+IFCH-1: dn[u] = d[i0+u+1], en[u] = e[i0+u]
  // (e[i0+u+1] is en[u+1], or the next chunk's en[0])
  auto fetch = [&](int i0, double *a, double *b) {
#pragma unroll
    for (int u = 0; u < IFCH; ++u) {
      const int i = i0 + u + vz;
      a[u] = d[min(i + 1, m - 1)];
      b[u] = eat(i);
    }
  };
  // x of the rows after steps i0 .. i0 + IFCH - 1
  auto xload = [&](int i0, double *a) {
#pragma unroll
    for (int u = 0; u < IFCH; ++u) a[u] = X(min(i0 + u + 1 + vz, m - 1));
  };
  __syncthreads();
  INVIT_T(0)
  for (int it = 0; it < iters; ++it) {
    double amax = 0.0;
    const bool fac2 = two && (it == 0 || refac);
    if (fac2) {
      if (lane == 0) {
        xc.pub = 0u;
        xc.con = 0u;
      }
      __syncthreads();
      if (lane == 0) {
        // wave 0: the pivot chain; each step's f, pivot, cur_u and inputs go
        // straight to the ring slot (no wait: wave 1 reads them a chunk later)
        opaque_zero();
        double cur_d = d[0] - lam, cur_u = eat(0);
        double dn[IFCH], en[IFCH], pd[IFCH], pe[IFCH];
        fetch(0, dn, en);
        for (int c = 0, i0 = 0; i0 < m - 1; ++c, i0 += IFCH) {
          const int cnt = min(IFCH, m - 1 - i0);
          fetch(i0 + IFCH, pd, pe);
          const int sl = c % IXS;
          if (c >= IXS) ixs_wait(&xc.con, unsigned(c - IXS + 1));
          unsigned msk = 0;
#pragma unroll
          for (int u = 0; u < IFCH; ++u)
            if (cnt == IFCH || u < cnt) {
              const double sub = en[u], nd = dn[u] - lam;
              const double nu = cnt == IFCH ? (u + 1 < IFCH ? en[u + 1] : pe[0]) : eat(i0 + u + 1);
              const uint64_t sw = __builtin_amdgcn_fcmp(fabs(cur_d), fabs(sub), 12);  // ULT
              const uint64_t tiny = __builtin_amdgcn_fcmp(fabs(cur_d), tol, 4);       // OLT
              const double den = vsel(sw, sub, vsel(tiny, copysign(tol, cur_d), cur_d));
              const double num = vsel(sw, cur_d, sub);
              const double r0 = __builtin_amdgcn_rcp(den);
              const double q0 = num * r0, ee = fma(-den, r0, 1.0);
              const double res = fma(-den, q0, num), r1 = fma(r0, ee, r0);
              const double f = fma(r1, res, q0);
              const double C = vsel(sw, cur_u, nd), D = vsel(sw, nd, cur_u);
              xc.fd[sl][u] = make_double2(f, den);
              xc.cn[sl][u] = make_double2(cur_u, nd);
              xc.nu[sl][u] = nu;
              cur_d = C - f * D;
              cur_u = vsel(sw, -f * nu, nu);
              msk |= unsigned(sw & 1u) << u;
            }
          xc.msk[sl] = msk;
          ixs_put(&xc.pub, unsigned(c + 1));
#pragma unroll
          for (int u = 0; u < IFCH; ++u) {
            dn[u] = pd[u];
            en[u] = pe[u];
          }
        }
        rows[2 * (m - 1)] = make_double2(rcp2(clampp(cur_d)), 0.0);
      } else if (lane == 64) {
        // wave 1: the factor rows, the multipliers' copies (Z's column) and the
        // forward substitution, chunk by chunk behind the chain -- the
        // operations of the one-wave step, on the chain's values
        opaque_zero();
        double xi = X(0);
        double xn[IFCH], xp[IFCH];
        xload(0, xn);
        for (int c = 0, i0 = 0; i0 < m - 1; ++c, i0 += IFCH) {
          const int cnt = min(IFCH, m - 1 - i0);
          xload(i0 + IFCH, xp);  // (rows this chunk does not write)
          const int sl = c % IXS;
          ixs_wait(&xc.pub, unsigned(c + 1));
          const unsigned msk = xc.msk[sl];
#pragma unroll
          for (int u = 0; u < IFCH; ++u)
            if (cnt == IFCH || u < cnt) {
              const double2 fd = xc.fd[sl][u], cn = xc.cn[sl][u];
              const double nu = xc.nu[sl][u];
              const uint64_t sw = ((msk >> u) & 1u) ? ~0ull : 0ull;
              const double f = fd.x, den = fd.y;
              const double r0 = __builtin_amdgcn_rcp(den);
              const double ee = fma(-den, r0, 1.0), r1 = fma(r0, ee, r0);
              const double A = vsel(sw, xi, xn[u]), B = vsel(sw, xn[u], xi);
              const double D = vsel(sw, cn.y, cn.x);
              rows[2 * (i0 + u)] = make_double2(fma(fma(-den, r1, 1.0), r1, r1), D);
              rows[2 * (i0 + u) + 1] = make_double2(vsel(sw, nu, 0.0), B);
              if (iters > 1) fz[size_t(b0 + i0 + u) * K] = f;
              xi = fma(-f, B, A);
            }
          ixs_put(&xc.con, unsigned(c + 1));
          swm[c] = msk;
#pragma unroll
          for (int u = 0; u < IFCH; ++u) xn[u] = xp[u];
        }
        rows[2 * (m - 1) + 1] = make_double2(0.0, xi);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the f (and GR: row) stores
      }
      __syncthreads();
    }
    if (lane == 0) {
      opaque_zero();
      double cur_d = d[0] - lam, cur_u = eat(0), xi = X(0);
      double dn[IFCH], en[IFCH], pd[IFCH], pe[IFCH];
      // one dgttrf step + forward substitution, branch-free.  Row interchange
      // when !(|cur_d| >= |sub|); lane masks + v_cndmask keep the compiler from
      // turning the selects into exec-mask branches.  a / b = q0 + r1 (a - b q0)
      // with r1 one Newton step from v_rcp_f64: the correction runs beside the
      // refinement, shortening the serial chain.
      auto step = [&](double sub, double nd, double nu, double xnext, double2 &o0, double2 &o1,
                      double &fo, unsigned &swb) {
        const uint64_t sw = __builtin_amdgcn_fcmp(fabs(cur_d), fabs(sub), 12);  // ULT
        const uint64_t tiny = __builtin_amdgcn_fcmp(fabs(cur_d), tol, 4);       // OLT
        const double den = vsel(sw, sub, vsel(tiny, copysign(tol, cur_d), cur_d));
        const double num = vsel(sw, cur_d, sub);
        const double r0 = __builtin_amdgcn_rcp(den);
        const double q0 = num * r0, ee = fma(-den, r0, 1.0);
        const double res = fma(-den, q0, num), r1 = fma(r0, ee, r0);
        const double f = fma(r1, res, q0);
        const double A = vsel(sw, xi, xnext), B = vsel(sw, xnext, xi);
        const double C = vsel(sw, cur_u, nd), D = vsel(sw, nd, cur_u);
        o0 = make_double2(fma(fma(-den, r1, 1.0), r1, r1), D);
        o1 = make_double2(vsel(sw, nu, 0.0), B);
        xi = fma(-f, B, A);
        cur_d = C - f * D;
        cur_u = vsel(sw, -f * nu, nu);
        fo = f;
        swb = unsigned(sw & 1u);  // lane 0's interchange
      };
      if (fac2) {
        // (the two waves factored and substituted above)
      } else if (TG_INVIT_ONEWAVE && (it == 0 || refac)) {
        // factor + forward substitution; the multipliers f go to Z's column
        // (free until the final write) and the interchanges to LDS bit masks,
        // so later iterations only substitute (the factors do not change)
        fetch(0, dn, en);
        double xn[IFCH], xp[IFCH];
        xload(0, xn);
        for (int i0 = 0; i0 < m - 1; i0 += IFCH) {
          const int cnt = min(IFCH, m - 1 - i0);
          fetch(i0 + IFCH, pd, pe);  // next chunk in flight while this one runs
          xload(i0 + IFCH, xp);      // (rows this chunk does not write)
          double fo[IFCH];
          unsigned msk = 0;
          if (cnt == IFCH) {
            // outputs leave in one batch after the chunk, off the chain
            double2 o0[IFCH], o1[IFCH];
#pragma unroll
            for (int u = 0; u < IFCH; ++u) {
              unsigned b;
              step(en[u], dn[u] - lam, u + 1 < IFCH ? en[u + 1] : pe[0], xn[u], o0[u], o1[u], fo[u],
                   b);
              msk |= b << u;
            }
#pragma unroll
            for (int u = 0; u < IFCH; ++u) {
              rows[2 * (i0 + u)] = o0[u];
              rows[2 * (i0 + u) + 1] = o1[u];
              if (iters > 1) fz[size_t(b0 + i0 + u) * K] = fo[u];
            }
          } else {
#pragma unroll
            for (int u = 0; u < IFCH; ++u)
              if (u < cnt) {
                double2 o0, o1;
                unsigned b;
                step(en[u], dn[u] - lam, eat(i0 + u + 1), xn[u], o0, o1, fo[0], b);
                msk |= b << u;
                rows[2 * (i0 + u)] = o0;
                rows[2 * (i0 + u) + 1] = o1;
                if (iters > 1) fz[size_t(b0 + i0 + u) * K] = fo[0];
              }
          }
          swm[i0 / IFCH] = msk;
#pragma unroll
          for (int u = 0; u < IFCH; ++u) {
            dn[u] = pd[u];
            en[u] = pe[u];
            xn[u] = xp[u];
          }
        }
        rows[2 * (m - 1)] = make_double2(rcp2(clampp(cur_d)), 0.0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the f stores land before they are read back
      } else {
        // forward substitution with the stored factors: x_i = B, xi = A - f B
        // with (A, B) = (xi, x_{i+1}) or swapped -- the same operations as the
        // factoring pass, so the same values
        double fc[IFCH], fp[IFCH];
        auto ffetch = [&](int i0, double *a) {
#pragma unroll
          for (int u = 0; u < IFCH; ++u)
            a[u] = fz[size_t(b0 + min(i0 + u + vz, max(m - 2, 0))) * K];
        };
        ffetch(0, fc);
        double xn[IFCH], xp[IFCH];
        xload(0, xn);
        for (int i0 = 0; i0 < m - 1; i0 += IFCH) {
          const int cnt = min(IFCH, m - 1 - i0);
          ffetch(i0 + IFCH, fp);
          xload(i0 + IFCH, xp);
          const unsigned msk = swm[i0 / IFCH];
          double xo[IFCH];
          if (cnt == IFCH) {
#pragma unroll
            for (int u = 0; u < IFCH; ++u) {
              const bool sw = (msk >> u) & 1u;
              const double A = sw ? xi : xn[u], B = sw ? xn[u] : xi;
              xo[u] = B;
              xi = fma(-fc[u], B, A);
            }
#pragma unroll
            for (int u = 0; u < IFCH; ++u) X(i0 + u) = xo[u];
          } else {
#pragma unroll
            for (int u = 0; u < IFCH; ++u)
              if (u < cnt) {
                const bool sw = (msk >> u) & 1u;
                const double A = sw ? xi : xn[u], B = sw ? xn[u] : xi;
                X(i0 + u) = B;
                xi = fma(-fc[u], B, A);
              }
          }
#pragma unroll
          for (int u = 0; u < IFCH; ++u) {
            fc[u] = fp[u];
            xn[u] = xp[u];
          }
        }
      }
      if (!fac2) rows[2 * (m - 1) + 1] = make_double2(0.0, xi);
      INVIT_T(1 + 3 * it)
      // backward substitution with U (du of row m-1 and du2 of rows m-2, m-1 are 0)
      double xn1 = 0.0, xn2 = 0.0;
      auto bstep = [&](double2 r0, double2 r1) {
        const double v = (r1.y - r1.x * xn2 - r0.y * xn1) * r0.x;
        xn2 = xn1;
        xn1 = v;
        amax = fmax(amax, fabs(v));
        return v;
      };
      if constexpr (GR) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sweep's row stores
      double2 q0[IFCH], q1[IFCH];  // the chunk below the current one, in flight
      auto rload = [&](int i0, double2 *a, double2 *b) {
#pragma unroll
        for (int u = 0; u < IFCH; ++u) {
          const int i = max(i0, 0) + u + vz;
          a[u] = rows[2 * i];
          b[u] = rows[2 * i + 1];
        }
      };
      if (m - IFCH >= 0) rload(m - IFCH, q0, q1);
      for (int i1 = m; i1 > 0; i1 -= IFCH) {
        const int i0 = i1 - IFCH;
        if (i0 >= 0) {
          double2 r0[IFCH], r1[IFCH];
          double xv[IFCH];
#pragma unroll
          for (int u = 0; u < IFCH; ++u) {
            r0[u] = q0[u];
            r1[u] = q1[u];
          }
          if (i0 - IFCH >= 0) rload(i0 - IFCH, q0, q1);
#pragma unroll
          for (int u = IFCH - 1; u >= 0; --u) xv[u] = bstep(r0[u], r1[u]);
#pragma unroll
          for (int u = 0; u < IFCH; ++u) X(i0 + u) = xv[u];
        } else {
          for (int i = i1 - 1; i >= 0; --i) X(i) = bstep(rows[2 * i], rows[2 * i + 1]);
        }
      }
    }
    INVIT_T(2 + 3 * it)
    __syncthreads();
    if (lane < 64) {  // wave 0 rescales
      amax = __shfl(amax, 0);
      const double sc = amax > 0.0 ? 1.0 / amax : 1.0;
      double nrm = 0.0;
      for (int i = lane; i < m; i += 64) {
        const double v = X(i) * sc;
        nrm += v * v;
        X(i) = v;
      }
      if (it == iters - 1) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nrm += __shfl_xor(nrm, o);
        const double inv = 1.0 / sqrt(nrm);
        for (int i = lane; i < m; i += 64) w.Z[size_t(b0 + i) * K + jj] = X(i) * inv;
      }
    }
    __syncthreads();
    INVIT_T(3 + 3 * it)
  }
}

// Re-orthogonalisation of clusters.  Inverse iteration leaves eigenvectors of
// eigenvalues a gap apart orthogonal to ~eps ||T|| / gap, so columns whose
// consecutive eigenvalues are within ortol * ||T|| (default 1e-6: the other
// pairs stay orthogonal to ~2e-10) are re-orthogonalised as a group (LAPACK
// dstein does the same with ortol = 1e-3, at O(c^2 n) per cluster of c).
// cluster_scan_kernel lists the clusters (columns jj = eigenvalue first + jj
// in descending order); clusters of <= MGS_MAX columns are handled by
// mgs_cols_kernel, one workgroup each, all at once; larger ones by block
// Gram-Schmidt twice (GEMMs against the finished columns) over MGS_MAX-column
// panels, each panel finished by mgs_cols_kernel.
constexpr int MGS_MAX = 64;
// Clusters of at most MGS_SMALL columns are re-orthogonalised by
// mgs_cols_kernel (all at once, one workgroup each); wider ones panel by
// panel (MGS_MAX columns): block Gram-Schmidt twice against the finished
// panels, then CholeskyQR2 of the panel (cq_* kernels below) -- MGS within a
// 64-column panel is 4032 dependent dot/axpy steps over strided rows (88 ms
// per panel at n = 8192), the panel's Gram matrix is one pass.
constexpr int MGS_SMALL = 8;

__global__ void cluster_scan_kernel(const double *__restrict__ w_asc, int n, int k, int first,
                                    const double *__restrict__ bnd, double reltol, int small,
                                    int32_t *__restrict__ cl) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double gap = reltol * bnd[2];
  const double *wd = w_asc + (n - 1 - first);  // wd[-jj] = eigenvalue of column jj
  int ns = 0, nb = 0, start = 0;
  while (start < k) {
    int end = start + 1;
    while (end < k && fabs(wd[-(end - 1)] - wd[-end]) <= gap) ++end;
    if (end - start > 1) {
      int32_t *dst = end - start <= small ? cl + 2 + 2 * ns++ : cl + 2 + 2 * n + 2 * nb++;
      dst[0] = start;
      dst[1] = end - start;
    }
    start = end;
  }
  cl[0] = ns;
  cl[1] = nb;
}

// Modified Gram-Schmidt twice ("twice is enough") over the columns
// [start, start + len) of Z (n x k), one workgroup per (start, len) entry.
// With `only_if` non-null it runs only when *only_if != 0 (the fallback of a
// panel whose CholeskyQR2 was refused).
__global__ __launch_bounds__(256) void mgs_cols_kernel(const int32_t *__restrict__ list, int n,
                                                       int k, double *__restrict__ Z,
                                                       const int *__restrict__ only_if) {
  __shared__ double scratch[8];
  if (only_if && *only_if == 0) return;
  const int start = list[2 * blockIdx.x], end = start + list[2 * blockIdx.x + 1];
  for (int c = start; c < end; ++c) {
    for (int pass = 0; pass < 2; ++pass)
      for (int b = start; b < c; ++b) {
        double dot = 0.0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) dot += Z[size_t(i) * k + b] * Z[size_t(i) * k + c];
        dot = tg::block_sum(dot, scratch);
        for (int i = threadIdx.x; i < n; i += blockDim.x) Z[size_t(i) * k + c] -= dot * Z[size_t(i) * k + b];
        __syncthreads();
      }
    double nrm = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) nrm += Z[size_t(i) * k + c] * Z[size_t(i) * k + c];
    nrm = tg::block_sum(nrm, scratch);
    const double inv = 1.0 / sqrt(nrm);
    for (int i = threadIdx.x; i < n; i += blockDim.x) Z[size_t(i) * k + c] *= inv;
    __syncthreads();
  }
}

// CholeskyQR2 of the panel P = Z[:, p0 : p0 + pw] (pw <= MGS_MAX), in place:
// twice { G = P^T P (partials over row blocks, summed in a fixed order),
// G = R^T R, P <- P R^-1 }.  Q = P R^-1 spans the same leading columns as P
// (R upper triangular), as Gram-Schmidt's result does.  A round whose
// Cholesky meets a column with less than 1e-5 of its norm left after the
// previous columns (kappa too large for two rounds) sets *bad and every later
// step of the panel is skipped; mgs_cols_kernel then takes the panel.
constexpr int CQ_ROWS = 32;  // rows staged per LDS round of the Gram kernel

__global__ __launch_bounds__(256) void cq_gram_kernel(const double *__restrict__ Z, int n, int k,
                                                      int p0, int pw, int rows_per,
                                                      const int *__restrict__ bad,
                                                      double *__restrict__ part) {
  __shared__ double S[CQ_ROWS][MGS_MAX + 1];
  if (*bad) return;
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * rows_per, r1 = min(n, r0 + rows_per);
  double acc[16];  // entry idx = tid + 256 q: (a, b) = (idx / 64, idx % 64)
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  for (int rb = r0; rb < r1; rb += CQ_ROWS) {
    for (int idx = tid; idx < CQ_ROWS * MGS_MAX; idx += 256) {
      const int rr = idx / MGS_MAX, c = idx % MGS_MAX, r = rb + rr;
      S[rr][c] = (r < r1 && c < pw) ? Z[size_t(r) * k + p0 + c] : 0.0;
    }
    __syncthreads();
    for (int rr = 0; rr < CQ_ROWS; ++rr) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int idx = tid + 256 * q;
        acc[q] += S[rr][idx / MGS_MAX] * S[rr][idx % MGS_MAX];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) part[size_t(blockIdx.x) * MGS_MAX * MGS_MAX + tid + 256 * q] = acc[q];
}

// Sum of the partials, Cholesky G = R^T R (upper, right-looking), R^-1 by
// column (one thread per column, back substitution) -> Rinv (row-major 64 x 64).
__global__ __launch_bounds__(256) void cq_chol_kernel(const double *__restrict__ part, int nparts,
                                                      int pw, double *__restrict__ Rinv,
                                                      int *__restrict__ bad) {
  __shared__ double G[MGS_MAX][MGS_MAX + 1];
  __shared__ double d0[MGS_MAX];
  __shared__ int sbad;
  if (*bad) return;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < MGS_MAX * MGS_MAX; idx += 256) {
    double sum = 0.0;
    for (int p = 0; p < nparts; ++p) sum += part[size_t(p) * MGS_MAX * MGS_MAX + idx];
    G[idx / MGS_MAX][idx % MGS_MAX] = sum;
  }
  if (tid == 0) sbad = 0;
  __syncthreads();
  if (tid < pw) d0[tid] = G[tid][tid];
  __syncthreads();
  for (int j = 0; j < pw; ++j) {
    if (tid == 0) {
      const double dj = G[j][j];
      if (!(dj > 1e-10 * d0[j]) || !(d0[j] > 0.0)) sbad = 1;
      G[j][j] = sqrt(fmax(dj, 1e-300));
    }
    __syncthreads();
    if (tid > j && tid < pw) G[j][tid] /= G[j][j];
    __syncthreads();
    for (int idx = tid; idx < MGS_MAX * MGS_MAX; idx += 256) {
      const int a = idx / MGS_MAX, b = idx % MGS_MAX;
      if (a > j && b >= a && b < pw) G[a][b] -= G[j][a] * G[j][b];
    }
    __syncthreads();
  }
  if (sbad) {
    if (tid == 0) *bad = 1;
    return;
  }
  // column c of R^-1: x_c = 1 / R_cc, x_i = -(sum_{j = i+1..c} R_ij x_j) / R_ii
  if (tid < MGS_MAX) {
    const int c = tid;
    double x[MGS_MAX];
#pragma unroll
    for (int i = 0; i < MGS_MAX; ++i) x[i] = 0.0;
    if (c < pw) {
      x[c] = 1.0 / G[c][c];
      for (int i = c - 1; i >= 0; --i) {
        double acc = 0.0;
        for (int j = i + 1; j <= c; ++j) acc += G[i][j] * x[j];
        x[i] = -acc / G[i][i];
      }
    }
#pragma unroll
    for (int i = 0; i < MGS_MAX; ++i) Rinv[i * MGS_MAX + c] = i <= c ? x[i] : 0.0;
  }
}

// P <- P R^-1, one row per thread: out[j] = sum_{b <= j} P[r][b] Rinv[b][j].
__global__ __launch_bounds__(256) void cq_apply_kernel(double *__restrict__ Z, int n, int k, int p0,
                                                       int pw, const double *__restrict__ Rinv,
                                                       const int *__restrict__ bad) {
  __shared__ double Ri[MGS_MAX][MGS_MAX];
  if (*bad) return;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < MGS_MAX * MGS_MAX; idx += 256) Ri[idx / MGS_MAX][idx % MGS_MAX] = Rinv[idx];
  __syncthreads();
  const int r = blockIdx.x * 256 + tid;
  if (r >= n) return;
  double *row = Z + size_t(r) * k + p0;
  // 16 outputs at a time, last block first: block jb reads row[b] only for
  // b < 16 (jb + 1), none of which a later-written block has touched (Rinv
  // is zero below its diagonal, so the sums need no b <= j test)
  for (int jb = MGS_MAX / 16 - 1; jb >= 0; --jb) {
    if (jb * 16 >= pw) continue;
    double out[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) out[jj] = 0.0;
    const int bmax = min(pw, jb * 16 + 16);
    for (int b = 0; b < bmax; ++b) {
      const double zb = row[b];
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) out[jj] += zb * Ri[b][jb * 16 + jj];
    }
#pragma unroll
    for (int jj = 0; jj < 16; ++jj)
      if (jb * 16 + jj < pw) row[jb * 16 + jj] = out[jj];
  }
}

// ---------------------------------------------------------------------------
// 4. back-transformation helpers
// ---------------------------------------------------------------------------
// T factor of block b (dlarft forward/columnwise): reflectors p..p+bw-1.
__global__ __launch_bounds__(256) void tfactor_kernel(const double *__restrict__ V, int n, int nref,
                                                      const double *__restrict__ tau,
                                                      double *__restrict__ Tf) {
  __shared__ double G[BT][BT + 1];
  __shared__ double rows[16][BT];
  __shared__ double Ts[BT][BT + 1];
  const int b = blockIdx.x;
  const int p = b * BT;
  const int bw = min(BT, nref - p);
  const int tid = threadIdx.x;
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  // entries (a, c) for idx = tid + 256*q, a = idx / BT, c = idx % BT
  for (int r0 = p + 1; r0 < n; r0 += 16) {
    for (int idx = tid; idx < 16 * BT; idx += blockDim.x) {
      const int rr = idx / BT, c = idx % BT;
      const int r = r0 + rr;
      rows[rr][c] = (r < n && c < bw) ? V[size_t(r) * n + p + c] : 0.0;
    }
    __syncthreads();
    for (int rr = 0; rr < 16; ++rr) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int idx = tid + 256 * q;
        acc[q] += rows[rr][idx / BT] * rows[rr][idx % BT];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int idx = tid + 256 * q;
    G[idx / BT][idx % BT] = acc[q];
  }
  for (int idx = tid; idx < BT * BT; idx += blockDim.x) Ts[idx / BT][idx % BT] = 0.0;
  __syncthreads();
  for (int a = 0; a < bw; ++a) {
    const double ta = tau[p + a];
    // z[r] = -tau_a G[r][a], r < a ; T[r][a] = sum_{c=r}^{a-1} T[r][c] z[c]
    if (tid < a) {
      double s = 0.0;
      for (int c = tid; c < a; ++c) s += Ts[tid][c] * (-ta * G[c][a]);
      Ts[tid][a] = s;
    }
    if (tid == 0) Ts[a][a] = ta;
    __syncthreads();
  }
  for (int idx = tid; idx < BT * BT; idx += blockDim.x)
    Tf[size_t(b) * BT * BT + idx] = Ts[idx / BT][idx % BT];
}

// Vh[jj][c] = Z[c][jj]  (n x k -> k x n)
__global__ void transpose_kernel(const double *__restrict__ Z, int n, int k, double *__restrict__ Vh,
                                 int ldv) {
  __shared__ double tile[32][33];
  const int c0 = blockIdx.y * 32, j0 = blockIdx.x * 32;
  for (int r = threadIdx.y; r < 32; r += blockDim.y) {
    const int c = c0 + r, jj = j0 + threadIdx.x;
    tile[r][threadIdx.x] = (c < n && jj < k) ? Z[size_t(c) * k + jj] : 0.0;
  }
  __syncthreads();
  for (int r = threadIdx.y; r < 32; r += blockDim.y) {
    const int jj = j0 + r, c = c0 + threadIdx.x;
    if (jj < k && c < n) Vh[size_t(jj) * ldv + c] = tile[threadIdx.x][r];
  }
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
// Two-stage reduction (band.hip) in front of the tridiagonalisation.
// TG_EIGH_TWOSTAGE=0 selects the one-stage reduction (kept for A/B tests).
bool two_stage(int n) {
  const char *e = getenv("TG_EIGH_TWOSTAGE");
  return !(e && e[0] == '0') && n > tg::SB_B + 1;
}

extern "C" size_t tg_eigh_workspace_size(int n) {
  tg::Sizer s;
  tri_layout(s, n, nullptr);
  tg::SbPlan pl(n);
  tg::sb_layout(s, n, n, pl, nullptr);
  return s.off + 256;
}

extern "C" int tg_eigh_values(void *stream, double *A, int n, int lda, double *w_asc, void *ws,
                              size_t ws_bytes) {
  TG_ARG(A, 2, "null A");
  TG_ARG(n >= 1, 3, "n < 1");
  TG_ARG(lda >= n, 4, "lda < n");
  TG_ARG(w_asc, 5, "null w");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  Tri w{};
  tri_layout(ar, n, &w);
  tg::SbPlan pl(n);
  tg::SbBufs sb{};
  tg::sb_layout(ar, n, n, pl, &sb);
  TG_WS(ar);
  const bool ts = two_stage(n);
  if (ts) {
    TG_HIP(tg::sy2sb(st, A, lda, n, pl, sb));
    TG_HIP(tg::sb2st(st, A, lda, n, sb.Bst, sb.V2, sb.prog, w.d, w.e));
    bool stalled = false, broken = false;
    TG_HIP(tg::sb2st_stalled(st, n, sb.prog, &stalled, &broken));
    bool ptmo = false;
    TG_HIP(tg::sy2sb_timed_out(st, pl, sb, &ptmo));
    if (ptmo) {
      tg::set_error("tg_eigh_values: panel-QR grid barrier timed out; the band form is invalid");
      return int(hipErrorLaunchTimeOut);
    }
    if (stalled || broken)  // all-ones bytes: NaN eigenvalues for any caller that ignores the code
      TG_HIP(hipMemsetAsync(w_asc, 0xff, sizeof(double) * size_t(n), st));
    if (stalled) {
      tg::set_error("tg_eigh_values: bulge-chasing pipeline stalled (a hand-off wait timed out); "
                    "the tridiagonal form is invalid");
      return int(hipErrorLaunchTimeOut);
    }
    if (broken) {
      tg::set_error("tg_eigh_values: the tridiagonal failed its invariant check (trace / "
                    "Frobenius norm of the band not preserved by the bulge chase); the "
                    "eigenvalues are poisoned");
      return int(hipErrorIllegalState);
    }
  }
  if (!ts) {
  TG_HIP(hipMemsetAsync(w.V, 0, sizeof(double) * size_t(n) * n, st));
  TG_HIP(hipMemsetAsync(w.cnt, 0, 16 * sizeof(unsigned), st));
  TG_HIP(hipMemsetAsync(w.e, 0, sizeof(double) * n, st));
  TG_HIP(hipMemsetAsync(w.tau, 0, sizeof(double) * n, st));
  const bool vlds = n <= 16384;
  const size_t vsh_bytes = vlds ? sizeof(double) * size_t(n) : 0;
  if (vsh_bytes > 64 * 1024)
    TG_HIP(hipFuncSetAttribute((const void *)tri_symv_kernel<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(vsh_bytes)));
  for (int p = 0; p < n; p += NB) {
    hipLaunchKernelGGL(tri_start_kernel, dim3(std::max(1, tg::cdiv(n - p, 256))), dim3(256), 0, st,
                       A, lda, n, p, w);
    TG_LAUNCHED();
    if (p >= n - 1) break;  // last column: only d[n-1]
    const int pe = min(p + NB, n - 1);
    for (int i = p; i < pe; ++i) {
      const double len = double(n - i - 1);
      auto tok = tg::prof_begin(st, tg::PROF_TRI_SYMV, 8.0 * len * len, 2.0 * len * len);
      const int gs = std::max(1, std::min(NG, tg::cdiv(n - i - 1, SYT / 64)));
      if (vlds)
        hipLaunchKernelGGL(tri_symv_kernel<true>, dim3(gs), dim3(SYT), vsh_bytes, st, A, lda, n,
                           i, p, w);
      else
        hipLaunchKernelGGL(tri_symv_kernel<false>, dim3(gs), dim3(SYT), 0, st, A, lda, n, i, p, w);
      tg::prof_end(st, tok);
      TG_LAUNCHED();
      const int do_next = (i + 1 < p + NB) ? 1 : 0;
      hipLaunchKernelGGL(tri_fin_kernel, dim3(std::max(1, tg::cdiv(n - i - 1, 64))), dim3(64), 0,
                         st, A, lda, n, i, p, do_next, w);
      TG_LAUNCHED();
    }
    const int q = p + NB;
    if (q <= n - 1) {  // trailing rank-2NB update of A[q:, q:]
      const int mt = n - q;
      double *C = A + size_t(q) * lda + q;
      // C -= [V W] [W V]^T : op(A) = ([V^T; W^T])^T, op(B) = [W^T; V^T]
      auto tok = tg::prof_begin(st, tg::PROF_SYR2K, 8.0 * 2.0 * double(mt) * mt,
                                4.0 * double(mt) * mt * NB);
      TG_HIP(tg::dgemm(st, true, false, mt, mt, 2 * NB, -1.0, w.PT + q, n,
                       w.PT + size_t(NB) * n + q, n, 1.0, C, lda));
      tg::prof_end(st, tok);
    }
  }
  }  // one-stage
  // eigenvalues of T
  double *bnd = w.scal;
  hipLaunchKernelGGL(tri_bounds_kernel, dim3(1), dim3(256), 0, st, w.d, w.e, n, bnd);
  TG_LAUNCHED();
  const int blocks = tg::cdiv(int64_t(n) * ML, 256);
  const size_t lds = 2 * sizeof(double) * size_t(n);
  hipLaunchKernelGGL(tri_split_kernel, dim3(1), dim3(1024), 0, st, w.e, n, bnd, w.es, w.bs, w.be);
  TG_LAUNCHED();
  hipLaunchKernelGGL(square_kernel, dim3(tg::cdiv(n, 256)), dim3(256), 0, st, w.es, n, w.acol);
  TG_LAUNCHED();
  if (getenv("TG_TRI_BLOCKS")) {  // development: the unreduced block structure of T
    std::vector<int32_t> hb(n), he(n);
    TG_HIP(hipMemcpyAsync(hb.data(), w.bs, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    TG_HIP(hipMemcpyAsync(he.data(), w.be, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    TG_HIP(hipStreamSynchronize(st));
    std::vector<int> len;
    for (int i = 0; i < n; i = he[i]) len.push_back(he[i] - hb[i]);
    std::vector<int> srt(len);
    std::sort(srt.rbegin(), srt.rend());
    int ones = 0;
    for (int l : len) ones += l == 1;
    fprintf(stderr, "T blocks: n %d, %zu blocks, %d of size 1, largest", n, len.size(), ones);
    for (size_t i = 0; i < srt.size() && i < 6; ++i) fprintf(stderr, " %d", srt[i]);
    fprintf(stderr, "; first block [%d, %d)\n", hb[0], he[0]);
  }
  auto btok = tg::prof_begin(st, tg::PROF_BISECT, 16.0 * n, 0.0);
  const int32_t *gcnt = nullptr;
  if (GRID_ROUNDS > 0 && n >= GRID_MIN_N && !getenv("TG_BISECT_NOGRID")) {
    hipLaunchKernelGGL(grid_count_kernel, dim3(tg::cdiv(GRID_PTS, 256)), dim3(256), 0, st, w.d,
                       w.acol, n, bnd, w.be, w.gcnt);
    TG_LAUNCHED();
    gcnt = w.gcnt;
  }
  if (lds <= 160 * 1024 && !getenv("TG_BISECT_CHUNK")) {  // env: tests force the chunked kernel
    if (lds > 64 * 1024)
      TG_HIP(hipFuncSetAttribute((const void *)bisect_kernel<true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipLaunchKernelGGL(bisect_kernel<true>, dim3(blocks), dim3(256), lds, st, w.d, w.acol, n, bnd,
                       w.bs, w.be, gcnt, w.wraw);
  } else {
    hipLaunchKernelGGL(bisect_chunk_kernel, dim3(blocks), dim3(256), 0, st, w.d, w.acol, n, bnd,
                       w.bs, w.be, gcnt, w.wraw);
  }
  tg::prof_end(st, btok);
  TG_LAUNCHED();
  hipLaunchKernelGGL(rank_sort_kernel, dim3(tg::cdiv(n, 256 / RS_G)), dim3(256), 2048 * sizeof(double), st,
                     w.wraw, n, w_asc, w.slot);
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_truncation_rank(void *stream, const double *w_asc, int n, double threshold,
                                  int rule, double *S_desc, int32_t *k_dev) {
  TG_ARG(w_asc, 2, "null w");
  TG_ARG(n >= 1, 3, "n < 1");
  TG_ARG(S_desc && k_dev, 6, "null output");
  if (n <= RANK_LDS_N) {
    const size_t lds = sizeof(double) * size_t(n);
    if (lds > 48 * 1024)
      TG_HIP(hipFuncSetAttribute((const void *)rank_kernel<true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipLaunchKernelGGL(rank_kernel<true>, dim3(1), dim3(256), lds, (hipStream_t)stream, w_asc, n,
                       threshold, rule, S_desc, k_dev);
  } else {
    hipLaunchKernelGGL(rank_kernel<false>, dim3(1), dim3(256), 0, (hipStream_t)stream, w_asc, n,
                       threshold, rule, S_desc, k_dev);
  }
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_eigh_vectors(void *stream, int n, const double *w_asc, int k, double *Vh, int ldv,
                               void *ws, size_t ws_bytes) {
  return tg_eigh_vectors_range(stream, n, w_asc, 0, k, Vh, ldv, ws, ws_bytes);
}

extern "C" int tg_eigh_vectors_range(void *stream, int n, const double *w_asc, int first, int k,
                                     double *Vh, int ldv, void *ws, size_t ws_bytes) {
  TG_ARG(n >= 1, 2, "n < 1");
  TG_ARG(w_asc, 3, "null w");
  TG_ARG(first >= 0 && first < n, 4, "first must be in [0, n)");
  TG_ARG(k >= 1 && first + k <= n, 5, "count must be in [1, n - first]");
  TG_ARG(Vh, 6, "null Vh");
  TG_ARG(ldv >= n, 7, "ldv < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  Tri w{};
  tri_layout(ar, n, &w);
  tg::SbPlan pl(n);
  tg::SbBufs sb{};
  tg::sb_layout(ar, n, n, pl, &sb);
  TG_WS(ar);
  const double *bnd = w.scal;
  // the few-vector back-transform's Q2 T factors depend only on the bulge
  // reflectors: formed on the side stream beside inverse iteration (14
  // one-wave workgroups) and the cluster checks, joined before the apply
  const bool ts = two_stage(n);
  const bool multi = getenv("TG_BT_MULTI") != nullptr;  // read per call (tests set it)
  const bool few = ts && !multi && tg::sb_apply_few_ok(pl, n, k) &&
                   tg::sb_apply_few_scratch(pl, n, k) <= sizeof(double) * size_t(n) * tg::SB_B;
  const char *tfs = getenv("TG_BT_TF_SIDE");  // development switch: 0 = in order, per call
  const bool tf_side = few && !(tfs && tfs[0] == '0');
  if (tf_side) {
    hipStream_t side = nullptr;
    TG_HIP(tg::side_fork(st, &side));
    TG_HIP(tg::sb_q2_tfactors(side, n, sb.V2, sb.T2));
  }
  auto itok = tg::prof_begin(st, tg::PROF_INVIT, 8.0 * 5 * 4 * double(n) * k, 0.0);
  const char *ie = getenv("TG_INVIT_ITERS");
  const int iters = ie ? std::max(1, std::min(5, atoi(ie))) : 2;
  // few vectors: one LDS-resident wave per vector (4 doubles per row of T,
  // + one interchange mask per IFCH rows)
  const size_t imask = 4 * size_t(tg::cdiv(n, IFCH));
  const size_t ilds = 4 * sizeof(double) * size_t(n) + imask;
  // TG_INVIT_REFACTOR=1 (tests): factor again in every iteration
  const char *rf = getenv("TG_INVIT_REFACTOR");
  const int refac = (rf && rf[0] == '1') ? 1 : 0;
  // (n > 5120: the rows in a per-vector slab of w.lu, 4 n k <= 3 n^2 doubles)
  const char *ig = getenv("TG_INVIT_GROWS");  // development switch: 1 = global rows at any n
  const bool grows = ilds + sizeof(InvitXch) > 160 * 1024 || (ig && ig[0] == '1');
  const int ith = TG_INVIT_ONEWAVE ? 64 : 128;
  const char *ir = getenv("TG_INVIT_REG");  // development switch: 1 = the register kernel
  if (k <= 256 && !(ir && ir[0] == '1')) {
    if (grows) {
      hipLaunchKernelGGL(invit_lds_kernel<true>, dim3(k), dim3(ith), imask, st, w.d, w.es, n, k,
                         first, w_asc, bnd, iters, refac, w);
    } else {
      TG_HIP(hipFuncSetAttribute((const void *)invit_lds_kernel<false>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, int(ilds)));
      hipLaunchKernelGGL(invit_lds_kernel<false>, dim3(k), dim3(ith), ilds, st, w.d, w.es, n, k,
                         first, w_asc, bnd, iters, refac, w);
    }
  } else {
    hipLaunchKernelGGL(invit_kernel, dim3(tg::cdiv(k, 64)), dim3(64), 0, st, w.d, w.es, n, k,
                       first, w_asc, bnd, iters, w);
  }
  tg::prof_end(st, itok);
  TG_LAUNCHED();
#if TG_INVIT_STATS
  {
    unsigned long long h[16];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_invit_stats), sizeof(h));
    fprintf(stderr, "invit n=%d k=%d (vector 0, us):", n, k);
    for (int q = 1; q <= 3 * iters; ++q) fprintf(stderr, " %.1f", (h[q] - h[q - 1]) / 100.0);
    fprintf(stderr, "\n");
  }
#endif
  {
    const char *ot = getenv("TG_INVIT_ORTOL");
    const double ortol = ot ? atof(ot) : 1e-6;
    // panel path: X (p x pw) + Gram partials + Rinv + flag in w.lu (3 n^2 doubles)
    const int cq_np = std::max(1, std::min(64, n / 256));
    const size_t cq_need = size_t(k) * MGS_MAX + size_t(cq_np + 1) * MGS_MAX * MGS_MAX + 1;
    const bool cq = cq_need <= 3 * size_t(n) * n && !getenv("TG_ORTH_MGS");  // (tests set it)
    hipLaunchKernelGGL(cluster_scan_kernel, dim3(1), dim3(64), 0, st, w_asc, n, k, first, bnd,
                       ortol, cq ? MGS_SMALL : MGS_MAX, w.cl);
    TG_LAUNCHED();
    int32_t cnt[2] = {0, 0};
    TG_HIP(hipMemcpyAsync(cnt, w.cl, sizeof(cnt), hipMemcpyDeviceToHost, st));
    TG_HIP(hipStreamSynchronize(st));
    if (cnt[0] > 0) {
      hipLaunchKernelGGL(mgs_cols_kernel, dim3(cnt[0]), dim3(256), 0, st, w.cl + 2, n, k, w.Z,
                         nullptr);
      TG_LAUNCHED();
    }
    if (cnt[1] > 0) {
      std::vector<int32_t> big(2 * size_t(cnt[1]));
      TG_HIP(hipMemcpyAsync(big.data(), w.cl + 2 + 2 * size_t(n), sizeof(int32_t) * big.size(),
                            hipMemcpyDeviceToHost, st));
      TG_HIP(hipStreamSynchronize(st));
      // panel entries (start, width) of every big cluster, for mgs_cols_kernel
      std::vector<int32_t> pan;
      for (int c = 0; c < cnt[1]; ++c)
        for (int p = 0; p < big[2 * c + 1]; p += MGS_MAX) {
          pan.push_back(big[2 * c] + p);
          pan.push_back(std::min(MGS_MAX, big[2 * c + 1] - p));
        }
      int32_t *plist = w.cl + 2 + 2 * size_t(n) + 2 * size_t(cnt[1]);
      TG_HIP(hipMemcpyAsync(plist, pan.data(), sizeof(int32_t) * pan.size(),
                            hipMemcpyHostToDevice, st));
      double *X = w.lu;  // (cluster columns done) x MGS_MAX scratch
      double *part = X + size_t(k) * MGS_MAX;
      double *Rinv = part + size_t(cq_np) * MGS_MAX * MGS_MAX;
      int *bad = reinterpret_cast<int *>(Rinv + MGS_MAX * MGS_MAX);
      const int rows_per = tg::cdiv(tg::cdiv(n, cq_np), CQ_ROWS) * CQ_ROWS;
      const int np = tg::cdiv(n, rows_per);
      int e = 0;
      for (int c = 0; c < cnt[1]; ++c) {
        const int cs = big[2 * c], cl = big[2 * c + 1];
        for (int p = 0; p < cl; p += MGS_MAX, ++e) {
          const int pw = std::min(MGS_MAX, cl - p), p0 = cs + p;
          for (int pass = 0; pass < 2 && p > 0; ++pass) {
            // Z_p -= Z_done (Z_done^T Z_p)
            TG_HIP(tg::dgemm(st, true, false, p, pw, n, 1.0, w.Z + cs, k, w.Z + p0, k, 0.0, X, pw));
            TG_HIP(tg::dgemm(st, false, false, n, pw, p, -1.0, w.Z + cs, k, X, pw, 1.0, w.Z + p0,
                             k));
          }
          if (cq) {
            TG_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
            for (int round = 0; round < 2; ++round) {
              hipLaunchKernelGGL(cq_gram_kernel, dim3(np), dim3(256), 0, st, w.Z, n, k, p0, pw,
                                 rows_per, bad, part);
              hipLaunchKernelGGL(cq_chol_kernel, dim3(1), dim3(256), 0, st, part, np, pw, Rinv, bad);
              hipLaunchKernelGGL(cq_apply_kernel, dim3(tg::cdiv(n, 256)), dim3(256), 0, st, w.Z, n,
                                 k, p0, pw, Rinv, bad);
            }
          }
          hipLaunchKernelGGL(mgs_cols_kernel, dim3(1), dim3(256), 0, st, plist + 2 * e, n, k, w.Z,
                             cq ? bad : nullptr);
          TG_LAUNCHED();
        }
      }
      TG_HIP(hipStreamSynchronize(st));  // pan is read by the copy above
    }
  }
  // back-transformation Z <- Q Z, Q = H_0 H_1 ... H_{n-2}
  const int nref = ts ? 0 : n - 1;
  if (ts) {
    // few vectors (the complement path's request): the LDS-resident kernels
    if (few) {
      if (tf_side)
        TG_HIP(tg::side_join(st));  // the T factors
      else
        TG_HIP(tg::sb_q2_tfactors(st, n, sb.V2, sb.T2));
      bool tmo = false;
      TG_HIP(tg::sb_apply_few(st, n, w.Z, k, pl, sb, sb.X, &tmo));
      if (tmo) {
        tg::set_error("tg_eigh_vectors_range: back-transformation grid barrier timed out");
        return int(hipErrorLaunchTimeOut);
      }
    } else {
      TG_HIP(tg::sb_apply_q2(st, n, w.Z, k, sb.V2, sb.T2));
      TG_HIP(tg::sb_apply_q1(st, n, w.Z, k, pl, sb));
    }
  }
  if (nref > 0) {
    const int nblk = tg::cdiv(nref, BT);
    hipLaunchKernelGGL(tfactor_kernel, dim3(nblk), dim3(256), 0, st, w.V, n, nref, w.tau, w.Tf);
    TG_LAUNCHED();
    auto btok2 = tg::prof_begin(st, tg::PROF_BACKTR, 0.0, 2.0 * double(n) * n * k);
    for (int b = nblk - 1; b >= 0; --b) {
      const int p = b * BT, bw = min(BT, nref - p), r0 = p + 1;
      const double *Vb = w.V + size_t(r0) * n + p;
      // X1 = Vb^T Z[r0:, :]   (bw x k)
      TG_HIP(tg::dgemm_splitk(st, true, false, bw, k, n - r0, 1.0, Vb, n, w.Z + size_t(r0) * k, k,
                              0.0, w.X1, k, SPLITK, w.skp));
      // X2 = T_b X1
      TG_HIP(tg::dgemm(st, false, false, bw, k, bw, 1.0, w.Tf + size_t(b) * BT * BT, BT, w.X1, k,
                       0.0, w.X2, k));
      // Z[r0:, :] -= Vb X2
      TG_HIP(tg::dgemm(st, false, false, n - r0, k, bw, -1.0, Vb, n, w.X2, k, 1.0,
                       w.Z + size_t(r0) * k, k));
    }
    tg::prof_end(st, btok2);
  }
  hipLaunchKernelGGL(transpose_kernel, dim3(tg::cdiv(k, 32), tg::cdiv(n, 32)), dim3(32, 8), 0, st,
                     w.Z, n, k, Vh, ldv);
  TG_LAUNCHED();
  return 0;
}
