// Back-transformation Z <- Q1 Q2 Z for few eigenvectors (k <= 32 columns) in
// ONE persistent launch.
//
// Second half of `torch.linalg.eigh` (/root/reference/src/TruncGPTQ/
// gptq_utils.py:93) for the complement path's ~14 dropped eigenvectors.
// The multi-launch path (sb_apply_q2: one launch per Q2 level, 255 at
// n = 4096; sb_apply_q1: one launch per TSQR level of every panel, ~240) is
// launch- and latency-bound for k this small (~8 ms for 14 columns against
// ~30 us of reflector traffic).  Here one grid of W workgroups (8 waves each)
// walks the same ~500 steps with an in-kernel grid barrier between steps:
//   Q2 level L: blocks (G2, s) with s + (NG2 - 1 - G2) = L, one wave per block
//               (63 x 32 staircase Y, Z -= Y (T (Y^T Z)) on FP64 MFMA);
//   Q1 step (panel p, level l), panels last to first, levels top down: one
//               workgroup per TSQR chunk (<= 512 rows, 8 waves x 64 rows).
// Hand-off between steps (cdna_hip_programming.md Guideline 16, counter
// form): Z is stored write-through (sc1, 8-B relaxed agent-scope stores),
// every wave drains vmcnt, one lane adds to the step counter, polls it
// relaxed (bounded spin; a timeout sets a flag the host reads), then ONE
// agent-scope acquire before the next step's plain loads.  Reflectors (Y, T,
// V2, T2) are written by earlier launches and read plainly.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "band.h"
#include "common.h"
#include "spin.h"

namespace {

using tg::SB_B;
using tg::SB_C;

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef double doublex2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int QB = 32;             // sweeps per Q2 block (= SB_B)
constexpr int QR = QB + SB_B - 1;  // rows per Q2 block (63)
constexpr int BW = 8;              // waves per workgroup

struct Q1Op {
  int r0, rows, nc, lv, yoff, toff;  // Z row offset, stacked rows, chunks, level, Y/T offsets
};

struct BtArgs {
  double *Z;
  int n, k;
  const double *V2, *T2;  // Q2 reflectors / block T factors
  int smax, ng2, nlev2;
  const double *Y, *T;    // Q1 (TSQR) reflectors / T factors
  const Q1Op *ops;
  int nops;
  int single;             // one-level panels (q1_big_a / q1_big_b)
  double *part;           // single: per-sub-chunk P partials (32 x 32 each)
  unsigned *cnt;          // [0] step counter, [1] timeout flag (zeroed per call)
  unsigned long long timeout;
  int wexp;               // XCD form: workers wanted (= workgroups per XCD)
  // Q2 as a wavefront (TG_BT_Q2_WAVE=1): colflag[G2] = blocks of
  // sweep group G2 applied (zeroed per call, ~0u once the group is done)
  unsigned *colflag;
  int q2_wave;
};

struct SmQ2 {
  double Vs[BW][QB][SB_B + 1];
  double Ts[BW][QB][QB + 1];
};
struct SmQ1 {
  double red[BW][SB_B][SB_B + 1];
  double Ps[SB_B][SB_B + 1];
  double Ms[SB_B][SB_B + 1];
};
union BtShared {
  SmQ2 q2;
  SmQ1 q1;
};

__device__ inline int ntasks(int n, int j) { return (j <= n - 3) ? (n - 3 - j) / SB_B + 1 : 0; }
__device__ inline bool refl_valid(int n, int j, int s) { return j <= n - 3 && s < ntasks(n, j); }

// TG_BT_XCD=1: the workers are the workgroups that landed on the first XCD
// to arrive (the rest exit), so Z hand-offs stay in that XCD's L2: plain
// stores drained by vmcnt, relaxed L2 counter, sc1 (L1-bypassing) Z loads,
// no release/acquire fences.  TG_BT_XCD=0: placement-independent form
// (write-through Z stores, agent-scope acquire after every barrier).
#ifndef TG_BT_XCD
#define TG_BT_XCD 1
#endif

__device__ inline void store_sc1(double *p, double v) {
#if TG_BT_XCD
  *p = v;
#else
  __hip_atomic_store((gu64 *)(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#endif
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
// Z element e (row-major index) as last stored by any worker of this launch
__device__ inline double load_z(const BtArgs &a, __amdgpu_buffer_rsrc_t rz, int64_t e) {
#if TG_BT_XCD
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rz, int(e * 8), 0, 16);  // sc1
  return __builtin_bit_cast(double, v);
#else
  return a.Z[e];
#endif
}

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Step done by this workgroup; wait for all workers.  Wave 0 arrives and
// polls as a whole wave (scalar loop, spin.h); a stalled barrier sets cnt[1]
// and every later barrier of the launch returns at once.
__device__ inline void grid_barrier(const BtArgs &a, unsigned target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's Z stores drained
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    tg::wave_arrive(a.cnt);
    tg::spin_geq(a.cnt, target, a.cnt + 1, a.timeout);
#if !TG_BT_XCD
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  }
  __syncthreads();
}

// Reflector data of one Q2 block in registers (issued before the barrier
// that precedes its use, so its HBM latency overlaps the hand-off).
struct Q2Pre {
  double vv[16], tt[16];
};
__device__ inline void q2_fetch(const BtArgs &a, int G2, int s, Q2Pre &p) {
  const int lane = threadIdx.x & 63, j0 = G2 * QB;
  const double *Tb = a.T2 + (int64_t(G2) * a.smax + s) * QB * QB;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int idx = lane + 64 * q, r = idx >> 5, d = idx & 31;
    const int jj = refl_valid(a.n, j0 + r, s) ? j0 + r : j0;
    p.vv[q] = d == 0 ? 1.0 : a.V2[(int64_t(jj) * a.smax + s) * SB_B + d];  // [0] holds tau
    p.tt[q] = Tb[idx];
  }
}

// One Q2 block (G2, s) by one wave: Z[rb0 .. rb0 + 62, 0 .. k) -= Y (T (Y^T Z)),
// NCB 16-column blocks of Z (k <= 16 NCB).
template <int NCB>
__device__ void q2_block(const BtArgs &a, __amdgpu_buffer_rsrc_t rz, int G2, int s,
                         const Q2Pre &pre, double (*Vs)[SB_B + 1], double (*Ts)[QB + 1]) {
  const int n = a.n, k = a.k, lane = threadIdx.x & 63;
  const int lr = lane >> 4, lc = lane & 15;
  const int j0 = G2 * QB;
  const int rb0 = j0 + 1 + s * SB_B;
  // Z tile first (its latency overlaps the LDS staging of V and T)
  double zl[4][4][NCB];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int row = min(rb0 + rb * 16 + lr + 4 * q, n - 1);
        const int col = min(cb * 16 + lc, k - 1);
        zl[rb][q][cb] = load_z(a, rz, int64_t(row) * k + col);
      }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int idx = lane + 64 * q, r = idx >> 5, d = idx & 31;
    Vs[r][d] = refl_valid(n, j0 + r, s) ? pre.vv[q] : 0.0;
    Ts[r][d] = pre.tt[q];
  }
  wave_sync();
  auto yval = [&](int i, int c) -> double {
    const int d = i - c;
    return (d >= 0 && d < SB_B) ? Vs[c][d] : 0.0;
  };
  doublex4 F[4][NCB];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = rb * 16 + lr + 4 * q;
      const bool ok = i < QR && rb0 + i < n;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb][q] = (ok && cb * 16 + lc < k) ? zl[rb][q][cb] : 0.0;
    }
  doublex4 Pa[2][NCB];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = rb * 16 + 4 * q + lr;
      double ya[2];
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) ya[ia] = yval(i, ia * 16 + lc);
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[ia], F[rb][cb][q], Pa[ia][cb], 0, 0, 0);
    }
  doublex4 Ma[2][NCB];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) Ma[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = kb * 16 + 4 * q + lr;
      double ta[2];
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) ta[ia] = Ts[ia * 16 + lc][kk];
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          Ma[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ta[ia], Pa[kb][cb][q], Ma[ia][cb], 0, 0, 0);
    }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = kb * 16 + 4 * q + lr;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const double ya = -yval(rb * 16 + lc, kk);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          F[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, Ma[kb][cb][q], F[rb][cb], 0, 0, 0);
      }
    }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = rb * 16 + lr + 4 * q;
      const int row = rb0 + i;
      if (i >= QR || row >= n) continue;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + lc;
        if (col < k) store_sc1(&a.Z[int64_t(row) * k + col], F[rb][cb][q]);
      }
    }
  wave_sync();  // Vs / Ts reused by this wave's next block
}

// Stacked row s of TSQR level lv -> level-0 row (band.hip RowMap::fwd).
__device__ inline int fwd_row(int lv, int s) {
  for (int l = lv; l >= 1; --l) s = (s / SB_B) * SB_C + s % SB_B;
  return s;
}

// Reflector data of one Q1 chunk for this wave: Y rows of the P = Y^T Z
// product in MFMA A-operand order, and this thread's two entries of T.
struct Q1Pre {
  double ya[4][4][2];
  double t[2];
};
__device__ inline void q1_fetch(const BtArgs &a, const Q1Op &d, int I, Q1Pre &p) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, lr = lane >> 4, lc = lane & 15;
  const int kb = I * SB_C, ke = (I == d.nc - 1) ? d.rows : kb + SB_C, h = ke - kb;
  const double *Y = a.Y + d.yoff;
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + 4 * q + lr;
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) p.ya[rb][q][ia] = Y[int64_t(kb + min(rl, h - 1)) * SB_B + ia * 16 + lc];
    }
#pragma unroll
  for (int t = 0; t < 2; ++t) p.t[t] = a.T[d.toff + size_t(I) * SB_B * SB_B + tid + 64 * BW * t];
}

// One Q1 chunk I of step d by the workgroup: Z_c -= Y (T (Y^T Z_c)), wave w
// owns chunk rows 64w .. 64w + 63.
template <int NCB>
__device__ void q1_chunk(const BtArgs &a, __amdgpu_buffer_rsrc_t rz, const Q1Op &d, int I,
                         const Q1Pre &pre, SmQ1 &sm) {
  const int k = a.k, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  const int kb = I * SB_C, ke = (I == d.nc - 1) ? d.rows : kb + SB_C, h = ke - kb;
  const double *Y = a.Y + d.yoff;
  double *Zs = a.Z + int64_t(d.r0) * k;
  doublex4 F[4][NCB];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
      const int zr = fwd_row(d.lv, kb + min(rl, h - 1));
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb][q] = load_z(a, rz, int64_t(d.r0 + zr) * k + min(cb * 16 + lc, k - 1));
    }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb][q] = (rl < h && cb * 16 + lc < k) ? F[rb][cb][q] : 0.0;
    }
  doublex4 Pa[2][NCB];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + 4 * q + lr;
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) {
        const double ya = rl < h ? pre.ya[rb][q][ia] : 0.0;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, F[rb][cb][q], Pa[ia][cb], 0, 0, 0);
      }
    }
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) sm.red[wid][ia * 16 + lr + 4 * q][cb * 16 + lc] = Pa[ia][cb][q];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int idx = tid + 64 * BW * t;
    sm.Ms[idx >> 5][idx & 31] = pre.t[t];
  }
  __syncthreads();
  for (int idx = tid; idx < SB_B * SB_B; idx += 64 * BW) {
    const int r = idx >> 5, cc = idx & 31;
    if (cc >= 16 * NCB) continue;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < BW; ++w) v += sm.red[w][r][cc];
    sm.Ps[r][cc] = v;
  }
  __syncthreads();
  double mval[2] = {0.0, 0.0};
  for (int idx = tid, t = 0; idx < SB_B * SB_B; idx += 64 * BW, ++t) {
    const int r = idx >> 5, cc = idx & 31;
    if (cc >= 16 * NCB) continue;
    double v = 0.0;
    for (int e = r; e < SB_B; ++e) v += sm.Ms[r][e] * sm.Ps[e][cc];
    mval[t] = v;
  }
  __syncthreads();  // T no longer read: Ms <- T P
  for (int idx = tid, t = 0; idx < SB_B * SB_B; idx += 64 * BW, ++t) sm.Ms[idx >> 5][idx & 31] = mval[t];
  __syncthreads();
#pragma unroll
  for (int k0 = 0; k0 < SB_B; k0 += 4) {
    double bm[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) bm[cb] = sm.Ms[k0 + lr][cb * 16 + lc];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int rl = wid * 64 + rb * 16 + lc;
      const double yl = Y[int64_t(kb + min(rl, h - 1)) * SB_B + k0 + lr];
      const double ya = rl < h ? -yl : 0.0;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, bm[cb], F[rb][cb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * 64 + rb * 16 + lr + 4 * q;
      if (rl >= h) continue;
      const int zr = fwd_row(d.lv, kb + rl);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + lc;
        if (col < k) store_sc1(&Zs[int64_t(zr) * k + col], F[rb][cb][q]);
      }
    }
  __syncthreads();  // red / Ps / Ms reused by the next chunk
}

// Q1 sub-chunk rows of the single-level back-transform: one 16-row block
// per wave (more workgroups, no serial row blocks: 512-row sub-chunks left
// 8 of 16 workers idle and each worker four load -> MFMA rounds).
constexpr int Q1S = 128;
constexpr int Q1RB = Q1S / (16 * BW);
static_assert(Q1RB >= 1 && Q1S % (16 * BW) == 0, "sub-chunk = whole 16-row blocks per wave");

// Single-level panels (one compact-WY block of m rows, band.h SbPlan::single):
// sub-chunks of Q1S rows, two phases with a grid barrier between them.
// Sub-chunks are aligned to absolute Z rows (sub-chunk j = rows [128 j,
// 128 j + 128) clipped to the panel's rows), so q1_lds_kernel -- whose
// workgroups hold fixed row ranges -- forms the same partials and sums them
// in the same order: the two Q1 forms are bit-identical.
// Phase A: sub-chunk I (the I-th at or below the panel) publishes
// P_I = Y_I^T Z_I (32 x k) to part[I].
__device__ inline void q1_sub_rows(const Q1Op &d, int I, int &g0, int &lo, int &hi) {
  g0 = (d.r0 / Q1S + I) * Q1S;              // first Z row of the sub-chunk
  lo = max(0, d.r0 - g0);                   // local rows [lo, hi) are the panel's
  hi = min(Q1S, d.r0 + d.rows - g0);
}
__device__ inline int q1_nsub(const Q1Op &d) {
  return (d.r0 + d.rows - 1) / Q1S - d.r0 / Q1S + 1;
}
// M = T P for the single-level Q1 (T 32 x 32 upper triangular, zeros below;
// P 32 x 16 ncb), on FP64 MFMA: wave w < 2 ncb forms the 16 x 16 tile
// (ia, cb) = (w & 1, w >> 1), k ascending in steps of 4.  bt_few_kernel and
// q1_lds_kernel both use it, so their M (and Z) agree bit for bit.
template <int TS, int PS>
__device__ __forceinline__ doublex4 q1_tp_mfma(const double *T, const double *P, int w) {
  const int lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
  const int ia = w & 1, cb = w >> 1;
  doublex4 acc = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < SB_B; k0 += 4)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(T[(ia * 16 + lc) * TS + k0 + lr],
                                               P[(k0 + lr) * PS + cb * 16 + lc], acc, 0, 0, 0);
  return acc;
}

template <int NCB>
__device__ void q1_big_a(const BtArgs &a, __amdgpu_buffer_rsrc_t rz, const Q1Op &d, int I,
                         SmQ1 &sm) {
  const int k = a.k, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  int g0, lo, hi;
  q1_sub_rows(d, I, g0, lo, hi);
  const double *Y = a.Y + d.yoff + int64_t(g0 - d.r0) * SB_B;
  doublex4 Pa[2][NCB];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int rb = 0; rb < Q1RB; ++rb) {
    double zl[4][NCB], ya[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * (16 * Q1RB) + rb * 16 + 4 * q + lr, rc = min(max(rl, lo), hi - 1);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        zl[q][cb] = load_z(a, rz, int64_t(g0 + rc) * k + min(cb * 16 + lc, k - 1));
#pragma unroll
      for (int ia = 0; ia < 2; ++ia) ya[q][ia] = Y[int64_t(rc) * SB_B + ia * 16 + lc];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * (16 * Q1RB) + rb * 16 + 4 * q + lr;
      const bool act = rl >= lo && rl < hi;
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const double zv = (act && cb * 16 + lc < k) ? zl[q][cb] : 0.0;
          const double yv = act ? ya[q][ia] : 0.0;
          Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(yv, zv, Pa[ia][cb], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) sm.red[wid][ia * 16 + lr + 4 * q][cb * 16 + lc] = Pa[ia][cb][q];
  __syncthreads();
  double *out = a.part + int64_t(I) * SB_B * SB_B;
  for (int idx = tid; idx < SB_B * SB_B; idx += 64 * BW) {
    const int r = idx >> 5, cc = idx & 31;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < BW; ++w) v += sm.red[w][r][cc];
    store_sc1(&out[idx], v);
  }
  __syncthreads();  // red reused by the next sub-chunk
}

// Phase B: P = sum_J P_J (sub-chunk order), M = T P, Z_I -= Y_I M.
template <int NCB>
__device__ void q1_big_b(const BtArgs &a, __amdgpu_buffer_rsrc_t rz, const Q1Op &d, int I,
                         int nsub, SmQ1 &sm) {
  const int k = a.k, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  int g0, lo, hi;
  q1_sub_rows(d, I, g0, lo, hi);
  const double *Y = a.Y + d.yoff + int64_t(g0 - d.r0) * SB_B;
  double *Zs = a.Z + int64_t(g0) * k;
  doublex4 F[Q1RB][NCB];
#pragma unroll
  for (int rb = 0; rb < Q1RB; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * (16 * Q1RB) + rb * 16 + lr + 4 * q, rc = min(max(rl, lo), hi - 1);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb][q] = load_z(a, rz, int64_t(g0 + rc) * k + min(cb * 16 + lc, k - 1));
    }
  for (int idx = tid; idx < SB_B * SB_B; idx += 64 * BW) {
    double v = 0.0;
    for (int j0 = 0; j0 < nsub; j0 += 8) {
      double t[8];
#pragma unroll
      for (int b = 0; b < 8; ++b)
        t[b] = j0 + b < nsub ? __hip_atomic_load(a.part + int64_t(j0 + b) * SB_B * SB_B + idx,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0.0;
#pragma unroll
      for (int b = 0; b < 8; ++b) v += t[b];
    }
    sm.Ps[idx >> 5][idx & 31] = v;
    sm.Ms[idx >> 5][idx & 31] = a.T[d.toff + idx];
  }
  __syncthreads();
  // M = T P (q1_tp_mfma), over T in Ms once every wave is done reading it
  doublex4 mt{};
  if (wid < 2 * NCB) mt = q1_tp_mfma<SB_B + 1, SB_B + 1>(&sm.Ms[0][0], &sm.Ps[0][0], wid);
  __syncthreads();
  if (wid < 2 * NCB) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sm.Ms[(wid & 1) * 16 + lr + 4 * q][(wid >> 1) * 16 + lc] = mt[q];
  }
  __syncthreads();
#pragma unroll
  for (int k0 = 0; k0 < SB_B; k0 += 4) {
    double bm[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) bm[cb] = sm.Ms[k0 + lr][cb * 16 + lc];
#pragma unroll
    for (int rb = 0; rb < Q1RB; ++rb) {
      const int rl = wid * (16 * Q1RB) + rb * 16 + lc;
      const double yl = Y[int64_t(min(max(rl, lo), hi - 1)) * SB_B + k0 + lr];
      const double ya = (rl >= lo && rl < hi) ? -yl : 0.0;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        F[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, bm[cb], F[rb][cb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < Q1RB; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = wid * (16 * Q1RB) + rb * 16 + lr + 4 * q;
      if (rl < lo || rl >= hi) continue;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int col = cb * 16 + lc;
        if (col < k) store_sc1(&Zs[int64_t(rl) * k + col], F[rb][cb][q]);
      }
    }
  __syncthreads();
}

template <int NCB, bool Q2W>
__global__ __launch_bounds__(64 * BW) void bt_few_kernel(BtArgs a) {
  __shared__ BtShared sm;
  __shared__ int sh_w[2];
  const int wid = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rz =
      __builtin_amdgcn_make_buffer_rsrc(a.Z, 0, int(int64_t(a.n) * a.k * 8), 0x00020000);
#if TG_BT_XCD
  // workers: the first a.wexp workgroups to arrive on the first XCD to
  // arrive; cnt[2] = XCD + 1, cnt[3] = worker tickets, cnt[4] = workgroups
  // checked in.  The workers start as soon as a.wexp tickets are out (the
  // usual case: the dispatcher deals the grid of a.wexp x XCDs workgroups
  // round-robin), or, when fewer land there, once every workgroup of the
  // grid has checked in (then the ticket count is final): both ways every
  // worker reads the same count.
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    unsigned expect = 0;
    __hip_atomic_compare_exchange_strong((gu32 *)(a.cnt + 2), &expect, x + 1, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool mine = (expect == 0 ? x + 1 : expect) == x + 1;
    int ticket = -1;
    if (mine)
      ticket = int(__hip_atomic_fetch_add((gu32 *)(a.cnt + 3), 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT));
    // the ticket is taken (returned) before this workgroup counts as checked in
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add((gu32 *)(a.cnt + 4), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_w[0] = ticket < a.wexp ? ticket : -1;
    if (sh_w[0] >= 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      unsigned tk;
      while ((tk = __hip_atomic_load((gu32 *)(a.cnt + 3), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT)) < unsigned(a.wexp) &&
             __hip_atomic_load((gu32 *)(a.cnt + 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 gridDim.x) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
          tg::stall_set(a.cnt + 1);
          break;
        }
      }
      tk = __hip_atomic_load((gu32 *)(a.cnt + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sh_w[1] = int(min(tk, unsigned(a.wexp)));
    }
  }
  __syncthreads();
  if (sh_w[0] < 0) return;
  const int W = sh_w[1], me = sh_w[0];
#else
  const int W = gridDim.x, me = blockIdx.x;
#endif
  unsigned step = 0;
#ifdef TG_BT_STATS
  uint64_t st_q2 = 0, st_b2 = 0, st_q1 = 0, st_b1 = 0;
#define BT_T(v) const uint64_t v = __builtin_amdgcn_s_memrealtime();
#else
#define BT_T(v)
#endif
  // the wave's first block of level L (t index), -1 if none
  auto q2_first = [&](int L, int &G2, int &s) {
    const int s_lo = max(0, L - (a.ng2 - 1)), s_hi = min(a.smax - 1, L);
    for (int t = me * BW + wid; t <= s_hi - s_lo; t += W * BW) {
      s = s_lo + t;
      G2 = a.ng2 - 1 - (L - s);
      if (G2 >= 0 && refl_valid(a.n, G2 * QB, s)) return true;
    }
    return false;
  };
  Q2Pre p2;
  if constexpr (Q2W) if (a.nlev2 > 0) {
    // Q2 as a wavefront instead of level by level: block (G2, s) needs the
    // blocks of the later sweep group G2 + 1 up to step s (the rows it
    // shares: (G2 + 1, s - 1) and (G2 + 1, s); everything else it overlaps
    // precedes those), and its own group's step s - 1.  So each wave takes
    // whole sweep groups, G2 descending, steps ascending, waits only for
    // colflag[G2 + 1] >= s + 1 and publishes colflag[G2] after its Z stores
    // drained -- point-to-point hand-offs in the one XCD's L2 (the level
    // form paid a grid barrier per level: 255 levels at n = 4096).  Same
    // blocks, same arithmetic, same order on every row: bit-identical Z.
    const int NW = W * BW, gw = me * BW + wid;
    unsigned *stall = a.cnt + 1;
    const int lane = threadIdx.x & 63;
    for (int c = gw; c < a.ng2; c += NW) {
      const int G2 = a.ng2 - 1 - c, nb = ntasks(a.n, G2 * QB);
      if (nb > 0) q2_fetch(a, G2, 0, p2);
      for (int s = 0; s < nb; ++s) {
        if (G2 + 1 < a.ng2) tg::spin_geq(a.colflag + G2 + 1, unsigned(s + 1), stall, a.timeout);
#if TG_BT_XCD
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // Z loads stay below the poll
#else
        // placement-independent build: Z is read through L1 (load_z), so the
        // producer's rows need an agent-scope acquire (its stores are
        // write-through, store_sc1)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
        q2_block<NCB>(a, rz, G2, s, p2, sm.q2.Vs[wid], sm.q2.Ts[wid]);
        if (s + 1 < nb) q2_fetch(a, G2, s + 1, p2);  // read-only reflectors: no wait needed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's Z stores drained
        if (lane == 0)
          __hip_atomic_store((gu32 *)(a.colflag + G2), unsigned(s + 1), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0)
        __hip_atomic_store((gu32 *)(a.colflag + G2), ~0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_barrier(a, unsigned(W) * ++step);  // every group done before Q1
  }
  int nG2 = 0, ns = 0;
  const int nlev2 = Q2W ? 0 : a.nlev2;
  bool have = nlev2 > 0 && q2_first(0, nG2, ns);
  if (have) q2_fetch(a, nG2, ns, p2);
  for (int L = 0; L < nlev2; ++L) {
    BT_T(t0)
    const int s_lo = max(0, L - (a.ng2 - 1)), s_hi = min(a.smax - 1, L);
    bool first = true;
    for (int t = me * BW + wid; t <= s_hi - s_lo; t += W * BW) {
      const int s = s_lo + t, G2 = a.ng2 - 1 - (L - s);
      if (G2 < 0 || !refl_valid(a.n, G2 * QB, s)) continue;
      if (!first) q2_fetch(a, G2, s, p2);  // more blocks than waves: no look-ahead
      first = false;
      q2_block<NCB>(a, rz, G2, s, p2, sm.q2.Vs[wid], sm.q2.Ts[wid]);
    }
    // next level's first block: its reflectors load across the barrier
    if (L + 1 < nlev2 && q2_first(L + 1, nG2, ns)) q2_fetch(a, nG2, ns, p2);
    BT_T(t1)
    grid_barrier(a, unsigned(W) * ++step);
    BT_T(t2)
#ifdef TG_BT_STATS
    st_q2 += t1 - t0;
    st_b2 += t2 - t1;
#endif
  }
  if (a.single) {
    for (int o = 0; o < a.nops; ++o) {
      BT_T(t0)
      const Q1Op d = a.ops[o];
      const int nsub = q1_nsub(d);
      for (int I = me; I < nsub; I += W) q1_big_a<NCB>(a, rz, d, I, sm.q1);
      BT_T(t1)
      grid_barrier(a, unsigned(W) * ++step);
      BT_T(t2)
      for (int I = me; I < nsub; I += W) q1_big_b<NCB>(a, rz, d, I, nsub, sm.q1);
      BT_T(t3)
      if (o + 1 < a.nops) grid_barrier(a, unsigned(W) * ++step);
      BT_T(t4)
#ifdef TG_BT_STATS
      st_q1 += (t1 - t0) + (t3 - t2);
      st_b1 += (t2 - t1) + (t4 - t3);
#endif
    }
#ifdef TG_BT_STATS
    if (me == 0 && threadIdx.x == 0) {
      unsigned long long *o = reinterpret_cast<unsigned long long *>(a.cnt + 8);
      o[0] = st_q2; o[1] = st_b2; o[2] = st_q1; o[3] = st_b1;
    }
#endif
    return;
  }
  Q1Pre p1;
  if (a.nops > 0 && me < a.ops[0].nc) q1_fetch(a, a.ops[0], me, p1);
  for (int o = 0; o < a.nops; ++o) {
    BT_T(t0)
    const Q1Op d = a.ops[o];
    for (int I = me; I < d.nc; I += W) {
      if (I != me) q1_fetch(a, d, I, p1);
      q1_chunk<NCB>(a, rz, d, I, p1, sm.q1);
    }
    if (o + 1 < a.nops) {
      const Q1Op dn = a.ops[o + 1];
      if (me < dn.nc) q1_fetch(a, dn, me, p1);
    }
    BT_T(t1)
    if (o + 1 < a.nops) grid_barrier(a, unsigned(W) * ++step);
    BT_T(t2)
#ifdef TG_BT_STATS
    st_q1 += t1 - t0;
    st_b1 += t2 - t1;
#endif
  }
#ifdef TG_BT_STATS
  if (me == 0 && threadIdx.x == 0) {
    unsigned long long *o = reinterpret_cast<unsigned long long *>(a.cnt + 8);
    o[0] = st_q2; o[1] = st_b2; o[2] = st_q1; o[3] = st_b1;
  }
#endif
}

// ---------------------------------------------------------------------------
// Q2 with Z resident in LDS (the default for k <= 16; TG_BT_Q2_LDS=0 keeps
// bt_few_kernel's level-by-level Q2).  Block (G2, s) touches Z rows
// [32 c + 1, 32 c + 64), c = G2 + s: row chunks c and c + 1 (chunk c = rows
// 32 c + 1 .. 32 c + 32), and must follow exactly (G2, s - 1) and (G2 + 1, s)
// (the blocks it shares a chunk with one level earlier; the last block of a
// group, s = nb(G2) - 1 = nb(G2 + 1), follows the whole of group G2 + 1).
// One wave per sweep group G2 walks its blocks s = 0, 1, ...; QW consecutive
// groups form a workgroup whose waves hand chunks down through LDS (group
// G2 + 1 finishes a chunk, G2 takes it one block later) with LDS progress
// counters (workgroup acquire / release).  A chunk enters a workgroup once,
// from the next workgroup's lowest wave (or from Z), and leaves it once,
// through its own lowest wave: that wave stores the first chunk of each block
// to global memory write-through (sc1), drains and publishes its progress in a
// global word; the next lower workgroup's top wave polls the word and loads
// the chunk with sc1 loads (MI355X_MICROARCH.md "Valid forms" row 1,
// placement-independent).  So the 255-block chain at n = 4096 crosses a
// global hand-off only once per workgroup (16); the rest are LDS hand-offs.
// (The first form, one wave per pair column c, shared each boundary chunk
// between two workgroups that alternated on it every level: 254 global
// hand-offs on the critical path, 1.76 ms.)  The workgroup keeps a ring of
// RS chunks; the top wave reuses a slot only after the lowest wave is done
// with its previous chunk.  Same blocks, reflectors, T factors and MFMA
// sequence as q2_block: Z is bit-identical to the level-by-level form.
// ---------------------------------------------------------------------------
// TG_Q2L_QW (build-time): sweep groups (waves) per workgroup.  4 = one wave
// per SIMD: a block's 80 FP64 MFMAs (64 cycles each) own their SIMD's
// matrix pipe; at 8 two waves share it and the MFMA phase doubles
#ifndef TG_Q2L_QW
#define TG_Q2L_QW 4
#endif
constexpr int QW = TG_Q2L_QW;
constexpr int RS = 16;  // chunk ring slots per workgroup

struct Q2LArgs {
  double *Z;
  int n, k;
  const double *V2, *T2;
  int smax, ng2;
  unsigned *gprog;  // [slabs x ng2]: blocks done by each group, per column slab (zeroed)
  unsigned *stall;  // set on a timed-out wait (the host reports it)
  unsigned long long timeout;
  int slab0;        // first column slab of this launch (slab = slab0 + blockIdx.y)
};

template <int NCB>
struct Q2LShared {  // (QW = 4: 104 KB)
  double Zs[RS][32][16 * NCB + 1];  // chunk c in slot c % RS
  double Vs[QW][QB][SB_B + 1];
  unsigned done[QW];
  unsigned dead;
};

__device__ __forceinline__ unsigned q2l_get(const unsigned *p) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// whole-wave bounded wait on an LDS counter (false once the launch is dead)
__device__ inline bool q2l_wait(const unsigned *p, unsigned v, unsigned *dead, unsigned *stall,
                                unsigned long long timeout) {
  if (q2l_get(p) >= v) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned it = 0;; ++it) {
    if (q2l_get(dead)) return false;
    __builtin_amdgcn_s_sleep(1);
    if (q2l_get(p) >= v) return true;
    if ((it & 63u) == 63u && (__builtin_amdgcn_readfirstlane(tg::ctl_load(stall)) != 0u ||
                              __builtin_amdgcn_s_memrealtime() - t0 > timeout)) {
      tg::stall_set(stall);
      __hip_atomic_store(dead, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
  }
}

// Reflector data of block (G2, s): V as q2_fetch (staged to LDS for the
// staircase reads), T straight into the A-operand layout of the T P product
// (tt[(kb * 4 + qq) * 2 + ia] = T[16 ia + lc][16 kb + 4 qq + lr]), so T needs
// no LDS of its own
__device__ inline void q2l_fetch(const Q2LArgs &a, int G2, int s, Q2Pre &p) {
  const int lane = threadIdx.x & 63, j0 = G2 * QB, lr = lane >> 4, lc = lane & 15;
  const double *Tb = a.T2 + (int64_t(G2) * a.smax + s) * QB * QB;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = lane + 64 * u, r = idx >> 5, d = idx & 31;
    const int jj = refl_valid(a.n, j0 + r, s) ? j0 + r : j0;
    p.vv[u] = d == 0 ? 1.0 : a.V2[(int64_t(jj) * a.smax + s) * SB_B + d];  // [0] holds tau
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
      for (int ia = 0; ia < 2; ++ia)
        p.tt[(kb * 4 + qq) * 2 + ia] = Tb[(ia * 16 + lc) * QB + kb * 16 + 4 * qq + lr];
}

__device__ __forceinline__ int q2l_nb(int n, int G2) { return ntasks(n, G2 * QB); }

// TG_Q2L_STATS (build-time): per-phase s_memtime cycles of every block,
// summed over waves (wait for the group above / the ring slot, Z tile + V
// staging, MFMA chain, stores + publish), read by the host after the launch
#ifndef TG_Q2L_STATS
#define TG_Q2L_STATS 0
#endif
#if TG_Q2L_STATS
__device__ unsigned long long g_q2l_stats[8];
#define Q2L_T(v) const uint64_t v = __builtin_amdgcn_s_memtime();
#else
#define Q2L_T(v)
#endif

template <int NCB>
__global__ __launch_bounds__(64 * QW, 1) void q2_lds_kernel(Q2LArgs a) {
  __shared__ Q2LShared<NCB> sm;
  constexpr int KC = 16 * NCB;
  // column slab slab0 + blockIdx.y: columns KC slab .. of Z (ld a.k), its own
  // progress words (the columns are independent: each slab is a back-transform
  // of its own, the same arithmetic as a call with those columns alone)
  const int slab = a.slab0 + int(blockIdx.y), ld = a.k;
  double *const Zb = a.Z + KC * slab;
  unsigned *const gprog = a.gprog + size_t(slab) * a.ng2;
  const int n = a.n, k = min(KC, a.k - KC * slab), tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = blockIdx.x, G0 = w * QW, G2 = G0 + g;
  const int gtop = min(QW, a.ng2 - G0) - 1;  // highest wave with a sweep group
  const int lr = lane >> 4, lc = lane & 15;
  // this workgroup's own chunks G0 .. G0 + QW - 1 from Z (no higher group touches them)
  for (int e = tid; e < QW * 32 * KC; e += 64 * QW) {
    const int q = e / (32 * KC), r = (e / KC) % 32, col = e % KC;
    const int c = G0 + q, row = 32 * c + 1 + r;
    sm.Zs[c % RS][r][col] = (row < n && col < k) ? Zb[int64_t(row) * ld + col] : 0.0;
  }
  if (tid < QW) sm.done[tid] = 0u;
  if (tid == 0) sm.dead = 0u;
  __syncthreads();
  const int nb = g <= gtop ? q2l_nb(n, G2) : 0;
  const int nbu = G2 + 1 < a.ng2 ? q2l_nb(n, G2 + 1) : 0;  // blocks of the group above
  Q2Pre pre;
  if (nb > 0) q2l_fetch(a, G2, 0, pre);
#if TG_Q2L_STATS
  uint64_t st[4] = {0, 0, 0, 0};
#endif
  for (int s = 0; s < nb; ++s) {
    const int j0 = G2 * QB, c = G2 + s, rb0 = j0 + 1 + s * SB_B;
    Q2L_T(t0)
    // Off the chain, before the waits: this block's reflectors into LDS and
    // from there the MFMA A operands of both V products into registers (the
    // staircase selects included), T's into tv, and the next block's
    // reflectors in flight -- none of it depends on Z.  After the waits only
    // the Z tile, the 80 MFMAs and the stores remain.
    double(*Vs)[SB_B + 1] = sm.Vs[g];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = lane + 64 * u, r = idx >> 5, d = idx & 31;
      Vs[r][d] = refl_valid(n, j0 + r, s) ? pre.vv[u] : 0.0;
    }
    double tv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) tv[u] = pre.tt[u];
    if (s + 1 < nb) q2l_fetch(a, G2, s + 1, pre);
    wave_sync();
    auto yval = [&](int i, int cc) -> double {
      const int d = i - cc;
      return (d >= 0 && d < SB_B) ? Vs[cc][d] : 0.0;
    };
    double ya1[4][4][2], ya3[2][4][4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int ia = 0; ia < 2; ++ia) ya1[rb][qq][ia] = yval(rb * 16 + 4 * qq + lr, ia * 16 + lc);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) ya3[kb][qq][rb] = -yval(rb * 16 + lc, kb * 16 + 4 * qq + lr);
    // (G2 + 1, s) -- or, for the last block, all of group G2 + 1
    if (nbu > 0) {
      const unsigned need = unsigned(min(s + 1, nbu));
      if (g < gtop) q2l_wait(&sm.done[g + 1], need, &sm.dead, a.stall, a.timeout);
      else if (!q2l_get(&sm.dead) && !tg::spin_geq(gprog + G2 + 1, need, a.stall, a.timeout))
        sm.dead = 1u;
    }
    // the top wave brings chunk c + 1 into the ring: its slot held chunk
    // c + 1 - RS, done once the lowest wave finished that as a first chunk
    const bool from_g = g == gtop;
    if (from_g) {
      const int prev = c + 1 - RS - G0;  // the lowest wave's block that released the slot
      if (prev >= 0) q2l_wait(&sm.done[0], unsigned(prev + 1), &sm.dead, a.stall, a.timeout);
    }
    Q2L_T(t1)
    // Z tile: rows i < 32 from chunk c (LDS), i >= 32 from chunk c + 1 (LDS,
    // or global for the top wave).  The block's 63 rows leave chunk c + 1's
    // last row (i = 63) out; the top wave still carries it into the ring
    // (x63, unchanged), since the blocks that take c + 1 as their first chunk
    // update it
    doublex4 F[4][NCB];
    double x63[NCB];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const bool gl = rb >= 2 && from_g;
      const int sl = (rb < 2 ? c : c + 1) % RS;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int i = rb * 16 + lr + 4 * qq, r = i & 31, row = rb0 + i;
        const bool ok = i < QR && row < n;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int col = cb * 16 + lc;
          double v;
          if (gl)
            v = __hip_atomic_load(&Zb[int64_t(min(row, n - 1)) * ld + min(col, k - 1)],
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            v = sm.Zs[sl][r][col];
          F[rb][cb][qq] = (ok && col < k) ? v : 0.0;
          if (rb == 3 && qq == 3) x63[cb] = v;  // row i = 63 on lanes lr = 3
        }
      }
    }
    Q2L_T(t2)
    doublex4 Pa[2][NCB];
#pragma unroll
    for (int ia = 0; ia < 2; ++ia)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int ia = 0; ia < 2; ++ia)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya1[rb][qq][ia], F[rb][cb][qq],
                                                              Pa[ia][cb], 0, 0, 0);
    doublex4 Ma[2][NCB];
#pragma unroll
    for (int ia = 0; ia < 2; ++ia)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) Ma[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int ia = 0; ia < 2; ++ia)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            Ma[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(tv[(kb * 4 + qq) * 2 + ia],
                                                              Pa[kb][cb][qq], Ma[ia][cb], 0, 0, 0);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            F[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya3[kb][qq][rb], Ma[kb][cb][qq],
                                                             F[rb][cb], 0, 0, 0);
#if TG_Q2L_STATS
    asm volatile("s_nop 0" : "+v"(F[3][0][3]));  // the chain's last MFMA issued
#endif
    Q2L_T(t3)
    // stores: the lowest wave hands its first chunk (and, at its last block,
    // the second) to global memory write-through; everything else to the ring
    const bool last = s + 1 == nb;
    if (from_g && !(g == 0 && last) && lr == 3 && rb0 + 63 < n) {
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        if (cb * 16 + lc < k) sm.Zs[(c + 1) % RS][31][cb * 16 + lc] = x63[cb];
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const bool gl = g == 0 && (rb < 2 || last);
      const int sl = (rb < 2 ? c : c + 1) % RS;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int i = rb * 16 + lr + 4 * qq, r = i & 31, row = rb0 + i;
        if (i >= QR || row >= n) continue;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int col = cb * 16 + lc;
          if (col >= k) continue;
          if (gl)
            __hip_atomic_store((gu64 *)&Zb[int64_t(row) * ld + col],
                               __double_as_longlong(F[rb][cb][qq]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          else
            sm.Zs[sl][r][col] = F[rb][cb][qq];
        }
      }
    }
    // publish block s: LDS release (this wave's ring stores before it); the
    // lowest wave also to its global word after draining its sc1 stores
    __hip_atomic_store(&sm.done[g], unsigned(s + 1), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    if (g == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_store((gu32 *)(gprog + G2), unsigned(s + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    wave_sync();  // Vs reused by the next block
#if TG_Q2L_STATS
    const uint64_t t4 = __builtin_amdgcn_s_memtime();
    st[0] += t1 - t0;
    st[1] += t2 - t1;
    st[2] += t3 - t2;
    st[3] += t4 - t3;
#endif
  }
#if TG_Q2L_STATS
  if (lane == 0 && nb > 0) {
    for (int x = 0; x < 4; ++x) atomicAdd(&g_q2l_stats[x], (unsigned long long)st[x]);
    atomicAdd(&g_q2l_stats[4], (unsigned long long)nb);
  }
#endif
}

// ---------------------------------------------------------------------------
// Q1 with Z resident in LDS (after q2_lds_kernel, the default for k <= 16 and
// single-level panels; TG_BT_Q1_LDS=0 keeps bt_few_kernel's Q1).  Q1 is 127
// panel steps (n = 4096), Z[r0:] -= Y (T (Y^T Z[r0:])) from the last panel to
// the first; each step needs P = Y^T Z over every row at or below the panel's,
// a reduction over the grid.  Here each workgroup holds one 128-row sub-chunk
// of Z in LDS for the whole launch; per step it stages the step's Y rows
// (prefetched into registers during the previous step's exchange), forms its
// sub-chunk's partial on MFMA, publishes it with one arrival on a counter,
// waits for all W arrivals, sums the partials in sub-chunk order (16-byte sc1
// loads, all in flight at once), forms M = T P on MFMA and updates its rows --
// one grid exchange per step instead of bt_few's two barriers, Z never
// re-read.  A sub-chunk wholly above the panel only keeps the step count.
// n <= 32 x 128: the workgroups of one XCD, plain partial stores in its L2
// (L2 = true); larger n: one workgroup per CU anywhere, write-through
// partials (L2 = false).
// Bit-identical to bt_few's Q1 (q1_big_a / q1_big_b): the same row-aligned
// sub-chunks, each the sum of eight 16-row MFMA partials in block order, the
// sub-chunk sum in the same order (leading sub-chunks above the panel are
// skipped, as bt_few has none), the same q1_tp_mfma and Z -= Y M chains.
// Partials are double-buffered by step parity: a workgroup can be at most one
// step ahead of the slowest (the arrival wait), so it never overwrites
// partials another is still summing.
// ---------------------------------------------------------------------------
constexpr int Q1W = 4;                 // waves per workgroup
constexpr int Q1R = Q1S;               // Z rows per workgroup: one sub-chunk (32 per wave)
constexpr int Q1BW = Q1R / (16 * Q1W); // 16-row blocks per wave
static_assert(Q1S == 16 * BW && Q1BW * Q1W == BW, "a sub-chunk is bt_few's BW 16-row blocks");

struct Q1LArgs {
  double *Z;
  int n, k;
  const double *Y, *T;
  const Q1Op *ops;
  int nops;
  double *part;     // 2 x W x 512 partials (step parity, sub-chunk, 32 x 16)
  unsigned *cnt;    // [0] arrivals (zeroed per call)
  unsigned *elect;  // [0] XCD + 1, [1] tickets, [2] checked in, [3] not placed (zeroed)
  unsigned *stall;  // timeout flag
  int nw;           // workers: cdiv(n, Q1R) (the grid is nw x XCDs)
  unsigned long long timeout;
  int slab0;        // (L2 = false) first 16-column slab of this launch: slab0 + blockIdx.y
};

struct Q1LShared {
  double Zs[Q1R][17];
  double Ys[Q1R][SB_B + 1];   // this step's Y rows (zero outside the panel)
  double red[BW][SB_B][17];   // the sub-chunk's block partials (block = bt_few's wave)
  double Ps[SB_B][17];
  double Ts[SB_B][SB_B + 1];
  double Ms[SB_B][17];
};

// step d's Y rows R0 .. R0 + Q1R - 1 (raw, clamped rows) and T into
// registers: issued a step ahead, masked and staged at the next step
struct Q1LPre {
  double y[Q1R * SB_B / (64 * Q1W)];
  double t[SB_B * SB_B / (64 * Q1W)];
};
__device__ __forceinline__ void q1l_fetch(const Q1LArgs &a, const Q1Op &d, int R0, Q1LPre &p) {
  const int tid = threadIdx.x, col = tid & 31, rsub = tid >> 5;
  const double *Y = a.Y + d.yoff;
#pragma unroll
  for (int u = 0; u < Q1R * SB_B / (64 * Q1W); ++u) {
    const int row = R0 + u * (64 * Q1W / SB_B) + rsub;
    p.y[u] = Y[int64_t(min(max(row - d.r0, 0), d.rows - 1)) * SB_B + col];
  }
#pragma unroll
  for (int u = 0; u < SB_B * SB_B / (64 * Q1W); ++u) p.t[u] = a.T[d.toff + tid + 64 * Q1W * u];
}

// Workers: the nw workgroups of one XCD (the first to arrive; tickets 0 ..
// nw - 1), so every hand-off below stays in that XCD's L2 (the one-L2 form
// of csrc/spin.h: plain stores, drained, then the arrival; sc1 loads).  Each
// worker holds a fixed row block, so the kernel needs all nw: if fewer land
// on the elected XCD (the dispatcher's placement is not guaranteed), every
// worker leaves before touching Z and elect[3] tells the host to run
// bt_few's Q1 instead.
__device__ inline int q1l_elect(const Q1LArgs &a) {
  __shared__ int sh_w;
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    unsigned expect = 0;
    __hip_atomic_compare_exchange_strong((gu32 *)a.elect, &expect, x + 1, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool mine = (expect == 0 ? x + 1 : expect) == x + 1;
    int ticket = -1;
    if (mine)
      ticket = int(__hip_atomic_fetch_add((gu32 *)(a.elect + 1), 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ticket taken before checking in
    __hip_atomic_fetch_add((gu32 *)(a.elect + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int me = ticket < a.nw ? ticket : -1;
    if (me >= 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load((gu32 *)(a.elect + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 unsigned(a.nw) &&
             __hip_atomic_load((gu32 *)(a.elect + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 gridDim.x) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
          tg::stall_set(a.stall);
          break;
        }
      }
      if (__hip_atomic_load((gu32 *)(a.elect + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
          unsigned(a.nw)) {
        if (me == 0) tg::ctl_record(a.elect + 3, 1u);
        me = -1;
      }
    }
    sh_w = me;
  }
  __syncthreads();
  return sh_w;
}

// TG_Q1L_STATS (build-time): s_memtime cycles per step of each phase, summed
// over workers (stage Y/T + partials, drain, exchange, P sum + M + Z update)
#ifndef TG_Q1L_STATS
#define TG_Q1L_STATS 0
#endif
#if TG_Q1L_STATS
__device__ unsigned long long g_q1l_stats[8];
#define Q1L_T(v) const uint64_t v = __builtin_amdgcn_s_memtime();
#else
#define Q1L_T(v)
#endif

// L2 = false (n > 32 x 128 = 4096): the placement-independent form -- the
// grid is the workers (all resident: one workgroup per CU), partials stored
// write-through (sc1) and read sc1 (MI355X guide "Valid forms" row 1).
template <bool L2>
__global__ __launch_bounds__(64 * Q1W) void q1_lds_kernel(Q1LArgs a) {
  __shared__ Q1LShared sm;
  const int w = L2 ? q1l_elect(a) : int(blockIdx.x);
  if (w < 0) return;
#if TG_Q1L_STATS
  uint64_t st[6] = {0, 0, 0, 0, 0, 0};
#endif
  const int W = a.nw, R0 = w * Q1R;
  // (L2 = false) column slab slab0 + blockIdx.y: Z columns 16 slab .. (ld
  // a.k), its own arrival counter and partials (the launch's blockIdx.y-th)
  const int ys = L2 ? 0 : int(blockIdx.y), slab = L2 ? 0 : a.slab0 + ys, ld = a.k;
  double *const Zb = a.Z + 16 * slab;
  double *const part = a.part + size_t(ys) * 2 * W * 512;
  unsigned *const cnt = a.cnt + 16 * slab;
  const int n = a.n, k = min(16, a.k - 16 * slab), tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane >> 4, lc = lane & 15;
  // the partials as a buffer: 16-byte sc1 loads of two entries
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      part, 0, int(size_t(2) * W * 512 * sizeof(double)), 0x00020000);
  constexpr int SC1 = 16;  // cache policy bit of the L1-bypassing loads
  for (int e = tid; e < Q1R * 16; e += 64 * Q1W) {
    const int r = e >> 4, col = e & 15, row = R0 + r;
    sm.Zs[r][col] = (row < n && col < k) ? Zb[int64_t(row) * ld + col] : 0.0;
  }
  Q1LPre pre;
  if (a.nops > 0) q1l_fetch(a, a.ops[0], R0, pre);
  for (int o = 0; o < a.nops; ++o) {
    Q1L_T(t0)
    const Q1Op d = a.ops[o];
    const int rend = d.r0 + d.rows;
    // a sub-chunk wholly above the panel neither contributes (the sum starts
    // at the panel's sub-chunk) nor changes: it only keeps the step count
    // (arrival + wait, so that it never runs more than a step ahead of the
    // partials it will write once the panels reach it)
    const bool live = R0 + Q1R > d.r0;  // uniform per workgroup
    if (live) {
#pragma unroll
      for (int u = 0; u < Q1R * SB_B / (64 * Q1W); ++u) {
        const int rl = u * (64 * Q1W / SB_B) + (tid >> 5), row = R0 + rl;
        sm.Ys[rl][tid & 31] = (row >= d.r0 && row < rend) ? pre.y[u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < SB_B * SB_B / (64 * Q1W); ++u) {
        const int e = tid + 64 * Q1W * u;
        sm.Ts[e >> 5][e & 31] = pre.t[u];
      }
      __syncthreads();
      // the 16-row blocks' partials Y^T Z (rows outside the panel: 0)
#pragma unroll
      for (int rb = 0; rb < Q1BW; ++rb) {
        const int blk = wid * Q1BW + rb;
        doublex4 Pa[2];
#pragma unroll
        for (int ia = 0; ia < 2; ++ia) Pa[ia] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = blk * 16 + 4 * q + lr, row = R0 + rl;
          const bool act = row >= d.r0 && row < rend;
          const double zv = act ? sm.Zs[rl][lc] : 0.0;
#pragma unroll
          for (int ia = 0; ia < 2; ++ia)
            Pa[ia] = __builtin_amdgcn_mfma_f64_16x16x4f64(sm.Ys[rl][ia * 16 + lc], zv, Pa[ia], 0, 0, 0);
        }
#pragma unroll
        for (int ia = 0; ia < 2; ++ia)
#pragma unroll
          for (int q = 0; q < 4; ++q) sm.red[blk][ia * 16 + lr + 4 * q][lc] = Pa[ia][q];
      }
      __syncthreads();
      // the sub-chunk partial (blocks in order, as bt_few sums its waves'),
      // published to the one XCD's L2
      double *mine = part + (size_t(o & 1) * W + w) * 512;
      for (int e = tid; e < 512; e += 64 * Q1W) {
        const int r = e >> 4, cc = e & 15;
        double v = 0.0;
#pragma unroll
        for (int b = 0; b < BW; ++b) v += sm.red[b][r][cc];
        if constexpr (L2)
          mine[e] = v;  // stays in the one XCD's L2
        else
          __hip_atomic_store(&mine[e], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    Q1L_T(t1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores drained
    __syncthreads();
    Q1L_T(t2)
    // the next step's Y and T: in flight through the exchange below (issued
    // after the drain, which would otherwise wait for them too)
    if (o + 1 < a.nops && R0 + Q1R > a.ops[o + 1].r0) q1l_fetch(a, a.ops[o + 1], R0, pre);
    if (wid == 0) {
      tg::wave_arrive(cnt);
      tg::spin_geq(cnt, unsigned(W) * unsigned(o + 1), a.stall, a.timeout);
    }
    __syncthreads();
    Q1L_T(t3)
    if (live) {
      // P = sum of the sub-chunk partials from the panel's first, in order:
      // entries 2 tid, 2 tid + 1 of every sub-chunk, all loads in flight at once
      {
        const int j0 = d.r0 / Q1S;
        double v0 = 0.0, v1 = 0.0;
        for (int jb = j0; jb < W; jb += 32) {
          doublex2 t[32];
#pragma unroll
          for (int b = 0; b < 32; ++b)
            t[b] = __builtin_bit_cast(
                doublex2, __builtin_amdgcn_raw_buffer_load_b128(
                              rp, int(((size_t(o & 1) * W + min(jb + b, W - 1)) * 512 + 2 * tid) * 8),
                              0, SC1));
#pragma unroll
          for (int b = 0; b < 32; ++b)
            if (jb + b < W) {
              v0 += t[b][0];
              v1 += t[b][1];
            }
        }
        const int e = 2 * tid;
        sm.Ps[e >> 4][e & 15] = v0;
        sm.Ps[e >> 4][(e & 15) + 1] = v1;
      }
      __syncthreads();
      // M = T P (q1_tp_mfma: waves 0, 1; T upper triangular)
      if (wid < 2) {
        const doublex4 mt = q1_tp_mfma<SB_B + 1, 17>(&sm.Ts[0][0], &sm.Ps[0][0], wid);
#pragma unroll
        for (int q = 0; q < 4; ++q) sm.Ms[wid * 16 + lr + 4 * q][lc] = mt[q];
      }
      __syncthreads();
      // Z -= Y M on this wave's rows
      doublex4 F[Q1BW];
#pragma unroll
      for (int rb = 0; rb < Q1BW; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) F[rb][q] = sm.Zs[(wid * Q1BW + rb) * 16 + lr + 4 * q][lc];
#pragma unroll
      for (int k0 = 0; k0 < SB_B; k0 += 4) {
        const double bm = sm.Ms[k0 + lr][lc];
#pragma unroll
        for (int rb = 0; rb < Q1BW; ++rb) {
          const int rl = (wid * Q1BW + rb) * 16 + lc, row = R0 + rl;
          const bool act = row >= d.r0 && row < rend;
          const double ya = act ? -sm.Ys[rl][k0 + lr] : 0.0;
          F[rb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya, bm, F[rb], 0, 0, 0);
        }
      }
#pragma unroll
      for (int rb = 0; rb < Q1BW; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) sm.Zs[(wid * Q1BW + rb) * 16 + lr + 4 * q][lc] = F[rb][q];
      __syncthreads();  // Ms, Ts, Ps, Ys, red reused by the next step
    }
    Q1L_T(t4)
    Q1L_T(t5)
#if TG_Q1L_STATS
    const uint64_t t6 = __builtin_amdgcn_s_memtime();
    st[0] += t1 - t0;
    st[1] += t2 - t1;
    st[2] += t3 - t2;
    st[3] += t4 - t3;
    st[4] += t5 - t4;
    st[5] += t6 - t5;
#endif
  }
#if TG_Q1L_STATS
  if (tid == 0) {
    for (int x = 0; x < 6; ++x) atomicAdd(&g_q1l_stats[x], (unsigned long long)st[x]);
    atomicAdd(&g_q1l_stats[6], (unsigned long long)a.nops);
  }
#endif
  for (int e = tid; e < Q1R * 16; e += 64 * Q1W) {
    const int r = e >> 4, col = e & 15, row = R0 + r;
    if (row < n && col < k) Zb[int64_t(row) * ld + col] = sm.Zs[r][col];
  }
}

}  // namespace

namespace tg {

int sb_smax(int n);

// ops: host-built step list; dev: >= ops.size() * sizeof(Q1Op) + FEW_HDR
// bytes of device scratch (control words: step counter, timeout flag, bt_few's
// XCD election [2..4], q1_lds arrivals [5], bt_few stats [8..23], q1_lds's XCD
// election [24..27], the column slabs' q1_lds arrivals [64 + 16 s]).
constexpr int FEW_HDR = 1024;
constexpr int FEW_SLABS = 8;  // 16-column slabs of the LDS-resident kernels: k <= 128
static_assert(64 + 16 * FEW_SLABS <= FEW_HDR / 4, "slab counters fit the header");
static size_t few_ops_bytes(const SbPlan &pl) {
  size_t c = 0;
  for (const SbPanel &P : pl.panels) c += size_t(P.nl);
  return (FEW_HDR + c * sizeof(Q1Op) + 255) & ~size_t(255);
}
static int few_nsub(const SbPlan &pl) {  // + 1: sub-chunks are row-aligned, not panel-aligned
  return pl.single && !pl.panels.empty() ? cdiv(pl.panels[0].m, Q1S) + 1 : 0;
}
// Column slabs (k > 16: TG_BT_SLABS=0 keeps bt_few for k = 17 .. 32): both
// LDS kernels take 16 columns a workgroup, slabs side by side in blockIdx.y,
// as many a launch as leave every workgroup a CU of its own (their spins need
// all resident); q1_lds's at most Q1_SLABS at once (partials per slab)
constexpr int Q1_SLABS = 3;
static int xcd_all_cus() {
  const XcdInfo x = xcd_info();
  return x.xcds * x.cus_per_xcd;
}
static bool few_slabs(int k) {
  if (k <= 16) return false;
  const char *e = getenv("TG_BT_SLABS");  // development switch, read per call
  return !(e && e[0] == '0');
}
static int q1_conc(int n, int k) {
  if (!few_slabs(k)) return 1;
  return std::max(1, std::min({cdiv(k, 16), Q1_SLABS, xcd_all_cus() / std::max(1, cdiv(n, Q1R))}));
}
static size_t few_part_bytes(const SbPlan &pl, int n, int k) {
  if (!pl.single || pl.panels.empty()) return 0;
  const size_t lds_form = size_t(q1_conc(n, k)) * 2 * cdiv(n, Q1R) * 512 * sizeof(double);
  return std::max(size_t(few_nsub(pl)) * SB_B * SB_B * sizeof(double), lds_form);
}
// + one progress word per Q2 sweep group (n / 32 + 1) and column slab, 16-byte padded
size_t sb_apply_few_scratch(const SbPlan &pl, int n, int k) {
  const size_t slabs = few_slabs(k) ? size_t(cdiv(k, 16)) : 1;
  return few_ops_bytes(pl) + few_part_bytes(pl, n, k) +
         ((size_t(n / QB + 1) * slabs * 4 + 15) & ~size_t(15));
}
// can sb_apply_few take k columns?  k <= 32 always (bt_few_kernel); up to 128
// when the LDS-resident kernels fit (single-level plans, n / 128 workgroups <=
// CUs) in at most 4 launches of the two: each launch is a chain of n / 32
// dependent steps whatever its slabs, so past that the level-by-level
// sb_apply_q2 / sb_apply_q1 are faster (measured: n = 28,672, k = 102 in 7 + 7
// launches 201.7 ms against 109.5 ms; n = 4096, k = 100 in 1 + 3: 7.9 against
// 11.1 ms; n = 14,336, k = 51 in 2 + 2: 29.4 against 39.9 ms)
bool sb_apply_few_ok(const SbPlan &pl, int n, int k) {
  if (k < 1) return false;
  if (k <= 32) return true;
  const int cus = xcd_all_cus(), wq = cdiv(cdiv(n - 2, QB), QW), w1 = cdiv(n, Q1R);
  if (!few_slabs(k) || k > 16 * FEW_SLABS || !pl.single || n <= 2 || wq > cus || w1 > cus)
    return false;
  const int ns = cdiv(k, 16);
  return cdiv(ns, cus / wq) + cdiv(ns, q1_conc(n, k)) <= 4;
}

hipError_t sb_apply_few(hipStream_t st, int n, double *Z, int k, const SbPlan &pl,
                        const SbBufs &b, void *dev, bool *timed_out) {
  *timed_out = false;
  if (!sb_apply_few_ok(pl, n, k)) return hipErrorInvalidValue;
  const bool slabs = few_slabs(k);
  const int nslab = slabs ? cdiv(k, 16) : 1;
  std::vector<Q1Op> ops;
  for (auto it = pl.panels.rbegin(); it != pl.panels.rend(); ++it)
    for (int l = it->nl - 1; l >= 0; --l) {
      const SbLevel &L = it->L[l];
      ops.push_back(Q1Op{it->r0, L.rows, L.nc, l, int(L.yoff), int(L.toff)});
    }
  unsigned *cnt = static_cast<unsigned *>(dev);
  Q1Op *dops = reinterpret_cast<Q1Op *>(static_cast<char *>(dev) + FEW_HDR);
  hipError_t e = hipMemsetAsync(cnt, 0, FEW_HDR, st);
  if (e != hipSuccess) return e;
  if (!ops.empty()) {
    e = hipMemcpyAsync(dops, ops.data(), ops.size() * sizeof(Q1Op), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
  }
  const int nsw = n - 2;
  BtArgs a{};
  a.Z = Z;
  a.n = n;
  a.k = k;
  a.V2 = b.V2;
  a.T2 = b.T2;
  a.smax = sb_smax(n);
  a.ng2 = nsw > 0 ? cdiv(nsw, QB) : 0;
  a.nlev2 = nsw > 0 ? a.smax + a.ng2 - 1 : 0;
  a.Y = b.Y;
  a.T = b.T;
  a.ops = dops;
  a.nops = int(ops.size());
  a.single = pl.single ? 1 : 0;
  a.part = reinterpret_cast<double *>(static_cast<char *>(dev) + few_ops_bytes(pl));
  a.cnt = cnt;
  a.timeout = spin_timeout_ticks("TG_BT_TIMEOUT_TICKS");
  a.colflag = reinterpret_cast<unsigned *>(static_cast<char *>(dev) + few_ops_bytes(pl) +
                                           few_part_bytes(pl, n, k));
  {
    const char *qw = getenv("TG_BT_Q2_WAVE");  // development switch, read per call
    a.q2_wave = (qw && qw[0] == '1') ? 1 : 0;
  }
  if (a.q2_wave && a.ng2 > 0) {
    e = hipMemsetAsync(a.colflag, 0, ((size_t(a.ng2) * 4 + 15) & ~size_t(15)), st);
    if (e != hipSuccess) return e;
  }
  // Q2 with Z in LDS (q2_lds_kernel; TG_BT_Q2_LDS=0: the level-by-level Q2
  // inside bt_few_kernel): one workgroup of QW pair columns per CU, all
  // resident (one per CU by their LDS), so at most one per CU of the device
  const XcdInfo xq = xcd_info();
  {
    const char *ql = getenv("TG_BT_Q2_LDS");  // development switch, read per call
    const int Wq = cdiv(a.ng2, QW);
    // (one 16-column block a workgroup: with two, registers spill at the
    // 256-VGPR cap of two waves per SIMD; k > 16 in column slabs, or with
    // TG_BT_SLABS=0 bt_few's Q2 for k = 17 .. 32)
    const bool q2l = !(ql && ql[0] == '0') && !a.q2_wave && a.nlev2 > 0 && (k <= 16 || slabs) &&
                     Wq <= xq.xcds * xq.cus_per_xcd;
    if (!q2l && k > 32) return hipErrorInvalidValue;
    if (q2l) {
      e = hipMemsetAsync(a.colflag, 0, ((size_t(a.ng2) * nslab * 4 + 15) & ~size_t(15)), st);
      if (e != hipSuccess) return e;
      Q2LArgs qa{Z, n, k, b.V2, b.T2, a.smax, a.ng2, a.colflag, cnt + 1, a.timeout, 0};
      const int c2 = std::max(1, std::min(nslab, xq.xcds * xq.cus_per_xcd / Wq));
      auto tq = prof_begin(st, PROF_Q2, 0.0, 0.0);
#if TG_Q2L_STATS
      {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_q2l_stats), z, sizeof(z), 0,
                                     hipMemcpyHostToDevice, st);
      }
#endif
      for (qa.slab0 = 0; qa.slab0 < nslab; qa.slab0 += c2) {
        hipLaunchKernelGGL(q2_lds_kernel<1>, dim3(Wq, std::min(c2, nslab - qa.slab0)), dim3(64 * QW),
                           0, st, qa);
        if ((e = hipGetLastError()) != hipSuccess) return e;
      }
      prof_end(st, tq);
#if TG_Q2L_STATS
      {
        unsigned long long h[8];
        (void)hipStreamSynchronize(st);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_q2l_stats), sizeof(h));
        const double nbk = double(h[4] ? h[4] : 1);
        fprintf(stderr, "q2_lds n=%d: %llu blocks; cycles per block: wait %.0f, tile+V %.0f, "
                "mfma %.0f, store+publish %.0f\n", n, h[4], h[0] / nbk, h[1] / nbk, h[2] / nbk,
                h[3] / nbk);
      }
#endif
      a.nlev2 = 0;  // bt_few_kernel: Q1 only
      // Q1 with Z in LDS as well (single-level plans; TG_BT_Q1_LDS=0: bt_few's)
      const char *q1l = getenv("TG_BT_Q1_LDS");  // development switch, read per call
      // (n <= 4096: the workgroups of one XCD; larger n: one workgroup per CU
      // of the device, placement-independent hand-offs)
      const int W1 = cdiv(n, Q1R);
      const bool q1l2 = W1 <= xq.cus_per_xcd && k <= 16;  // (column slabs: the other form)
      const bool q1 = !(q1l && q1l[0] == '0') && a.single && a.nops > 0 &&
                      (q1l2 || W1 <= xq.xcds * xq.cus_per_xcd);
      if (!q1 && k > 32) return hipErrorInvalidValue;
      if (q1) {
        // partials in bt_few's sub-chunk partial area; arrivals in cnt[5]
        // (column slabs: cnt[64 + 16 s]), the XCD election in cnt[24..27]
        Q1LArgs la{Z, n, k, b.Y, b.T, dops, a.nops, a.part, q1l2 ? cnt + 5 : cnt + 64, cnt + 24,
                   cnt + 1, W1, a.timeout, 0};
        auto t1 = prof_begin(st, PROF_Q1, 0.0, 0.0);
        // TG_BT_Q1_LDS=2 (tests): a grid of W1 only, spread over the XCDs, so
        // the election comes up short and the bt_few fallback runs
        if (q1l2) {
          const int g1 = (q1l && q1l[0] == '2') ? W1 : W1 * xq.xcds;
          hipLaunchKernelGGL(q1_lds_kernel<true>, dim3(g1), dim3(64 * Q1W), 0, st, la);
          if ((e = hipGetLastError()) != hipSuccess) return e;
        } else {
          // slabs a launch: each its own arrival counter, partials reused by
          // the next launch (stream order)
          const int c1 = q1_conc(n, k);
          for (la.slab0 = 0; la.slab0 < nslab; la.slab0 += c1) {
            hipLaunchKernelGGL(q1_lds_kernel<false>, dim3(W1, std::min(c1, nslab - la.slab0)),
                               dim3(64 * Q1W), 0, st, la);
            if ((e = hipGetLastError()) != hipSuccess) return e;
          }
        }
        prof_end(st, t1);
        // did the workers land on one XCD?  (the sync is the one the
        // all-LDS path makes anyway to read the timeout flag)
        unsigned h[28];
        e = hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);  // also: ops read before they go
        if (e != hipSuccess) return e;
        *timed_out = h[1] != 0u;
        if (*timed_out) return hipSuccess;
#if TG_Q1L_STATS
        {
          unsigned long long q[8];
          (void)hipMemcpyFromSymbol(q, HIP_SYMBOL(g_q1l_stats), sizeof(q));
          const double ns = double(q[6] ? q[6] : 1);
          fprintf(stderr, "q1_lds n=%d: %llu worker-steps; cycles per step: stage + partials %.0f, "
                  "drain %.0f, exchange %.0f, P sum + M + update %.0f\n", n, q[6], q[0] / ns,
                  q[1] / ns, q[2] / ns, q[3] / ns + q[4] / ns + q[5] / ns);
          const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          (void)hipMemcpyToSymbol(HIP_SYMBOL(g_q1l_stats), z, sizeof(z));
        }
#endif
        if (h[27] == 0u) return hipSuccess;  // done: Q2 and Q1 both ran with Z in LDS
        // not placed: Z untouched, bt_few_kernel's Q1 below
      }
    }
  }
  // one wave per Q2 block of the widest level, one workgroup per TSQR chunk
  int W = std::min(256, std::max(std::max(std::max(1, cdiv(a.smax, BW)), pl.ncmax), few_nsub(pl)));
  // the workers (one CU each: BtShared fills the LDS) must all be resident:
  // in the XCD form they are workgroups of one XCD, so at most its CUs
  // (sub-chunks beyond W are taken in turn by the loops)
  const XcdInfo xi = xcd_info();
  if (TG_BT_XCD) W = std::min(W, xi.cus_per_xcd);
  a.wexp = W;
  if (a.nlev2 == 0 && a.nops == 0 && !a.q2_wave) {
    // everything ran in the LDS-resident kernels: only the timeout flag to read
    unsigned h2[2] = {0u, 0u};
    e = hipMemcpyAsync(h2, cnt, sizeof(h2), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);  // also: ops read before it goes
    *timed_out = h2[1] != 0u;
    return e;
  }
  auto tok = prof_begin(st, a.nlev2 > 0 ? PROF_Q2 : PROF_Q1, 0.0, 0.0);
  const int grid = TG_BT_XCD ? xi.xcds * W : W;  // XCD form: W land on each XCD
  if (a.q2_wave) {
    if (k <= 16)
      hipLaunchKernelGGL((bt_few_kernel<1, true>), dim3(grid), dim3(64 * BW), 0, st, a);
    else
      hipLaunchKernelGGL((bt_few_kernel<2, true>), dim3(grid), dim3(64 * BW), 0, st, a);
  } else {
    if (k <= 16)
      hipLaunchKernelGGL((bt_few_kernel<1, false>), dim3(grid), dim3(64 * BW), 0, st, a);
    else
      hipLaunchKernelGGL((bt_few_kernel<2, false>), dim3(grid), dim3(64 * BW), 0, st, a);
  }
  prof_end(st, tok);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  unsigned h[24] = {0};
  e = hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);  // also: ops read before it goes
  *timed_out = h[1] != 0u;
#ifdef TG_BT_STATS
  const unsigned long long *q = reinterpret_cast<const unsigned long long *>(h + 8);
  fprintf(stderr, "bt_few: W %u  Q2 work %.3f ms barrier %.3f ms (%d levels)  Q1 work %.3f ms "
          "barrier %.3f ms (%d steps)\n", h[3], q[0] / 1e5, q[1] / 1e5, a.nlev2, q[2] / 1e5,
          q[3] / 1e5, a.nops);
#endif
  return e;
}

}  // namespace tg
