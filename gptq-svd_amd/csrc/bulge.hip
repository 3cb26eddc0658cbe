// Stage 2 of the two-stage eigensolver: band (half-bandwidth b = SB_B) ->
// symmetric tridiagonal by bulge chasing, plus the back-transformation Q2.
//
// Second half of the reduction inside `torch.linalg.eigh`
// (/root/reference/src/TruncGPTQ/gptq_utils.py:92).  Algorithm (one column
// per sweep): sweep j, task s takes the reflector rows R = [r1, r1 + b),
// r1 = j + 1 + s b, annihilating column j (s = 0) or the first bulge column
// r1 - b (s > 0), and applies it two-sided to the window [r1 - b, r1 + 2b):
//   B[R, Lft] <- H B[R, Lft],  B[R, R] <- H B[R, R] H,  B[Rgt, R] <- B[Rgt, R] H.
// Task (j, s) overlaps sweep j-1's tasks s-1 .. s+2, but its overlap with
// (j-1, s+2) is the single element B[r1 + 2b - 1][r1 + b - 1], the pivot of
// (j-1, s+2), whose final value (beta, zeros below) is known one task early:
// the wave that forms a reflector writes its pivot column at once (the G wave
// of (j, s-1) for s > 0, first_refl for s = 0) and the left-block wave skips
// it.  So sweeps run as a pipeline with a lag of LAG = 2 tasks (3 if every
// write stayed with its task).  GPU mapping: three waves per task; a
// workgroup owns G_SW consecutive sweeps and advances them in lock-step
// (pair q runs task t - LAG q at step t; the tasks of one step are disjoint).
// Workgroups hand over through a per-group step counter.
//
// Band storage (lower, with bulge room): Bst[c * LDB + d] = B[c + d][c],
// d < 2b.  Reflector of (j, s): the b-double record V2[(j * smax + s) * b ..]
// holds tau in element 0 (v_0 = 1 is implicit) and v_1 .. v_{b-1} after it,
// written as one 256-B line pair of 16-B stores.
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

#include "../../include/truncgptq.h"
#include "band.h"
#include "common.h"
#include "spin.h"

namespace {

using tg::SB_B;
constexpr int LDB = 2 * SB_B;

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
// Full wave sum in every lane without the LDS crossbar: pairings lane^32,
// lane^16 (permlane swaps), lane^15 / lane^7 (DPP row mirrors), lane^3,
// lane^1 (quad_perm) flip a new bit each.
__device__ inline double wsum(double s) {
  s = hsum32(s);
  s = hsum16(s);
  s += xdpp<0x140>(s);
  s += xdpp<0x141>(s);
  s += xdpp<0x1B>(s);
  s += xdpp<0xB1>(s);
  return s;
}

__device__ inline int ntasks(int n, int j) { return (j <= n - 3) ? (n - 3 - j) / SB_B + 1 : 0; }

// ---------------------------------------------------------------------------
// LDS-resident pipeline.  A workgroup owns G_SW consecutive sweeps; at step t
// pair q runs task t - LAG q.  The band columns the group touches at step t
// span [low(t), high(t)), so the group keeps them in an LDS ring of RING band
// columns (64 doubles each): each step the loader wave brings in the b
// columns step t+1 adds, and the writer wave writes back the columns no later
// task of the group touches.
//
// Hand-off to the next group (progress word prog[G] = steps whose retired
// columns are in memory):
//   producer (writer wave): plain 16-B stores of the retired columns ->
//     s_waitcnt vmcnt(0) (every store acknowledged by the XCD's L2) ->
//     progress store (TG_BULGE_FLAG_L2=1: plain `sc0` store, the line stays
//     in that L2; 0: relaxed agent `sc1` store, written through);
//   consumer (loader wave): relaxed agent `sc1` poll of prog[G-1] (L1
//     bypassed) until it covers the columns of the next step, then `sc1`
//     16-B buffer loads of those columns (L1 bypassed, served by the L2).
// Every store of the band and every load of it go through ONE L2: the
// workgroups read HW_REG_XCC_ID, the first arrival fixes the XCD and the
// workgroups of the other XCDs exit before touching the band.  The XCD's L2
// is the point of coherence of all its CUs and nothing in this hand-off is
// cached in an L1, so no agent-scope release (an L2 write-back to HBM, >= 1.7
// us per step, MI355X_MICROARCH.md price list) or acquire (an L1 invalidate
// the sc1 loads make unnecessary) is needed.  The order is enforced where the
// compiler could break it: the vmcnt wait is an asm with a memory clobber
// before the progress store, and the column loads are issued after the poll
// returns (they depend on it through the wave barrier).
// (A form with the workers of every XCD -- write-through band stores, `sc1`
// progress words -- gave bit-identical eigenvalues but was slower: 112 vs
// 83 ms at n = 12,288, 449 vs 378 ms at 28,672, every step's transfers going
// to memory instead of the XCD's L2; its template also cost the one-XCD
// kernel 1 ms at n = 4096 through a different schedule, so it was removed.)
// Workers take sweep groups from a queue in increasing order (dependencies
// point only to lower groups, so any number of resident workers is safe).
// Waits are bounded (spin.h): the first wait past the timeout sets the stall
// word, every later wait of the launch gives up at once, and the host
// poisons (d, e) with NaN.
// ---------------------------------------------------------------------------
#ifndef TG_BULGE_GSW
#define TG_BULGE_GSW 2
#endif
#ifndef TG_BULGE_FLAG_L2
#define TG_BULGE_FLAG_L2 1
#endif
#ifndef TG_BULGE_SPLIT
#define TG_BULGE_SPLIT 3  // bit 0: wave 0 takes half of the write-back; bit 1: wave 3 half of the load
#endif
#ifndef TG_BULGE_STATS
#define TG_BULGE_STATS 0  // per-step s_memrealtime stamps (build-time: they slow every step)
#endif
constexpr int G_SW = TG_BULGE_GSW;   // sweeps per group (wave triples per workgroup)
constexpr int LAG = 2;               // pipeline lag between consecutive sweeps (tasks)
constexpr int RING = 256;            // ring slots (power of two)
// live columns: the tasks of step t, the columns step t-1 retired (being
// written back) and the columns step t+1 adds (being loaded):
// high(t+1) - low(t-1) = (4 + LAG (G_SW - 1)) b - G_SW
static_assert((4 + LAG * (G_SW - 1)) * 32 - G_SW <= RING, "LDS ring too small for G_SW");
constexpr int NCW = 3 * G_SW;        // compute waves (three per sweep: left, diagonal, lower block)
constexpr int BT = 64 * (NCW + 2);   // + a writer wave and a loader wave

struct WaveScratch {
  double ws[SB_B];
  double trash[64];  // target of the masked (upper-triangle) stores of the D update
};

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline int rslot(int c) { return c & (RING - 1); }

// Task (j, s) by three waves on the LDS ring (element (r, c) at
// R[slot(c)][r - c]): role 0 applies the reflector to the left block
// A = B[R, Lft] (and stores it for Q2), role 1 to the diagonal block
// D = B[R, R], role 2 to the lower block G = B[Rgt, R].  The blocks are
// disjoint, so the waves never exchange data.  No wave reads the pivot
// column the role-0 wave overwrites: the reflector of (j, s > 0) annihilates
// the first column of the G block (j, s-1) just updated, so the role-2 wave
// of (j, s-1) forms it from its registers and forwards (v, tau, beta) through
// LDS (`rin` / `rout`, double-buffered by step); that of (j, 0) is formed one
// step ahead by the same (then idle) role-2 wave (`first_refl`).
struct Refl {
  double v[SB_B];
  double tau, beta;
  double tu[SB_B];  // dataflow kernel: tau u of the lower block (row-indexed), see df_task
};

__device__ __forceinline__ void make_refl(double x, int li, int hf, double &v, double &tau,
                                          double &beta) {
  const double sig = wsum((hf == 0 && li >= 1) ? x * x : 0.0);
  const double alpha = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                                        __builtin_amdgcn_readfirstlane(__double2loint(x)));
  double scal = 0.0;
  tau = 0.0;
  beta = alpha;
  if (sig != 0.0) {
    beta = -copysign(sqrt(alpha * alpha + sig), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
  }
  v = (li == 0) ? 1.0 : x * scal;
}

// Reflector of task (j, 0) (x = B[j+1 .. j+b, j], final once task (j-1, 0)
// has run: its G wave wrote B[j+b][j]), formed one step ahead by one wave,
// which also writes the annihilated column (beta, 0, ..., 0).
__device__ __forceinline__ void first_refl(double (*R)[LDB], int n, int j, Refl &out) {
  const int lane = threadIdx.x & 63, li = lane & 31, hf = lane >> 5;
  const int r1 = j + 1, L = min(SB_B, n - r1);
  const double x = R[rslot(j)][1 + min(li, L - 1)];
  double v, tau, beta;
  make_refl(li < L ? x : 0.0, li, hf, v, tau, beta);
  if (hf == 0 && li < L) R[rslot(j)][1 + li] = (li == 0) ? beta : 0.0;
  if (hf == 0) out.v[li] = v;
  if (lane == 0) {
    out.tau = tau;
    out.beta = beta;
  }
}


// The reflector record (tau, v_1, .., v_{b-1}) by 16 lanes, 16 B each, as
// non-temporal stores: the 68 MB record stream (n = 4096) is read back only
// by the back-transform, and in the default policy it pushed the L2-resident
// band's dirty lines out to memory (WRITE_SIZE 2x the record bytes).
__device__ __forceinline__ void store_refl(double *rec, const Refl &r, int lane) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  if (lane < SB_B / 2) {
    const double x0 = lane == 0 ? r.tau : r.v[2 * lane];
    __builtin_nontemporal_store(d2{x0, r.v[2 * lane + 1]}, reinterpret_cast<d2 *>(rec) + lane);
  }
}

template <bool FULL>
__device__ __forceinline__ void bulge_task_lds(double (*R)[LDB], int n, int j, int s, int role,
                                               bool has_next, double *__restrict__ V2, int smax,
                                               WaveScratch &W, const Refl &rin, Refl &rout) {
  const int lane = threadIdx.x & 63, li = lane & 31, hf = lane >> 5;
  const int r1 = j + 1 + s * SB_B;
  const int L = FULL ? SB_B : min(SB_B, n - r1);
  const int col = (s == 0) ? j : r1 - SB_B;
  const int lo = FULL ? r1 - SB_B : max(0, r1 - SB_B);
  const int nl = FULL ? SB_B : r1 - lo;
  const int ng = FULL ? SB_B : min(SB_B, n - (r1 + L));
  double *Rf = &R[0][0];
  auto at = [&](int c, int d) { return rslot(c) * LDB + d; };
  if (role == 0 && s == 0) {
    // the left block of (j, 0) is column j (written by first_refl) next to
    // columns that are already tridiagonal (zero in rows R): nothing to apply
    store_refl(V2 + int64_t(j) * smax * SB_B, rin, lane);
    return;
  }
  // block loads (issued before the reflector is needed)
  double e[16];  // role 0: A (lane column c = li, rows hf + 2q); role 1: D (lane row li,
                 // k = hf + 2q); role 2: G (lane row li, k = hf + 2q)
  if (role == 0) {
    const int ca = FULL ? li : min(li, max(nl - 1, 0));
    const int abase = at(lo + ca, r1 - lo - ca);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = hf + 2 * q;
      if (FULL) e[q] = Rf[abase + i];
      else e[q] = (li < nl && i < L) ? Rf[abase + min(i, L - 1)] : 0.0;
    }
  } else if (role == 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      const int cc = min(li, k), off = li > k ? li - k : k - li;
      if (FULL) e[q] = Rf[at(r1 + cc, off)];
      else e[q] = (li < L && k < L) ? Rf[at(r1 + min(cc, L - 1), off)] : 0.0;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      if (FULL) e[q] = Rf[at(r1 + k, SB_B + li - k)];
      else {
        const int kc = min(k, L - 1);
        const double gv = Rf[at(r1 + kc, L + min(li, max(ng - 1, 0)) - kc)];
        e[q] = (li < ng && k < L) ? gv : 0.0;
      }
    }
  }
  const double v = rin.v[li], tau = rin.tau;
  double vk[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) vk[q] = rin.v[hf + 2 * q];
  if (role == 2) {
    // lower block: u_r = sum_k G[r][k] v_k, G -= tau u v^T (row r = li)
    double u0 = 0.0, u1 = 0.0, u2 = 0.0, u3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      u0 += e[q] * vk[q];
      u1 += e[q + 1] * vk[q + 1];
      u2 += e[q + 2] * vk[q + 2];
      u3 += e[q + 3] * vk[q + 3];
    }
    double u = (u0 + u1) + (u2 + u3);
    u = hsum32(u);
    const double tu = tau * u;
#pragma unroll
    for (int q = 0; q < 16; ++q) e[q] = e[q] - tu * vk[q];
    if (has_next) {
      // next reflector: x = updated column 0 of G (lanes hf == 0 hold G[li][0]);
      // that column is stored as its final (beta, 0, ..., 0) right away
      double vn, tn, bn;
      make_refl((FULL || li < ng) ? e[0] : 0.0, li, hf, vn, tn, bn);
      if (hf == 0) {
        rout.v[li] = vn;
        e[0] = (li == 0) ? bn : 0.0;
      }
      if (lane == 0) {
        rout.tau = tn;
        rout.beta = bn;
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      if (FULL || (li < ng && k < L)) Rf[at(r1 + k, L + li - k)] = e[q];
    }
  } else if (role == 0) {
    // left block: w_c = sum_i v_i A[i][c]
    double w0 = 0.0, w1 = 0.0, w2 = 0.0, w3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      w0 += vk[q] * e[q];
      w1 += vk[q + 1] * e[q + 1];
      w2 += vk[q + 2] * e[q + 2];
      w3 += vk[q + 3] * e[q + 3];
    }
    double wc = (w0 + w1) + (w2 + w3);
    wc = hsum32(wc);
    // the pivot column (lo + c == col, s > 0) was written by the G wave of
    // (j, s-1) when it formed this reflector
    if ((FULL || li < nl) && lo + li != col) {
      const int c = li;
      double *Ac = Rf + at(lo + c, r1 - lo - c);
      const double twc = tau * wc;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = hf + 2 * q;
        if (FULL || i < L) Ac[i] = e[q] - twc * vk[q];
      }
    }
    store_refl(V2 + (int64_t(j) * smax + s) * SB_B, rin, lane);
  } else {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      p0 += e[q] * vk[q];
      p1 += e[q + 1] * vk[q + 1];
      p2 += e[q + 2] * vk[q + 2];
      p3 += e[q + 3] * vk[q + 3];
    }
    double p = (p0 + p1) + (p2 + p3);
    p = hsum32(p);
    p *= tau;
    const double pv = wsum(hf == 0 ? p * v : 0.0);
    const double w = p - 0.5 * tau * pv * v;
    if (hf == 0) W.ws[li] = w;
    wave_sync();
    double wk[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) wk[q] = W.ws[hf + 2 * q];
    // branch-free: lanes outside the lower triangle store to a trash slot
    double *tr = W.trash + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      const bool ok = (FULL || li < L) && k <= li;
      double *dst = ok ? Rf + at(r1 + k, li - k) : tr;
      *dst = e[q] - v * wk[q] - w * vk[q];
    }
  }
}

__device__ inline int group_steps(int n, int nsw, int G) {
  const int j0 = G * G_SW;
  const int g = min(G_SW, nsw - j0);
  return LAG * (g - 1) + ntasks(n, j0);
}

// Lowest column any task of the group touches at step >= t (n if none):
// sweep j touches column j in first_refl (s = -1), columns >= r1 = j + 1 in
// task 0, and columns >= r1 - b + 1 in task s > 0 (the pivot column r1 - b
// is final before the task starts).
__device__ inline int group_low(int n, int nsw, int j0, int g, int t) {
  int lowc = n;
  for (int q = 0; q < g; ++q) {
    const int j = j0 + q;
    const int s = t - LAG * q;
    if (s >= ntasks(n, j)) continue;
    const int c = (s < 0) ? j : (s == 0) ? j + 1 : j + 2 + (s - 1) * SB_B;
    lowc = min(lowc, c);
  }
  return lowc;
}
// Producer step the consumer group needs before it may load the columns of
// its step t: low_{G-1}(T) >= high_G(t) for T >= t + 2 + LAG (G_SW - 1).
__device__ inline int group_need(int t) { return t + 2 + LAG * (G_SW - 1); }
// One past the highest column any task of the group touches at steps <= t.
__device__ inline int group_high(int n, int j0, int t) {
  return min(n, j0 + 1 + (t + 1) * SB_B);
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Lane-0 operations without a lane-0 branch.  A `if (tid == 0)` block next to
// the group loop's back edge let the compiler's CFG structurizer give lane 0
// of wave 0 a loop nest of its own (it left the inner loop through an exec
// mask at the group end and re-entered at the group take), so that wave
// executed the group's barriers once for lane 0 and once for lanes 1-63 and
// the workgroup deadlocked (diagnosed with a per-wave live-lane heartbeat:
// wave 0 ran with 63 lanes).  Every lane of the wave executes these: lane 0
// on the real word, the others on a private dummy word of their own.
__device__ __forceinline__ unsigned *lane0_or_dummy(unsigned *real, unsigned *dummy, int wlane) {
  return wlane == 0 ? real : dummy + wlane;
}

__device__ __forceinline__ void publish(unsigned *p, unsigned v) {
#if TG_BULGE_FLAG_L2
  __hip_atomic_store((tg::spin_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  tg::ctl_store(p, v);
#endif
}

#if TG_BULGE_STATS
#define BSTAMP(v) const uint64_t v = __builtin_amdgcn_s_memrealtime();
#else
#define BSTAMP(v)
#endif
#ifndef TG_BULGE_HB
#define TG_BULGE_HB 0  // debug: per-wave heartbeat (group, step, phase) into host memory
#endif
#if TG_BULGE_HB
// record (group, step, live lanes, phase) from the first active lane
#define HB(ph)                                                                          \
  {                                                                                     \
    const unsigned long long ex_ = __builtin_amdgcn_read_exec();                        \
    if (int(__lane_id()) == __builtin_ctzll(ex_))                                       \
      ((volatile unsigned long long *)stats)[blockIdx.x * 16 + wid] =                   \
          (unsigned long long)(G + 1) << 32 | (unsigned long long)(t + 1) << 16 |       \
          (unsigned long long)__builtin_popcountll(ex_) << 8 | (ph);                    \
  }
#else
#define HB(ph)
#endif

// ctl[0] = chosen XCD + 1, ctl[1] = group queue, ctl[2] = stall word
__global__ __launch_bounds__(BT) void bulge_lds_kernel(double *__restrict__ B, int n,
                                                       double *__restrict__ V2, int smax,
                                                       unsigned *__restrict__ prog,
                                                       unsigned *__restrict__ ctl,
                                                       unsigned long long *__restrict__ stats,
                                                       unsigned long long timeout) {
#if TG_BULGE_STATS
  uint64_t sw = 0, stk = 0, sbar = 0, nsteps = 0;
  const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  __shared__ double R[RING][LDB];
  __shared__ WaveScratch wsc[NCW];
  __shared__ Refl rfl[G_SW][2];
  __shared__ int sh_G;
  __shared__ int sh_dead;  // a wait of this workgroup gave up: no further waits
  __shared__ unsigned sh_wdone[2];  // write-back half h drained for step number sh_wdone[h] - 1
  // wave index as an SGPR: every role branch below is a scalar (SCC) branch, no exec masks
  const int tid = threadIdx.x, wlane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned *stall = ctl + 2;
  unsigned *dummy = ctl + 4;  // 64 words: the lanes 1-63 targets of lane-0 operations
  if (tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    unsigned expect = 0;
    __hip_atomic_compare_exchange_strong(ctl, &expect, x + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const unsigned chosen = expect == 0 ? x + 1 : expect;
    sh_G = (chosen == x + 1) ? 0 : -1;
    sh_dead = 0;
    sh_wdone[0] = sh_wdone[1] = 0;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(sh_G) < 0) return;  // uniform: no exec-masked kernel body
  const int nsw = n - 2;
  const int ngroups = tg::cdiv(nsw, G_SW);
  const int bytes = n * LDB * int(sizeof(double));
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(B, 0, bytes, 0x00020000);
  constexpr int SC1 = 16;                 // cache policy bit of the L1-bypassing loads
  constexpr int NTC = LDB / 2;            // 16-B chunks per column
  constexpr int PFN = SB_B * NTC / BT + 1;  // chunks per thread of a whole-workgroup load
  // halves of each step's write-back (NH) and load (NHL), 1 KB blocks by parity
  constexpr int NH = (TG_BULGE_SPLIT & 1) ? 2 : 1;
  constexpr int NHL = (TG_BULGE_SPLIT & 2) ? 2 : 1;
  constexpr int NBLK = SB_B * NTC / 64;  // 1 KB blocks per step's load
  constexpr int PW = NBLK / NHL;         // blocks (chunks per lane) of one load half
  unsigned nstep = 0;  // steps this workgroup has run over all its groups (sh_wdone's clock)
  while (true) {
    if (wid == 0) {
      // a stalled launch: stop taking groups (the results are poisoned anyway)
      const unsigned v = atomicAdd(lane0_or_dummy(ctl + 1, dummy, wlane), 1u);
      const int Gn = tg::ctl_load(stall) ? ngroups : int(__builtin_amdgcn_readfirstlane(v));
      sh_G = Gn;  // every lane writes the same value
    }
    __syncthreads();
    // scalar (SGPR) copy: every loop bound below is wave-uniform to the compiler too,
    // so the step loop is a plain scalar loop around its barrier
    const int G = __builtin_amdgcn_readfirstlane(sh_G);
    __syncthreads();
    if (G >= ngroups) break;
    const int j0 = G * G_SW;
    const int g = min(G_SW, nsw - j0);
    const int total = group_steps(n, nsw, G);
    const int ptotal = G > 0 ? group_steps(n, nsw, G - 1) : 0;
    // progress of the producer group known to this thread (the loader wave's
    // lanes and the group-start wait keep it; ptotal + 1 = finished + written back)
    unsigned known = __builtin_amdgcn_readfirstlane((G > 0) ? 0u : ~0u);
    // one whole wave: wait until the producer published `need` (wave-uniform)
    auto wait_wave = [&](unsigned need) -> unsigned {
      unsigned seen = 0;
      if (!__builtin_amdgcn_readfirstlane(sh_dead) &&
          !tg::spin_geq(prog + G - 1, need, stall, timeout, &seen))
        sh_dead = 1;
      return seen;
    };
    // initial window [j0, high(0)): every thread loads, after one wait
    {
      const unsigned need = unsigned(min(group_need(0), ptotal + 1));
      BSTAMP(tw)
      if (G > 0 && wid == 0) wait_wave(need);
      __syncthreads();
      if (G > 0) known = need;
#if TG_BULGE_STATS
      sw += __builtin_amdgcn_s_memrealtime() - tw;
#endif
    }
    const int h0 = group_high(n, j0, 0);
    for (int c0 = j0; c0 < h0; c0 += SB_B) {
      const int c1 = min(c0 + SB_B, h0);
      double2 pf[PFN];
#pragma unroll
      for (int u = 0; u < PFN; ++u) {
        const int idx = tid + u * BT;
        const int c = min(c0 + idx / NTC, c1 - 1), h = idx % NTC;
        const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rb, (c * LDB + 2 * h) * 8, 0, SC1);
        pf[u] = make_double2(__builtin_bit_cast(double, u32x2{v4[0], v4[1]}),
                             __builtin_bit_cast(double, u32x2{v4[2], v4[3]}));
      }
#pragma unroll
      for (int u = 0; u < PFN; ++u) {
        const int idx = tid + u * BT;
        const int c = c0 + idx / NTC, h = idx % NTC;
        if (c < c1 && idx < SB_B * NTC) {
          R[rslot(c)][2 * h] = pf[u].x;
          R[rslot(c)][2 * h + 1] = pf[u].y;
        }
      }
    }
    int ld = h0, wb = j0;  // ring holds [wb, ld); every wave tracks both
    __syncthreads();
    if (wid == 2) first_refl(R, n, j0, rfl[0][0]);
    __syncthreads();
    for (int t = 0; t < total; ++t) {
      BSTAMP(c0t)
      HB(1)
      // Transfers of step t, each split in NH halves (64-chunk blocks by parity):
      // write-back of the columns step t-1 retired (drained, then the last half
      // to drain publishes t) and the load of the columns step t+1 adds (after
      // the producer's progress covers them).  One wave moves ~16 KB per
      // ~1.5 us, so with TG_BULGE_SPLIT the left-block waves (the lightest
      // tasks) take the second halves: wave 0 stores before its task, wave 3
      // loads after its task.
      auto wb_issue = [&](int half) {
        const int nl = group_low(n, nsw, j0, g, t);
        // wave-uniform trip count (scalar loop), the tail masked by an if
        const int lim = (nl - wb) * NTC;
        for (int b0 = 64 * half; b0 < lim; b0 += 64 * NH) {
          const int idx = b0 + wlane;
          if (idx < lim) {
            const int c = wb + idx / NTC, h = idx % NTC;
            const u32x2 lo2 = __builtin_bit_cast(u32x2, R[rslot(c)][2 * h]);
            const u32x2 hi2 = __builtin_bit_cast(u32x2, R[rslot(c)][2 * h + 1]);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo2[0], lo2[1], hi2[0], hi2[1]}, rb,
                                                   (c * LDB + 2 * h) * 8, 0, 0);
          }
        }
      };
      auto wb_finish = [&](int half) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (NH == 1) {
          publish(lane0_or_dummy(prog + G, dummy, wlane), unsigned(t));
        } else {
          // each half marks its word, then reads the other's: LDS serves one
          // CU's requests in order, so the later of the two sees both marks
          // (both publishing the same step is harmless)
          __hip_atomic_store(&sh_wdone[half], nstep + 1, __ATOMIC_SEQ_CST,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
          const unsigned o = __hip_atomic_load(&sh_wdone[half ^ 1], __ATOMIC_SEQ_CST,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          if (__builtin_amdgcn_readfirstlane(o) >= nstep + 1)
            publish(lane0_or_dummy(prog + G, dummy, wlane), unsigned(t));
        }
      };
      // the load as two parts (issue after the poll; LDS writes once the data is in)
      auto load_issue = [&](int half, double2 (&buf)[PW]) -> bool {
        const int nh = group_high(n, j0, t + 1);
        if (!(t + 1 < total && nh > ld)) return false;
        const unsigned need = unsigned(min(group_need(t + 1), ptotal + 1));
        if (known < need) {
          HB(4)
          // the column loads below issue after the poll has returned
          known = max(need, wait_wave(need));
          HB(5)
        }
#pragma unroll
        for (int u = 0; u < PW; ++u) {
          const int idx = wlane + 64 * (half + NHL * u);
          const int c = min(ld + idx / NTC, nh - 1), h = idx % NTC;
          const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rb, (c * LDB + 2 * h) * 8, 0, SC1);
          buf[u] = make_double2(__builtin_bit_cast(double, u32x2{v4[0], v4[1]}),
                                __builtin_bit_cast(double, u32x2{v4[2], v4[3]}));
        }
        return true;
      };
      auto load_finish = [&](int half, const double2 (&buf)[PW]) {
        const int nh = group_high(n, j0, t + 1);
#pragma unroll
        for (int u = 0; u < PW; ++u) {
          const int idx = wlane + 64 * (half + NHL * u);
          const int c = ld + idx / NTC, h = idx % NTC;
          if (c < nh) {
            R[rslot(c)][2 * h] = buf[u].x;
            R[rslot(c)][2 * h + 1] = buf[u].y;
          }
        }
        HB(10)
      };
      auto load_half = [&](int half) {
        double2 buf[PW];
        if (load_issue(half, buf)) load_finish(half, buf);
      };
      if (wid < NCW) {
        const int pair = wid / 3, role = wid % 3;
        const int s = t - LAG * pair;
        if (NH == 2 && wid == 0) wb_issue(1);
        if (pair < g && s >= 0 && s < ntasks(n, j0 + pair)) {
          const int jj = j0 + pair, r1 = jj + 1 + s * SB_B;
          const bool nx = s + 1 < ntasks(n, jj);
          const Refl &ri = rfl[pair][t & 1];
          Refl &ro = rfl[pair][(t + 1) & 1];
          HB(6)
          if (r1 >= SB_B && r1 + 2 * SB_B <= n)
            bulge_task_lds<true>(R, n, jj, s, role, nx, V2, smax, wsc[wid], ri, ro);
          else
            bulge_task_lds<false>(R, n, jj, s, role, nx, V2, smax, wsc[wid], ri, ro);
          HB(7)
        } else if (pair < g && pair > 0 && s == -1 && role == 2) {
          first_refl(R, n, j0 + pair, rfl[pair][(t + 1) & 1]);
        }
        if (NH == 2 && wid == 0) wb_finish(1);
        if (NHL == 2 && wid == 3) load_half(1);
      } else if (wid == NCW) {
        // writer: retire the columns step t-1 left behind, drain, publish t
        wb_issue(0);
        HB(8)
        wb_finish(0);
        HB(9)
      } else {
        // loader: the columns step t + 1 adds
        load_half(0);
      }
      BSTAMP(c1t)
      HB(2)
      __syncthreads();
      ++nstep;
      if (t + 1 < total) ld = max(ld, group_high(n, j0, t + 1));
      wb = max(wb, group_low(n, nsw, j0, g, t));
#if TG_BULGE_STATS
      const uint64_t c2t = __builtin_amdgcn_s_memrealtime();
      stk += c1t - c0t;
      sbar += c2t - c1t;
      ++nsteps;
      if (wlane == 0 && stats) atomicAdd(stats + 8 + wid, (unsigned long long)(c1t - c0t));
#endif
    }
    // group end: write back what is left, drain, publish done
    {
      const int lim = (ld - wb) * NTC;  // uniform trip count, masked tail
      for (int b0 = 0; b0 < lim; b0 += BT) {
        const int idx = b0 + tid;
        if (idx < lim) {
          const int c = wb + idx / NTC, h = idx % NTC;
          const u32x2 lo2 = __builtin_bit_cast(u32x2, R[rslot(c)][2 * h]);
          const u32x2 hi2 = __builtin_bit_cast(u32x2, R[rslot(c)][2 * h + 1]);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo2[0], lo2[1], hi2[0], hi2[1]}, rb,
                                                 (c * LDB + 2 * h) * 8, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wid == 0) publish(lane0_or_dummy(prog + G, dummy, wlane), unsigned(total + 1));
  }
#if TG_BULGE_STATS
  if (stats && tid == 0) {
    atomicAdd(stats + 0, 1ull);
    atomicAdd(stats + 1, (unsigned long long)sw);
    atomicAdd(stats + 2, (unsigned long long)stk);
    atomicAdd(stats + 3, (unsigned long long)sbar);
    atomicAdd(stats + 6, (unsigned long long)nsteps);
    // shader clock over the launch: s_memtime cycles per 100 MHz tick
    atomicAdd(stats + 4, (unsigned long long)(__builtin_amdgcn_s_memtime() - clk0));
    atomicAdd(stats + 5, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - rt0));
  }
#endif
}

// ---------------------------------------------------------------------------
// Dataflow form of the same pipeline (the default; TG_BULGE_DF=0 selects the
// step-synchronous kernel above).  The
// step-synchronous kernel above runs every task of a step behind one
// workgroup barrier, so a sweep advances by one task per slowest-wave step
// and the next sweep trails by LAG whole steps.  Here every role wave of
// every sweep runs its own task loop and waits only for the LDS progress
// counters it depends on (counts of finished tasks per sweep and role):
//   role 2 (G, + next reflector) of sweep q, task s:
//       own reflector v(s) (cntG[q] >= s + 1: step 0 is first_refl),
//       sweep q-1's A and D of task s + 1 (cntA/cntD[q-1] >= s + 2) and its
//       G of task s + 1 (the pivot beta of its task s + 2: cntG[q-1] >= s + 3),
//       a free reflector slot (cntA/cntD[q] >= s + 2 - DK);
//   role 0 (A) of task s: cntG[q] >= s + 1 (v(s) and the block G(s-1) = A(s));
//   role 1 (D) of task s: cntG[q] >= s + 1 and cntA/cntD[q-1] >= s + 2.
// Sweep 0 of a group takes "sweep q-1"'s data from the loader instead
// (columns [j0, loaded) of the ring hold the previous group's final values).
// These are the task-window overlaps of the LAG = 2 pipeline (file header):
// every hazard between the waves is read-after-write on those counters, so
// the tasks compute exactly what the step-synchronous kernel computes, in
// the same order on every element -- bit-identical d, e and reflectors.
// A loader wave fills the ring b columns at a time once the previous group's
// column watermark (prog[G-1], columns below it written back) covers them
// and the ring slot is free; a writer wave writes back every column no task
// of the group will touch again (below the lowest column of the slowest
// role of every sweep), drains, and publishes that watermark as prog[G].
// Waits are bounded (spin.h): a wait past the timeout sets the stall word and
// the workgroup's dead flag, after which no wave waits again and the launch
// drains with poisoned output.
// ---------------------------------------------------------------------------
#ifndef TG_BULGE_DF_GSW
#define TG_BULGE_DF_GSW 2
#endif
constexpr int DG = TG_BULGE_DF_GSW;   // sweeps per group
constexpr int DK = 4;                 // reflector slots per sweep
constexpr int DNCW = 3 * DG;          // role waves
#ifndef TG_BULGE_DF_XF
#define TG_BULGE_DF_XF 1
#endif
// 1: the loader issues a chunk's loads before it waits for ring space (the
// space is needed only by the LDS write).  Measured 69.0 -> 68.4 ms at n =
// 12,288 with a relaxed poll; with an ordered poll 69.1 ms, no gain, and it
// was the order that exposed the round-5 race, so the default is 0 (loads
// after the ring-space wait)
#ifndef TG_BULGE_LD_EARLY
#define TG_BULGE_LD_EARLY 0
#endif

constexpr int DXF = TG_BULGE_DF_XF;           // loader waves = writer waves (each moves 1/DXF)
constexpr int DBT = 64 * (DNCW + 2 * DXF);    // + loaders + writers
// ring span at the tightest spacing: the loader's chunk ahead of sweep 0
// plus LAG b columns per later sweep, plus the write-back chunk
static_assert((2 * DG + 1) * SB_B <= RING, "LDS ring too small for TG_BULGE_DF_GSW");

// Task (j, s) for the dataflow kernel: bulge_task_lds's arithmetic with two
// changes of WHO does it (the values and their order are the same):
// * the lower block's rank-1 update G -= tau u v^T is applied by the role-0
//   wave of the NEXT task, whose left block A(s+1) is exactly G(s): role 2
//   forms u, the next reflector from the updated column 0 and writes only
//   that pivot column (beta, 0, ..., 0) and tau u (into its reflector slot),
//   so the next reflector is out after one matrix-vector product instead of
//   a whole block update and store (on the last task of a sweep there is no
//   next left block, and role 2 updates and stores G as before);
// * each role loads its block first and waits for its reflector afterwards
//   (`wait_v`), so the block loads overlap the wait.
template <bool FULL, class WaitV>
__device__ __forceinline__ void df_task(double (*R)[LDB], int n, int j, int s, int role,
                                        bool has_next, double *__restrict__ V2, int smax,
                                        WaveScratch &W, Refl *slots, int DKs, WaitV wait_v) {
  // the lane index is opaque to the compiler here, so the per-lane block
  // addresses are formed per task instead of being hoisted out of the task
  // loop for every role (that kept ~80 loop-invariant registers live)
  int lane = threadIdx.x & 63;
  if constexpr (DBT > 512) asm volatile("" : "+v"(lane));  // only under a < 256-VGPR cap
  const int li = lane & 31, hf = lane >> 5;
  const int r1 = j + 1 + s * SB_B;
  const int L = FULL ? SB_B : min(SB_B, n - r1);
  const int col = (s == 0) ? j : r1 - SB_B;
  const int lo = FULL ? r1 - SB_B : max(0, r1 - SB_B);
  const int nl = FULL ? SB_B : r1 - lo;
  const int ng = FULL ? SB_B : min(SB_B, n - (r1 + L));
  double *Rf = &R[0][0];
  auto at = [&](int c, int d) { return rslot(c) * LDB + d; };
  const Refl &rin = slots[s % DKs];
  if (role == 0 && s == 0) {
    wait_v();
    store_refl(V2 + int64_t(j) * smax * SB_B, rin, lane);
    return;
  }
  double e[16];
  if (role == 0) {
    const int ca = FULL ? li : min(li, max(nl - 1, 0));
    const int abase = at(lo + ca, r1 - lo - ca);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = hf + 2 * q;
      if (FULL) e[q] = Rf[abase + i];
      else e[q] = (li < nl && i < L) ? Rf[abase + min(i, L - 1)] : 0.0;
    }
  } else if (role == 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      const int cc = min(li, k), off = li > k ? li - k : k - li;
      if (FULL) e[q] = Rf[at(r1 + cc, off)];
      else e[q] = (li < L && k < L) ? Rf[at(r1 + min(cc, L - 1), off)] : 0.0;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      if (FULL) e[q] = Rf[at(r1 + k, SB_B + li - k)];
      else {
        const int kc = min(k, L - 1);
        const double gv = Rf[at(r1 + kc, L + min(li, max(ng - 1, 0)) - kc)];
        e[q] = (li < ng && k < L) ? gv : 0.0;
      }
    }
  }
  wait_v();
  const double v = rin.v[li], tau = rin.tau;
  double vk[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) vk[q] = rin.v[hf + 2 * q];
  if (role == 2) {
    double u0 = 0.0, u1 = 0.0, u2 = 0.0, u3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      u0 += e[q] * vk[q];
      u1 += e[q + 1] * vk[q + 1];
      u2 += e[q + 2] * vk[q + 2];
      u3 += e[q + 3] * vk[q + 3];
    }
    double u = (u0 + u1) + (u2 + u3);
    u = hsum32(u);
    const double tu = tau * u;
    if (has_next) {
      Refl &rout = slots[(s + 1) % DKs];
      const double x0 = e[0] - tu * vk[0];  // updated column 0 (lanes hf == 0)
      double vn, tn, bn;
      make_refl((FULL || li < ng) ? x0 : 0.0, li, hf, vn, tn, bn);
      if (hf == 0) {
        rout.v[li] = vn;
        const_cast<Refl &>(rin).tu[li] = tu;
        if (FULL || li < ng) Rf[at(r1, L + li)] = (li == 0) ? bn : 0.0;
      }
      if (lane == 0) {
        rout.tau = tn;
        rout.beta = bn;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) e[q] = e[q] - tu * vk[q];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = hf + 2 * q;
        if (FULL || (li < ng && k < L)) Rf[at(r1 + k, L + li - k)] = e[q];
      }
    }
  } else if (role == 0) {
    // the previous task's lower-block update, on this block (= that block):
    // element (row i, column c) -= (tau u)_i v_c, as role 2 formed it
    const Refl &rp = slots[(s - 1) % DKs];
    const double vc = rp.v[li];
#pragma unroll
    for (int q = 0; q < 16; ++q) e[q] = e[q] - rp.tu[hf + 2 * q] * vc;
    double w0 = 0.0, w1 = 0.0, w2 = 0.0, w3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      w0 += vk[q] * e[q];
      w1 += vk[q + 1] * e[q + 1];
      w2 += vk[q + 2] * e[q + 2];
      w3 += vk[q + 3] * e[q + 3];
    }
    double wc = (w0 + w1) + (w2 + w3);
    wc = hsum32(wc);
    if ((FULL || li < nl) && lo + li != col) {
      const int c = li;
      double *Ac = Rf + at(lo + c, r1 - lo - c);
      const double twc = tau * wc;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = hf + 2 * q;
        if (FULL || i < L) Ac[i] = e[q] - twc * vk[q];
      }
    }
    store_refl(V2 + (int64_t(j) * smax + s) * SB_B, rin, lane);
  } else {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q += 4) {
      p0 += e[q] * vk[q];
      p1 += e[q + 1] * vk[q + 1];
      p2 += e[q + 2] * vk[q + 2];
      p3 += e[q + 3] * vk[q + 3];
    }
    double p = (p0 + p1) + (p2 + p3);
    p = hsum32(p);
    p *= tau;
    const double pv = wsum(hf == 0 ? p * v : 0.0);
    const double w = p - 0.5 * tau * pv * v;
    if (hf == 0) W.ws[li] = w;
    wave_sync();
    double wk[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) wk[q] = W.ws[hf + 2 * q];
    double *tr = W.trash + lane;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = hf + 2 * q;
      const bool ok = (FULL || li < L) && k <= li;
      double *dst = ok ? Rf + at(r1 + k, li - k) : tr;
      *dst = e[q] - v * wk[q] - w * vk[q];
    }
  }
}

struct DfSync {
  unsigned cnt[3][DG];  // [role][sweep]: tasks finished (role 2: + 1 for first_refl)
  unsigned loaded;      // columns [j0, loaded) are in the ring, final from the previous group
  unsigned wbs;         // columns below wbs are written back (their ring slots are free)
  unsigned dead;        // a wait gave up: nothing waits any more
  unsigned ldone[DXF];  // chunks finished by each loader wave
  unsigned wdone[DXF];  // write-back turns finished by each writer wave
  unsigned wturn;       // turns posted by writer 0 (the others follow)
  unsigned wrange[2][2];  // [turn & 1] = {lo, hi) of a posted turn
};

// The LDS progress words are the waves' only hand-offs inside a workgroup,
// and every one is a memory-model edge: the waits read them with workgroup-
// scope ACQUIRE loads (no later LDS or global access of the waiting wave is
// moved above the read) and the producers write them with workgroup-scope
// RELEASE stores (every earlier LDS access of the producing wave is complete
// first).  On gfx950 (no threadgroup split) these lower to exactly the
// hand-placed form of round 5 -- `ds_read; s_waitcnt lgkmcnt(0)` and
// `s_waitcnt lgkmcnt(0); ds_write` -- with no vmcnt wait (a workgroup-scope
// release needs none there), so the reflector records' global stores stay in
// flight; the difference is that the compiler now knows the order, which the
// round-5 race (a relaxed poll, the loader's ring writes scheduled above it)
// showed it did not (tools/check_handoff_isa.py checks the lowering).
// TG_BULGE_RACE_DEMO=1 (build-time, tools/bulge_hunt.py only): the round-5
// relaxed form, to show the tridiagonal guard catching the race it allowed.
#ifndef TG_BULGE_RACE_DEMO
#define TG_BULGE_RACE_DEMO 0
#endif
constexpr int LDS_ACQ = TG_BULGE_RACE_DEMO ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE;
constexpr int LDS_REL = TG_BULGE_RACE_DEMO ? __ATOMIC_RELAXED : __ATOMIC_RELEASE;
__device__ __forceinline__ unsigned lds_get(const unsigned *p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, LDS_ACQ, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_put(unsigned *p, unsigned v) {
  if constexpr (TG_BULGE_RACE_DEMO) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, LDS_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}

#if TG_BULGE_STATS
#ifndef TG_BULGE_TR0
#define TG_BULGE_TR0 100
#endif
constexpr int DF_TR0 = TG_BULGE_TR0;  // traced groups DF_TR0 .. DF_TR0 + 2
#define DF_NOW() __builtin_amdgcn_s_memrealtime()
#define DF_T0() uint64_t tw0_ = __builtin_amdgcn_s_memrealtime();
#define DF_ACC(k) st[k] += __builtin_amdgcn_s_memrealtime() - tw0_, tw0_ = __builtin_amdgcn_s_memrealtime();
#else
#define DF_T0()
#define DF_ACC(k)
#endif

// whole-wave wait until *p >= v (LDS word); false once the launch is dead
__device__ inline bool df_wait(const unsigned *p, unsigned v, DfSync &sy, unsigned *stall,
                               unsigned long long timeout) {
  // Both exits leave through an acquire load of *p (lds_get), so the caller's
  // accesses stay below the wait on every path.  (Round 5: the poll was a
  // relaxed load, which orders nothing; with the loader's loads issued before
  // its ring-space wait ~1 in 1500 launches at n = 384 and 1024 returned a
  // different last 32 (d, e), tools/bulge_hunt.py.)
  if (lds_get(p) >= v) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned it = 0;; ++it) {
    if (lds_get(&sy.dead)) return false;
    __builtin_amdgcn_s_sleep(1);
    if (lds_get(p) >= v) break;
    if ((it & 63u) == 63u) {
      if (__builtin_amdgcn_readfirstlane(tg::ctl_load(stall)) != 0u ||
          __builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        tg::stall_set(stall);
        lds_put(&sy.dead, 1u);
        return false;
      }
    }
  }
  return true;
}

// lowest column any role of sweep j still touches (n once the sweep is done):
// first_refl (cntG = 0) touches column j, task 0 columns >= j + 1, task s > 0
// columns >= r1 - b + 1 (its pivot column is final before it starts)
__device__ inline int df_low(int n, int j, unsigned ca, unsigned cd, unsigned cg) {
  if (cg == 0) return j;
  const int s = int(min(min(ca, cd), cg - 1));
  if (s >= ntasks(n, j)) return n;
  return s == 0 ? j + 1 : j + 2 + (s - 1) * SB_B;
}

// ctl[0] = chosen XCD + 1, ctl[1] = group queue, ctl[2] = stall word, ctl[4..68) dummies;
// prog[G] = column watermark of group G (columns below it written back)
__global__ __launch_bounds__(DBT) void bulge_df_kernel(double *__restrict__ B, int n,
                                                      double *__restrict__ V2, int smax,
                                                      unsigned *__restrict__ prog,
                                                      unsigned *__restrict__ ctl,
                                                      unsigned long long *__restrict__ stats,
                                                      unsigned long long timeout) {
  __shared__ double R[RING][LDB];
  __shared__ WaveScratch wsc[DNCW];
  __shared__ Refl rfl[DG][DK];
  __shared__ DfSync sy;
  __shared__ int sh_G;
  const int tid = threadIdx.x, wlane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned *stall = ctl + 2;
  unsigned *dummy = ctl + 4;
#if TG_BULGE_STATS
  // per wave: [0] first wait kind, [1] second wait kind, [2] busy, [3] count
  // (task waves: own reflector or slot / previous sweep or loader / task;
  //  loader: producer watermark / ring space / load; writer: idle / drain / issue)
  uint64_t st[6] = {0, 0, 0, 0, 0, 0};  // [5] = count
  const uint64_t st_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    unsigned expect = 0;
    __hip_atomic_compare_exchange_strong(ctl, &expect, x + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const unsigned chosen = expect == 0 ? x + 1 : expect;
    sh_G = (chosen == x + 1) ? 0 : -1;
  }
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(sh_G) < 0) return;
  const int nsw = n - 2;
  const int ngroups = tg::cdiv(nsw, DG);
  const int bytes = n * LDB * int(sizeof(double));
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(B, 0, bytes, 0x00020000);
  constexpr int SC1 = 16;
  constexpr int NTC = LDB / 2;               // 16-B chunks per column
  constexpr int PL = SB_B * NTC / 64;        // chunks per lane of a b-column load
  while (true) {
    if (wid == 0) {
      const unsigned v = atomicAdd(lane0_or_dummy(ctl + 1, dummy, wlane), 1u);
      const int Gn = tg::ctl_load(stall) ? ngroups : int(__builtin_amdgcn_readfirstlane(v));
      sh_G = Gn;
      // reset the group's counters: every lane writes one word (no lane-0 branch)
      unsigned *w = &sy.cnt[0][0];
      constexpr int NWD = int(sizeof(DfSync) / sizeof(unsigned));
      const int k = min(wlane, NWD - 1);
      const int j0n = Gn * DG;
      w[k] = (k == int(offsetof(DfSync, loaded) / sizeof(unsigned))) ? unsigned(j0n)
             : (k == int(offsetof(DfSync, wbs) / sizeof(unsigned))) ? unsigned(j0n)
                                                                     : 0u;
    }
    __syncthreads();
    const int G = __builtin_amdgcn_readfirstlane(sh_G);
    __syncthreads();
    if (G >= ngroups) break;
    const int j0 = G * DG;
    const int g = min(DG, nsw - j0);
    if (wid < DNCW) {
      const int q = wid / 3, role = wid % 3;
      const int j = j0 + q;
      if (q < g) {
        const int nt = ntasks(n, j);
        const int ntp = q > 0 ? ntasks(n, j - 1) : 0;
        unsigned *own = &sy.cnt[role][q];
        // columns [.., c) must hold the previous sweep's results
        auto need_prev = [&](int s_next, bool with_g) -> bool {
          // sweep q-1 finished tasks < s_next (A, D) and its G of task s_next - 1
          if (q > 0) {
            const unsigned a = unsigned(min(s_next, ntp));
            bool ok = df_wait(&sy.cnt[0][q - 1], a, sy, stall, timeout);
            ok = ok && df_wait(&sy.cnt[1][q - 1], a, sy, stall, timeout);
            if (with_g) ok = ok && df_wait(&sy.cnt[2][q - 1], unsigned(min(s_next + 1, ntp + 1)), sy,
                                           stall, timeout);
            return ok;
          }
          return true;
        };
        if (role == 2) {
          DF_T0()
          if (q > 0) {
            df_wait(&sy.cnt[1][q - 1], 1u, sy, stall, timeout);
            df_wait(&sy.cnt[2][q - 1], unsigned(min(2, ntp + 1)), sy, stall, timeout);
          } else {
            df_wait(&sy.loaded, unsigned(j + 1), sy, stall, timeout);
          }
          DF_ACC(1)
          first_refl(R, n, j, rfl[q][0]);
          lds_put(own, 1u);
        }
        for (int s = 0; s < nt; ++s) {
          const int r1 = j + 1 + s * SB_B;
          DF_T0()
          // the block's inputs: for role 0 the region of G(s-1) (what sweep
          // q-1 must have finished for role 2's task s-1), else this task's
          if (!(role == 0 && s == 0)) {
            const int sp = role == 0 ? s - 1 : s;
            if (q == 0)
              df_wait(&sy.loaded, unsigned(min(n, j + 1 + (sp + 1) * SB_B)), sy, stall, timeout);
            else
              need_prev(sp + 2, role != 1);
            // D (q, s) overlaps G (q - 1, s) in its last row (r1 + b - 1).
            // That G block's rank-1 update is normally deferred to A (q - 1,
            // s + 1), which need_prev waits for -- but the LAST task of sweep
            // q - 1 has no next task and applies it itself, and a 1-row G
            // block remains when n - r1' = b + 1.  So D of the task with the
            // previous sweep's last index waits for that sweep's G roles too.
            // (Found by the tridiagonal guard: ~1 in 7000 launches at n = 384
            // let D read the row before the store, moving the last 32 d by
            // up to 9e-2 -- the round-5 symptom, whose compiler barrier had
            // only shifted its timing.)
            if (role == 1 && q > 0 && s == ntp - 1)
              df_wait(&sy.cnt[2][q - 1], unsigned(ntp + 1), sy, stall, timeout);
          }
          DF_ACC(1)
          auto wait_v = [&]() {
            if (role != 2) {
              df_wait(&sy.cnt[2][q], unsigned(s + 1), sy, stall, timeout);
            } else if (s + 1 < nt) {
              // the slot of v(s+1) held v(s+1-DK): read by A up to task s+2-DK
              // (its tau u too), by D at task s+1-DK
              if (s + 3 - DK > 0) df_wait(&sy.cnt[0][q], unsigned(s + 3 - DK), sy, stall, timeout);
              if (s + 2 - DK > 0) df_wait(&sy.cnt[1][q], unsigned(s + 2 - DK), sy, stall, timeout);
            }
            DF_ACC(0)
          };
          const bool nx = s + 1 < nt;
          if (r1 >= SB_B && r1 + 2 * SB_B <= n)
            df_task<true>(R, n, j, s, role, nx, V2, smax, wsc[wid], rfl[q], DK, wait_v);
          else
            df_task<false>(R, n, j, s, role, nx, V2, smax, wsc[wid], rfl[q], DK, wait_v);
          lds_put(own, unsigned(s + 1 + (role == 2)));
          DF_ACC(2)
#if TG_BULGE_STATS
          ++st[5];
          if (stats && G >= DF_TR0 && G < DF_TR0 + 3 && s < 128 && wlane == 0)
            stats[128 + ((G - DF_TR0) * 4 + role) * DG * 128 + q * 128 + s] =
                __builtin_amdgcn_s_memrealtime();
#endif
        }
      }
    } else if (wid < DNCW + DXF) {
      // loaders: b columns at a time once the producer's watermark covers them
      // and their ring slots are written back.  Chunks end at j0 + 1 + k b --
      // the columns task k - 1 of sweep 0 needs, and the watermarks the
      // producer's last sweep publishes -- after a first chunk of column j0
      // alone (first_refl).  Loader x takes chunks x, x + DXF, ... (each wave's
      // poll -> load -> LDS round trip is latency, so DXF chunks are in
      // flight at once); chunks are published in order.
      const int x = wid - DNCW;
      const int nch = n - j0 <= 1 ? 1 : 2 + (n - j0 - 2) / SB_B;  // chunks of the group
      for (int k = x; k < nch; k += DXF) {
        const int ld = k == 0 ? j0 : j0 + 1 + (k - 1) * SB_B;
        const int ce = min(k == 0 ? j0 + 1 : ld + SB_B, n);
        DF_T0()
        if (G > 0 && !lds_get(&sy.dead) && !tg::spin_geq(prog + G - 1, unsigned(ce), stall, timeout))
          lds_put(&sy.dead, 1u);
        DF_ACC(0)
#if !TG_BULGE_LD_EARLY
        df_wait(&sy.wbs, unsigned(max(0, ce - RING)), sy, stall, timeout);
#endif
        DF_ACC(1)
        double2 buf[PL];
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int idx = wlane + 64 * u;
          const int c = min(ld + idx / NTC, ce - 1), h = idx % NTC;
          const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rb, (c * LDB + 2 * h) * 8, 0, SC1);
          buf[u] = make_double2(__builtin_bit_cast(double, u32x2{v4[0], v4[1]}),
                                __builtin_bit_cast(double, u32x2{v4[2], v4[3]}));
        }
#if TG_BULGE_LD_EARLY
        // the ring space is needed only by the LDS write: the chunk's loads
        // are in flight while the writer retires the slots
        df_wait(&sy.wbs, unsigned(max(0, ce - RING)), sy, stall, timeout);
#endif
#if TG_BULGE_STATS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        DF_ACC(2)
#endif
        // one 16-B LDS write per chunk (two 8-B halves were 4-way bank-conflicted:
        // lanes 16 B apart, the column pair 512 B apart)
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int idx = wlane + 64 * u;
          const int c = ld + idx / NTC, h = idx % NTC;
          if (c < ce) *reinterpret_cast<double2 *>(&R[rslot(c)][2 * h]) = buf[u];
        }
        if (DXF > 1) df_wait(&sy.loaded, unsigned(ld), sy, stall, timeout);  // in order
        lds_put(&sy.loaded, unsigned(ce));
        DF_ACC(3)
#if TG_BULGE_STATS
        ++st[5];
        if (stats && G >= DF_TR0 && G < DF_TR0 + 3 && wlane == 0 && k < 128)
          stats[128 + ((G - DF_TR0) * 4 + 3) * DG * 128 + k] = __builtin_amdgcn_s_memrealtime();
#endif
      }
    } else {
      // writers: every column below the group's low watermark, then publish it.
      // Writer 0 decides each turn's range [lo, hi) and posts it; writer x
      // stores the range's 1 KB blocks x, x + DXF, ...; the last to drain a
      // turn publishes hi (turns publish in order: a writer publishes turn t
      // only once every other writer has finished t, hence every earlier turn).
      const int x = wid - DNCW - DXF;
      DF_T0()
      unsigned t = 0;
      for (int hi = j0; hi < n; ++t) {
        int lo = hi;
        if (x == 0) {
          int low;
          while (true) {
            low = int(lds_get(&sy.loaded));
            if (lds_get(&sy.dead)) low = n;
            for (int q = 0; q < g; ++q)
              low = min(low, df_low(n, j0 + q, lds_get(&sy.cnt[0][q]), lds_get(&sy.cnt[1][q]),
                                    lds_get(&sy.cnt[2][q])));
            if (low > lo) break;
            __builtin_amdgcn_s_sleep(1);
          }
          hi = low;
          if (DXF > 1) {
            // the range slot of turn t held turn t - 2: every follower past it
            if (t >= 2)
              for (int y = 1; y < DXF; ++y) df_wait(&sy.wdone[y], t - 1, sy, stall, timeout);
            sy.wrange[t & 1][0] = unsigned(lo);
            sy.wrange[t & 1][1] = unsigned(hi);
            lds_put(&sy.wturn, t + 1);
          }
        } else {
          df_wait(&sy.wturn, t + 1, sy, stall, timeout);
          lo = int(lds_get(&sy.wrange[t & 1][0]));
          hi = int(lds_get(&sy.wrange[t & 1][1]));
          if (lds_get(&sy.dead)) hi = max(hi, n);
        }
        DF_ACC(0)
        // this writer's blocks of b columns at a time: LDS reads first, then the stores
        constexpr int PX = PL / DXF;
        for (int c0 = lo; c0 < hi; c0 += SB_B) {
          const int lim = (min(c0 + SB_B, hi) - c0) * NTC;
          double2 wv[PX];
#pragma unroll
          for (int u = 0; u < PX; ++u) {
            const int idx = min(wlane + 64 * (x + DXF * u), lim - 1);
            const int c = c0 + idx / NTC, h = idx % NTC;
            wv[u] = *reinterpret_cast<const double2 *>(&R[rslot(c)][2 * h]);
          }
#if TG_BULGE_STATS
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          DF_ACC(1)
#endif
#pragma unroll
          for (int u = 0; u < PX; ++u) {
            const int idx = wlane + 64 * (x + DXF * u);
            if (idx < lim) {
              const int c = c0 + idx / NTC, h = idx % NTC;
              const u32x2 lo2 = __builtin_bit_cast(u32x2, wv[u].x);
              const u32x2 hi2 = __builtin_bit_cast(u32x2, wv[u].y);
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo2[0], lo2[1], hi2[0], hi2[1]}, rb,
                                                     (c * LDB + 2 * h) * 8, 0, 0);
            }
          }
        }
        DF_ACC(2)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        DF_ACC(3)
        bool last = true;
        if (DXF > 1) {
          lds_put(&sy.wdone[x], t + 1);
#pragma unroll
          for (int y = 0; y < DXF; ++y) last = last && lds_get(&sy.wdone[y]) >= t + 1;
        }
        if (last) {
          publish(lane0_or_dummy(prog + G, dummy, wlane), unsigned(hi));
          // the ring slots below hi are free: release (this wave's LDS reads
          // of them are complete) to the loader's acquire in df_wait
          __hip_atomic_fetch_max(&sy.wbs, unsigned(hi), __ATOMIC_RELEASE,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        DF_ACC(4)
#if TG_BULGE_STATS
        ++st[5];
#endif
      }
    }
    __syncthreads();
  }
#if TG_BULGE_STATS
  if (stats && wlane == 0) {
    for (int k = 0; k < 6; ++k) atomicAdd(stats + 8 + 6 * wid + k, (unsigned long long)st[k]);
    if (wid == 0) {
      atomicAdd(stats + 0, 1ull);
      atomicAdd(stats + 5, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - st_t0));
    }
  }
#endif
}

// Bst[c][d] = A[c + d][c] for d <= b, 0 for b < d < 2b.
__global__ void extract_band_kernel(const double *__restrict__ A, int64_t lda, int n,
                                    double *__restrict__ Bst) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * LDB) return;
  const int c = idx / LDB, d = idx % LDB;
  Bst[idx] = (d <= SB_B && c + d < n) ? A[int64_t(c + d) * lda + c] : 0.0;
}

// ---------------------------------------------------------------------------
// Tridiagonal guard.  Band -> tridiagonal is an orthogonal similarity, so it
// keeps trace(B) = sum d and ||B||_F^2 = sum d^2 + 2 sum e^2.  Both sides are
// O(n) sums: band_inv_kernel sums the band (GINV workgroups, fixed order)
// before the chase, tri_check_kernel the tridiagonal after it and compares.
// A violation (a race or fault in the pipeline, the round-5 kind: one bad
// launch in ~1500 moved the last 32 d by up to 9e-2) sets the guard word
// (ctl[3]): extract_tri_kernel then poisons (d, e) with NaN and the host
// raises, so a corrupted tridiagonal never reaches k, perm or U.  Bars
// (relative): |sum d - tr B| <= TRI_TOL_TR sqrt(n) ||B||_F and
// |F(T) - F(B)| <= TRI_TOL_F F(B), F = squared Frobenius norm; measured
// residuals are ~1e-15 .. 1e-14 (TG_TRI_GUARD_PRINT=1 prints them), so the
// bars leave three to four orders of margin and still catch a change of one
// d by ~1e-7 ||B||_F.
// ---------------------------------------------------------------------------
constexpr int GINV = 64;                 // band-sum workgroups
constexpr double TRI_TOL_TR = 1e-10, TRI_TOL_F = 1e-10;

template <int NT>
__device__ inline void block_sum2(double &a, double &b, double (*sh)[NT]) {
  const int t = threadIdx.x;
  sh[0][t] = a;
  sh[1][t] = b;
  __syncthreads();
#pragma unroll
  for (int h = NT / 2; h > 0; h >>= 1) {
    if (t < h) {
      sh[0][t] += sh[0][t + h];
      sh[1][t] += sh[1][t + h];
    }
    __syncthreads();
  }
  a = sh[0][0];
  b = sh[1][0];
}

// part[2 b + {0, 1}] = (trace, squared Frobenius norm) of workgroup b's slice
__global__ __launch_bounds__(256) void band_inv_kernel(const double *__restrict__ Bst, int n,
                                                       double *__restrict__ part) {
  __shared__ double sh[2][256];
  const int64_t tot = int64_t(n) * LDB, per = (tot + GINV - 1) / GINV;
  const int64_t e0 = blockIdx.x * per, e1 = min(tot, e0 + per);
  double tr = 0.0, fr = 0.0;
  for (int64_t x = e0 + threadIdx.x; x < e1; x += 256) {
    const double v = Bst[x];
    const bool dg = (x % LDB) == 0;  // d > b entries are zero in the extracted band
    tr += dg ? v : 0.0;
    fr += (dg ? 1.0 : 2.0) * v * v;
  }
  block_sum2<256>(tr, fr, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = tr;
    part[2 * blockIdx.x + 1] = fr;
  }
}

// One workgroup.  corrupt >= 0 (TG_TRI_GUARD_CORRUPT, tests): first change
// d[corrupt] by 1e-3 (1 + |d|), as a faulty pipeline would.  res[0..1] =
// the two relative residuals; *guard = 1 on a violation (or a NaN).
__global__ __launch_bounds__(256) void tri_check_kernel(double *__restrict__ Bst, int n,
                                                        const double *__restrict__ part,
                                                        int corrupt, int nopoison,
                                                        double *__restrict__ res,
                                                        unsigned *__restrict__ guard) {
  __shared__ double sh[2][256];
  if (corrupt >= 0 && corrupt < n && threadIdx.x == 0) {
    const double v = Bst[int64_t(corrupt) * LDB];
    Bst[int64_t(corrupt) * LDB] = v + 1e-3 * (1.0 + fabs(v));
  }
  __syncthreads();
  double tr = 0.0, fr = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const double dv = Bst[int64_t(i) * LDB];
    const double ev = i + 1 < n ? Bst[int64_t(i) * LDB + 1] : 0.0;
    tr += dv;
    fr += dv * dv + 2.0 * ev * ev;
  }
  block_sum2<256>(tr, fr, sh);
  if (threadIdx.x == 0) {
    double t0 = 0.0, f0 = 0.0;
    for (int b = 0; b < GINV; ++b) {
      t0 += part[2 * b];
      f0 += part[2 * b + 1];
    }
    const double rt = f0 > 0.0 ? fabs(tr - t0) / (sqrt(double(n)) * sqrt(f0)) : fabs(tr - t0);
    const double rf = f0 > 0.0 ? fabs(fr - f0) / f0 : fabs(fr - f0);
    res[0] = rt;
    res[1] = rf;
    // bit 0: poison (d, e); bit 1: violated (TG_TRI_GUARD_NOPOISON, the race
    // hunt: report but keep the values for comparison)
    if (!(rt <= TRI_TOL_TR && rf <= TRI_TOL_F)) tg::ctl_record(guard, nopoison ? 2u : 3u);
  }
}

__global__ void extract_tri_kernel(const double *__restrict__ Bst, int n,
                                   const unsigned *__restrict__ stall, double *__restrict__ dg,
                                   double *__restrict__ e) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // a stalled pipeline chased on stale band data, or a tridiagonal that
  // failed the invariant check (stall[1], the guard word): poison (d, e) so
  // no consumer takes its eigenvalues for real ones
  const bool bad = stall && (stall[0] != 0u || (stall[1] & 1u) != 0u);
  dg[i] = bad ? __builtin_nan("") : Bst[int64_t(i) * LDB];
  e[i] = bad ? __builtin_nan("") : (i + 1 < n) ? Bst[int64_t(i) * LDB + 1] : 0.0;
}

}  // namespace

namespace tg {

int sb_smax(int n) { return n >= 3 ? (n - 3) / SB_B + 1 : 1; }

// progress word per sweep group (at most one group per sweep, whichever
// kernel runs) + control words + 64 dummy words; the control words start at
// prog + (n - 2)
// + the tridiagonal guard's doubles (band partials, residuals) from the next
// even word
static size_t guard_off(int n) { return (size_t(std::max(1, n - 2)) + 4 + 64 + 1) & ~size_t(1); }
size_t sb2st_prog_words(int n) { return guard_off(n) + 2 * (2 * GINV + 2); }

// TG_BULGE_DF=0: the step-synchronous kernel (bulge_lds_kernel); default the
// dataflow kernel (bulge_df_kernel: bit-identical, 21.1 -> 19.0 ms at n =
// 4096 and 80.8 -> 69.0 ms at n = 12,288 on MI355X)
static bool bulge_dataflow() {
  const char *e = getenv("TG_BULGE_DF");
  return !(e && e[0] == '0');
}

// TG_TRI_GUARD=0 (development switch, read per call): no invariant check
static bool guard_on() {
  const char *g = getenv("TG_TRI_GUARD");
  return !(g && g[0] == '0');
}

hipError_t sb2st(hipStream_t st, const double *A, int lda, int n, double *Bst, double *V2,
                 unsigned *prog, double *d, double *e) {
  hipLaunchKernelGGL(extract_band_kernel, dim3(cdiv(int64_t(n) * LDB, 256)), dim3(256), 0, st, A,
                     int64_t(lda), n, Bst);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  const int nsw = n - 2;
  const unsigned *stall = nullptr;
  if (nsw > 0) {
    const bool df = bulge_dataflow();
    err = hipMemsetAsync(prog, 0, sizeof(unsigned) * sb2st_prog_words(n), st);
    if (err != hipSuccess) return err;
    double *gpart = reinterpret_cast<double *>(prog + guard_off(n));
    if (guard_on()) {
      hipLaunchKernelGGL(band_inv_kernel, dim3(GINV), dim3(256), 0, st, Bst, n, gpart);
      err = hipGetLastError();
      if (err != hipSuccess) return err;
    }
    unsigned *ctl = prog + nsw;  // [0] XCD + 1, [1] group queue, [2] stall flag
    stall = ctl + 2;
    const unsigned long long timeout = spin_timeout_ticks("TG_BULGE_TIMEOUT_TICKS");
    // TG_BULGE_STATS (environment): elapsed time of the launch; with a
    // -DTG_BULGE_STATS=1 build also the per-step clock stamps per wave
    const bool want = getenv("TG_BULGE_STATS") != nullptr;
    unsigned long long *stats = nullptr;
#if TG_BULGE_HB
    unsigned long long *hbh = nullptr;
    (void)hipHostMalloc(&hbh, 256 * 16 * 8, hipHostMallocMapped);
    memset(hbh, 0, 256 * 16 * 8);
    (void)hipHostGetDevicePointer((void **)&stats, hbh, 0);
    hipEvent_t hbe;
    (void)hipEventCreateWithFlags(&hbe, hipEventDisableTiming);
#endif
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (want) {
      if (TG_BULGE_STATS) {
        const size_t ns = 128 + 3 * 4 * 4 * 128;
        (void)hipMalloc(&stats, ns * sizeof(unsigned long long));
        (void)hipMemsetAsync(stats, 0, ns * sizeof(unsigned long long), st);
      }
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, st);
    }
    // ~12.3 kflop per task (3 blocks of b x b, rank-1 each), n^2/(2b) tasks;
    // band streamed once per sweep group (load + write-back, L2-resident)
    double ntask = 0.0;
    for (int j = 0; j < nsw; ++j) ntask += (n - 3 - j) / SB_B + 1;
    auto tok = tg::prof_begin(st, tg::PROF_BULGE, 8.0 * LDB * double(n) * n / (df ? DG : G_SW),
                              12.0 * SB_B * SB_B * ntask);
    // one workgroup per CU (the ring fills the LDS): the elected XCD's share
    // of the grid is its CUs, the other XCDs' workgroups exit at once
    const XcdInfo xi = xcd_info();
    if (df)
      hipLaunchKernelGGL(bulge_df_kernel, dim3(xi.xcds * xi.cus_per_xcd), dim3(DBT), 0, st, Bst,
                         n, V2, sb_smax(n), prog, ctl, stats, timeout);
    else
      hipLaunchKernelGGL(bulge_lds_kernel, dim3(xi.xcds * xi.cus_per_xcd), dim3(BT), 0, st, Bst,
                         n, V2, sb_smax(n), prog, ctl, stats, timeout);
    tg::prof_end(st, tok);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
#if TG_BULGE_HB
    (void)hipEventRecord(hbe, st);
    for (int it = 0; it < 300 && hipEventQuery(hbe) == hipErrorNotReady; ++it) usleep(10000);
    if (hipEventQuery(hbe) == hipErrorNotReady) {
      fprintf(stderr, "bulge HANG: heartbeat (block: wave=G/step/lanes/phase)\n");
      for (int bk = 0; bk < 256; ++bk) {
        bool any = false;
        for (int w = 0; w < NCW + 2; ++w) any |= hbh[bk * 16 + w] != 0;
        if (!any) continue;
        fprintf(stderr, "  b%3d:", bk);
        for (int w = 0; w < NCW + 2; ++w) {
          const unsigned long long v = hbh[bk * 16 + w];
          fprintf(stderr, " %llu/%llu/%llu/%llu", (v >> 32) - 1, ((v >> 16) & 0xffff) - 1, (v >> 8) & 255,
                  v & 255);
        }
        fprintf(stderr, "\n");
      }
      fflush(stderr);
      _exit(3);
    }
    stats = nullptr;
#endif
    if (want) {
      (void)hipEventRecord(e1, st);
      unsigned long long h[128] = {0};
      if (stats) (void)hipMemcpyAsync(h, stats, sizeof(h), hipMemcpyDeviceToHost, st);
      (void)hipStreamSynchronize(st);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      fprintf(stderr, "bulge: %.2f ms (%s, G_SW %d)\n", ms, df ? "dataflow" : "step", df ? DG : G_SW);
#if TG_BULGE_STATS
      if (stats && df && getenv("TG_BULGE_TRACE")) {
        // role end times (us, relative) of tasks 0..15 of the traced groups
        static unsigned long long tr[3 * 4 * DG * 128];
        (void)hipMemcpy(tr, stats + 128, sizeof(tr), hipMemcpyDeviceToHost);
        unsigned long long t0 = ~0ull;
        for (auto x : tr) if (x && x < t0) t0 = x;
        const char *rn[4] = {"A", "D", "G", "L"};
        for (int gg = 0; gg < 3; ++gg)
          for (int r = 0; r < 4; ++r)
            for (int q = 0; q < (r == 3 ? 1 : DG); ++q) {
              fprintf(stderr, "  trace G%d %s%d:", DF_TR0 + gg, rn[r], q);
              for (int t = 0; t < 16; ++t) {
                const unsigned long long x = tr[(gg * 4 + r) * DG * 128 + q * 128 + t];
                fprintf(stderr, " %6.2f", x ? (x - t0) / 100.0 : -1.0);
              }
              fprintf(stderr, "\n");
            }
      }
#endif
      if (stats && df) {
        const double W = double(h[0] ? h[0] : 1);
        fprintf(stderr, "  workers %llu, worker time %.1f us; per wave and worker (us): "
                "[t0 t1 t2 t3 t4] count; per unit (us)\n"
                "  (tasks: own refl/slot, prev sweep/loader, task; loader: producer, ring, "
                "issue->data, LDS+publish; writer: idle, LDS read, store issue, drain, publish)\n",
                h[0], h[5] / 100.0 / W);
        for (int w = 0; w < DNCW + 2 * DXF; ++w) {
          const unsigned long long *x = h + 8 + 6 * w;
          const double c = double(x[5] ? x[5] : 1);
          fprintf(stderr, "   w%d %s: %.0f %.0f %.0f %.0f %.0f  %llu;  %.2f %.2f %.2f %.2f %.2f\n", w,
                  w < DNCW ? (w % 3 == 0 ? "A" : w % 3 == 1 ? "D" : "G")
                           : (w < DNCW + DXF ? "load" : "write"),
                  x[0] / 100.0 / W, x[1] / 100.0 / W, x[2] / 100.0 / W, x[3] / 100.0 / W,
                  x[4] / 100.0 / W, x[5], x[0] / 100.0 / c, x[1] / 100.0 / c, x[2] / 100.0 / c,
                  x[3] / 100.0 / c, x[4] / 100.0 / c);
        }
        (void)hipFree(stats);
        stats = nullptr;
      }
      if (stats) {
        const double W = double(h[0]), S = double(h[6]);
        fprintf(stderr,
                "  workers %.0f, steps/worker %.0f; per step (us): wait %.2f task %.2f bar %.2f\n",
                W, S / W, h[1] / 100.0 / S, h[2] / 100.0 / S, h[3] / 100.0 / S);
        if (h[5]) fprintf(stderr, "  shader clock %.2f GHz\n", 0.1 * double(h[4]) / double(h[5]));
        fprintf(stderr, "  per-wave busy per step (us):");
        for (int w = 0; w < NCW + 2; ++w) fprintf(stderr, " w%d %.2f", w, h[8 + w] / 100.0 / S);
        fprintf(stderr, "\n");
        (void)hipFree(stats);
      }
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
  }
  if (nsw > 0 && guard_on()) {
    const char *cx = getenv("TG_TRI_GUARD_CORRUPT");  // tests: corrupt one d before the check
    double *gpart = reinterpret_cast<double *>(prog + guard_off(n));
    hipLaunchKernelGGL(tri_check_kernel, dim3(1), dim3(256), 0, st, Bst, n, gpart,
                       cx ? atoi(cx) : -1, getenv("TG_TRI_GUARD_NOPOISON") ? 1 : 0,
                       gpart + 2 * GINV, prog + nsw + 3);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  hipLaunchKernelGGL(extract_tri_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, Bst, n, stall, d,
                     e);
  return hipGetLastError();
}

hipError_t sb2st_stalled(hipStream_t st, int n, const unsigned *prog, bool *stalled,
                         bool *broken) {
  *stalled = false;
  if (broken) *broken = false;
  const int nsw = n - 2;
  if (nsw <= 0) return hipSuccess;
  unsigned h[2] = {0u, 0u};
  double r[2] = {0.0, 0.0};
  hipError_t e = hipMemcpyAsync(h, prog + nsw + 2, sizeof(h), hipMemcpyDeviceToHost, st);
  // TG_TRI_GUARD_PRINT=1: print the residuals of every call, =2: of violations only
  const char *pe = getenv("TG_TRI_GUARD_PRINT");
  const int pr = pe ? atoi(pe) : 0;
  if (e == hipSuccess && pr)
    e = hipMemcpyAsync(r, prog + guard_off(n) + 4 * GINV, sizeof(r), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (pr == 1 || (pr == 2 && h[1]))
    fprintf(stderr, "tri_guard n=%d: trace %.3e frobenius %.3e%s\n", n, r[0], r[1],
            h[1] ? " VIOLATED" : "");
  *stalled = h[0] != 0u;
  if (broken) *broken = h[1] != 0u;
  return e;
}

}  // namespace tg

// ---------------------------------------------------------------------------
// Back-transformation Z <- Q2 Z.  Reflectors are grouped into blocks
// (G2, s) = sweeps 32 G2 .. 32 G2 + 31 at step s: a staircase Y of 63 rows
// (column a = reflector of sweep 32 G2 + a, rows a .. a + 31 of the block,
// block rows start at 32 G2 + 1 + 32 s) with Q_block = H_0 H_1 ... H_31 =
// I - Y T Y^T.  Valid order (== applying the reflectors in reverse): later
// sweep groups first, steps ascending within a group; blocks overlap only
// with (G2, s-1) and (G2+1 or later, s' < s + 1), so level
// s + (NG2 - 1 - G2) is a set of row-disjoint blocks: one launch per level.
// ---------------------------------------------------------------------------
namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));
constexpr int QB = 32;           // sweeps per block (= SB_B)
constexpr int QR = QB + SB_B - 1;  // rows per block (63)

__device__ inline bool refl_valid(int n, int j, int s) { return j <= n - 3 && s < ntasks(n, j); }

__global__ __launch_bounds__(256) void q2_tfactor_kernel(const double *__restrict__ V2, int n,
                                                         int smax, double *__restrict__ T2) {
  __shared__ double Vs[QB][SB_B];
  __shared__ double Gs[QB][QB + 1];
  __shared__ double Ts[QB][QB + 1];
  __shared__ double taus[QB];
  const int G2 = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
  const int j0 = G2 * QB;
  double *Tout = T2 + (int64_t(G2) * smax + s) * QB * QB;
  if (!refl_valid(n, j0, s)) return;
  for (int idx = tid; idx < QB * SB_B; idx += 256) {
    const int a = idx / SB_B, i = idx % SB_B;
    const bool ok = refl_valid(n, j0 + a, s);
    const double x = ok ? V2[(int64_t(j0 + a) * smax + s) * SB_B + i] : 0.0;
    Vs[a][i] = i == 0 ? (ok ? 1.0 : 0.0) : x;
    if (i == 0) taus[a] = x;  // element 0 of the record is tau
  }
  __syncthreads();
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + 256 * q, a = idx >> 5, c = idx & 31;
    double g = 0.0;
    if (a < c)
      for (int i = c; i < a + SB_B; ++i) g += Vs[a][i - a] * Vs[c][i - c];
    Gs[a][c] = g;
    Ts[a][c] = 0.0;
  }
  __syncthreads();
  // row a of T is independent of the other rows (dlarft forward columnwise):
  // T[a][c] = -tau_c sum_{a<=e<c} T[a][e] G[e][c], T[a][a] = tau_a; thread a
  // keeps its row in registers (no barrier per column).  The terms e < a are
  // exact zeros, so the sums match the column-by-column order bit for bit.
  if (tid < QB) {
    double trow[QB];
#pragma unroll
    for (int c = 0; c < QB; ++c) {
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < c; ++e) acc += trow[e] * Gs[e][c];
      const double tc = taus[c];
      trow[c] = tid < c ? -tc * acc : (tid == c ? tc : 0.0);
    }
#pragma unroll
    for (int c = 0; c < QB; ++c) Ts[tid][c] = trow[c];
  }
  __syncthreads();
  for (int idx = tid; idx < QB * QB; idx += 256) Tout[idx] = Ts[idx >> 5][idx & 31];
}

// One level: blockIdx.y enumerates the level's blocks, each wave one
// 32-column slab of Z (n x k row-major) over the block's rows (64-row tile
// in registers as eight 16x16 C-layout fragments).
__global__ __launch_bounds__(256) void q2_apply_kernel(double *__restrict__ Z, int k, int n,
                                                       const double *__restrict__ V2,
                                                       const double *__restrict__ T2, int smax,
                                                       int ng2, int level, int s_lo) {
  const int s = s_lo + blockIdx.y;
  const int G2 = ng2 - 1 - (level - s);
  const int j0 = G2 * QB;
  if (G2 < 0 || !refl_valid(n, j0, s)) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  const int c0 = (blockIdx.x * 4 + wid) * 32;
  const int rb0 = j0 + 1 + s * SB_B;  // first row of the block
  __shared__ double Vs[QB][SB_B + 1];
  __shared__ double Ts[QB][QB + 1];
  {
    const double *Tb = T2 + (int64_t(G2) * smax + s) * QB * QB;
    double vv[4], tt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q, a = idx >> 5, d = idx & 31;
      const int jj = refl_valid(n, j0 + a, s) ? j0 + a : j0;  // clamp to a valid reflector
      vv[q] = V2[(int64_t(jj) * smax + s) * SB_B + d];
      tt[q] = Tb[idx];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = threadIdx.x + 256 * q, a = idx >> 5, d = idx & 31;
      Vs[a][d] = refl_valid(n, j0 + a, s) ? (d == 0 ? 1.0 : vv[q]) : 0.0;
      Ts[a][d] = tt[q];
    }
  }
  __syncthreads();
  if (c0 >= k) return;
  // Y[i][a] = v_a[i - a]  (rows past n hold zeros in v)
  auto yval = [&](int i, int a) -> double {
    const int d = i - a;
    return (d >= 0 && d < SB_B) ? Vs[a][d] : 0.0;
  };
  doublex4 F[4][2];
  {
    double zl[4][4][2];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int row = min(rb0 + rb * 16 + lr + 4 * q, n - 1);
          const int col = min(c0 + cb * 16 + lc, k - 1);
          zl[rb][q][cb] = Z[int64_t(row) * k + col];
        }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = rb * 16 + lr + 4 * q;
        const bool ok = i < QR && rb0 + i < n;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          F[rb][cb][q] = (ok && c0 + cb * 16 + lc < k) ? zl[rb][q][cb] : 0.0;
      }
  }
  // P = Y^T Z  (32 x 32)
  doublex4 Pa[2][2];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) Pa[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
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
        for (int cb = 0; cb < 2; ++cb)
          Pa[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[ia], F[rb][cb][q], Pa[ia][cb], 0, 0, 0);
    }
  // M = T P   (T upper triangular 32 x 32); B operand of K-step (ia, q) = Pa[ia][cb][q]
  doublex4 Ma[2][2];
#pragma unroll
  for (int ia = 0; ia < 2; ++ia)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) Ma[ia][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
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
        for (int cb = 0; cb < 2; ++cb)
          Ma[ia][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ta[ia], Pa[kb][cb][q], Ma[ia][cb], 0, 0, 0);
    }
  // Z -= Y M
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = kb * 16 + 4 * q + lr;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const double ya = -yval(rb * 16 + lc, kk);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
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
      for (int cb = 0; cb < 2; ++cb) {
        const int col = c0 + cb * 16 + lc;
        if (col < k) Z[int64_t(row) * k + col] = F[rb][cb][q];
      }
    }
}

}  // namespace

namespace tg {

hipError_t sb_q2_tfactors(hipStream_t st, int n, const double *V2,
                          double *T2) {
  const int nsw = n - 2;
  if (nsw <= 0) return hipSuccess;
  hipLaunchKernelGGL(q2_tfactor_kernel, dim3(sb_smax(n), cdiv(nsw, QB)), dim3(256), 0, st, V2,
                     n, sb_smax(n), T2);
  return hipGetLastError();
}

hipError_t sb_apply_q2(hipStream_t st, int n, double *Z, int k, const double *V2,
                       double *T2) {
  const int nsw = n - 2;
  if (nsw <= 0) return hipSuccess;
  const int smax = sb_smax(n);
  const int ng2 = cdiv(nsw, QB);
  hipLaunchKernelGGL(q2_tfactor_kernel, dim3(smax, ng2), dim3(256), 0, st, V2, n, smax, T2);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  const int nlev = smax + ng2 - 1;
  for (int level = 0; level < nlev; ++level) {
    const int s_lo = std::max(0, level - (ng2 - 1)), s_hi = std::min(smax - 1, level);
    if (s_hi < s_lo) continue;
    const double rows = double(s_hi - s_lo + 1) * QR;
    auto tok = tg::prof_begin(st, tg::PROF_Q2, 16.0 * rows * k, 4.0 * rows * QB * k + 2.0 * QB * QB * k);
    hipLaunchKernelGGL(q2_apply_kernel, dim3(cdiv(k, 128), s_hi - s_lo + 1), dim3(256), 0, st, Z,
                       k, n, V2, T2, smax, ng2, level, s_lo);
    tg::prof_end(st, tok);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

size_t sb2st_t2_count(int n) {
  const int nsw = std::max(1, n - 2);
  return size_t(cdiv(nsw, QB)) * sb_smax(n) * QB * QB;
}

}  // namespace tg

// ---------------------------------------------------------------------------
// C ABI: the band -> tridiagonal stage on its own (tests and tools).
// ---------------------------------------------------------------------------
namespace {
struct BandWs {
  double *Bst, *V2;
  unsigned *prog;
};
template <class A>
void band_ws_layout(A &ar, int n, BandWs *p) {
  BandWs d{};
  BandWs &b = p ? *p : d;
  const size_t nsw = size_t(std::max(1, n - 2)), smax = size_t(tg::sb_smax(n));
  if constexpr (std::is_same_v<A, tg::Arena>) {
    b.Bst = ar.template take<double>(size_t(n) * LDB);
    b.V2 = ar.template take<double>(nsw * smax * SB_B);
    b.prog = ar.template take<unsigned>(tg::sb2st_prog_words(n));
  } else {
    ar.template take<double>(size_t(n) * LDB);
    ar.template take<double>(nsw * smax * SB_B);
    ar.template take<double>(nsw * smax);
    ar.template take<unsigned>(tg::sb2st_prog_words(n));
  }
}
}  // namespace

extern "C" size_t tg_band_tridiag_workspace_size(int n) {
  if (n < 1) return 0;
  tg::Sizer s;
  band_ws_layout(s, n, nullptr);
  return s.off + 256;
}

extern "C" int tg_band_tridiag(void *stream, const double *A, int n, int lda, double *d, double *e,
                               void *ws, size_t ws_bytes) {
  TG_ARG(A != nullptr, 2, "A is null");
  TG_ARG(n >= 1, 3, "n must be >= 1");
  TG_ARG(lda >= n, 4, "lda < n");
  TG_ARG(d != nullptr && e != nullptr, 5, "d / e is null");
  hipStream_t st = static_cast<hipStream_t>(stream);
  tg::Arena ar(ws, ws_bytes);
  BandWs b{};
  band_ws_layout(ar, n, &b);
  TG_WS(ar);
  TG_HIP(tg::sb2st(st, A, lda, n, b.Bst, b.V2, b.prog, d, e));
  bool stalled = false, broken = false;
  TG_HIP(tg::sb2st_stalled(st, n, b.prog, &stalled, &broken));
  if (stalled) {
    tg::set_error("tg_band_tridiag: bulge-chasing pipeline stalled (a hand-off wait timed out)");
    return int(hipErrorLaunchTimeOut);
  }
  if (broken) {
    tg::set_error("tg_band_tridiag: the tridiagonal failed its invariant check (trace / Frobenius "
                  "norm of the band not preserved); d and e are poisoned");
    return int(hipErrorIllegalState);
  }
  return 0;
}
