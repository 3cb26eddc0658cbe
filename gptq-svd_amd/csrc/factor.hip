// Pivot order, R_x and U of the truncated spectral factorisation (A4, A5).
//
// Replaces, in /root/reference/src/TruncGPTQ/gptq_utils.py:
//   H_sqrt = S[:, None] * Vh; jax.scipy.linalg.qr(H_sqrt, pivoting=True)  :112-117
//       (XLA -> MAGMA dgeqp3)                      -> tg_pivoted_factor
//   torch.linalg.qr(H_inv_partial[:, perm]) + sign normalisation        :118-124
//       (cuSOLVER geqrf)                           -> tg_u_factor
//
// Pivot order.  dgeqp3 picks, at step i, the remaining column of largest
// residual norm (first index on ties) and swaps it into position i.  The
// residual column norms of S_k after i Householder steps equal the diagonal
// of the Schur complement of H_k = S_k^T S_k after i pivoted Cholesky steps,
// and the R factor equals the pivoted Cholesky factor (both with positive
// diagonal).  So the pivot sequence (identical swap bookkeeping) and R_x come
// from a greedy diagonal-pivoted Cholesky of H_k (SYRK on FP64 MFMA), one
// launch per pivot; the panel's rank-32 Schur update runs on FP64 MFMA.
//
// U.  U (k x n, upper trapezoidal, positive diagonal) is the R factor of
// A = diag(1/S_k) Vh_k[:, perm].  U^T U = A^T A, so U is the first k rows of
// the upper Cholesky factor of G = A^T A: form G[:k, :] = A[:, :k]^T A on
// FP64 MFMA, then a right-looking blocked Cholesky over those k rows (panel
// factor in LDS, triangular solve across all n columns, MFMA trailing update).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "../../include/truncgptq.h"
#include "common.h"
#include "spin.h"
#include "gemm64.h"
#include "reduce.h"

namespace {

constexpr int PB = 32;    // pivoted-Cholesky panel (steps between Schur updates)
constexpr int CB = 32;    // Cholesky row panel for U
constexpr int PGMAX = 64; // max workgroups of the per-pivot kernel

struct PivWs {
  double *B;     // k x n  S_k-scaled eigenvectors (H_sqrt)
  double *Hk;    // n x n  H_k, then its Schur complements
  double *dsc;   // n      Schur diagonal (by original index)
  double *L;     // n x k  L[r][i] (original row index r, pivot step i)
  double *LT;    // PB x n current panel of L, column-major (coalesced per step)
  double *part;  // 2 x PGMAX
  int32_t *perm; // n      position -> original index
  int32_t *pos;  // n      original index -> position
  unsigned *cnt;
  double *pp;    // PGMAX x PPS  per-workgroup step partials (value, position, row, L row)
  double *bc;    // PPS          last arriver's broadcast (pivot, its L row, swap)
  unsigned *flag;
  // candidate-set pivoting (piv_sel_kernel / piv_fill_kernel)
  int32_t *sstate;  // [0] steps done, [1] steps of the last panel
  int32_t *prow;    // PB  pivot rows of the panel
  double *pinv;     // PB  1 / L[piv][step]
  double *Lpp;      // PB x PB  L rows of the panel's pivots (panel columns)
  double *Hk2;      // n x n  second buffer: the compacted Schur complements alternate
  int32_t *oidx;    // n  new position ps + x -> its compact index in the panel's H_k
  // candidate block (piv_sel_kernel<SEL_SELECT / SEL_STEPS>)
  int32_t *cand;    // SEL + 8: candidate rows, then [SEL] nset, [SEL+1] bp, [SEL+2] brow, [SEL+3] bo
  double *cselv;    // 2: tau, bv (the selection's bound and step-0 maximum)
  int32_t *cidx;    // n: compact index (next panel) -> candidate slot, or -1
  double *Cc;       // SEL x SEL: H_k of the candidate pairs, by slot (both triangles)
};
constexpr int PPS = PB + 8;  // partial / broadcast record (doubles)
constexpr int SEL_WS = 1024;  // = SEL (candidates), for the workspace layout above it
static_assert(PGMAX * PPS % 256 == 0, "slot copy assumes whole rounds of 256 threads");

// The candidate-set pivot order with compacted Schur complements (two n x n
// buffers) for n <= 32768; above (or TG_PIVOT_OLD=1, read per call) the
// cross-workgroup per-pivot path, which needs only one.
inline bool compact_pivot(int n) { return n <= 32768 && getenv("TG_PIVOT_OLD") == nullptr; }

template <class A>
void piv_layout(A &ar, int n, int k, PivWs *p) {
  PivWs d{};
  PivWs &q = p ? *p : d;
  auto take = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<A, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  // the two compacted H_k buffers on 2 MB boundaries (their rows are
  // gathered by the candidate steps and the fill kernel)
  auto take2m = [&](double *&dst, size_t cnt) {
    constexpr size_t AL = size_t(2) << 20;
    if constexpr (std::is_same_v<A, tg::Arena>) dst = ar.template take_aligned<double>(cnt, AL);
    else ar.template take_aligned<double>(cnt, AL);
  };
  take(q.B, size_t(k) * n);
  take(q.pp, size_t(2) * PGMAX * PPS);
  take(q.bc, PPS);
  take(q.flag, 16);
  take2m(q.Hk, size_t(n) * n);
  take(q.dsc, n);
  take(q.L, size_t(n) * k);
  take(q.LT, size_t(PB) * n);
  take(q.part, PGMAX * 2);
  take(q.perm, n);
  take(q.pos, n);
  take(q.cnt, 16);
  take(q.sstate, 16);
  take(q.prow, PB);
  take(q.pinv, PB);
  take(q.Lpp, PB * PB);
  take2m(q.Hk2, compact_pivot(n) ? size_t(n) * n : size_t(1));
  take(q.oidx, n);
  take(q.cand, SEL_WS + 8);
  take(q.cselv, 2);
  take(q.cidx, n);
  take(q.Cc, compact_pivot(n) ? size_t(SEL_WS) * SEL_WS : size_t(1));
}

// B[t][c] = S[t] * Vh[t][c]    (gptq_utils.py:112)
__global__ void scale_rows_kernel(const double *__restrict__ Vh, int ldv, const double *__restrict__ S,
                                  int n, int k, double *__restrict__ B) {
  const int t = blockIdx.y;
  const double s = S[t];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
    B[size_t(t) * n + c] = s * Vh[size_t(t) * ldv + c];
}

// (value, position) argmax with first-position tie break, published for the
// last workgroup, which then swaps perm[i] <-> perm[q].
__device__ inline void argmax_publish(double bv, int bp, int i, int n, PivWs w) {
  __shared__ double sv[256];
  __shared__ int sp[256];
  __shared__ double vals[2];
  const int tid = threadIdx.x;
  sv[tid] = bv;
  sp[tid] = bp;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      const double ov = sv[tid + off];
      const int op = sp[tid + off];
      if (ov > sv[tid] || (ov == sv[tid] && op < sp[tid])) {
        sv[tid] = ov;
        sp[tid] = op;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    vals[0] = sv[0];
    vals[1] = double(sp[0]);
  }
  __syncthreads();
  if (tg::publish_partials(vals, 2, w.part, w.cnt)) {
    if (tid < 64) {  // one wave: lanes cover the partials, fixed butterfly argmax
      const int G = int(gridDim.x);
      double best = -INFINITY;
      int q = n;
      for (int g = tid; g < G; g += 64) {
        const double v = tg::load_partial(&w.part[g]);
        const int p = int(tg::load_partial(&w.part[G + g]));
        if (v > best || (v == best && p < q)) {
          best = v;
          q = p;
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(best, off);
        const int op = __shfl_xor(q, off);
        if (ov > best || (ov == best && op < q)) {
          best = ov;
          q = op;
        }
      }
      if (tid == 0) {
        if (q < n && q != i) {
          const int a = w.perm[i], b = w.perm[q];
          w.perm[i] = b;
          w.perm[q] = a;
          w.pos[b] = i;
          w.pos[a] = q;
        }
        *w.cnt = 0u;
      }
    }
  }
}

// dsc = diag(Hk), perm = identity, first pivot swapped into position 0.
__global__ __launch_bounds__(256) void piv_init_kernel(int n, PivWs w) {
  double bv = -INFINITY;
  int bp = n;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const double v = w.Hk[size_t(j) * n + j];
    w.dsc[j] = v;
    w.perm[j] = j;
    w.pos[j] = j;
    if (v > bv || (v == bv && j < bp)) {
      bv = v;
      bp = j;
    }
  }
  argmax_publish(bv, bp, 0, n, w);
}

// One pivot step i (pivot already swapped into position i).  Threads walk the
// rows in ORIGINAL order (coalesced row of H_k, panel of L^T, Schur diagonal);
// rows already pivoted (pos <= i) are skipped; the argmax breaks ties on the
// dgeqp3 position.
__global__ __launch_bounds__(256) void piv_step_kernel(int n, int k, int i, int ps, PivWs w) {
  __shared__ double lp[PB];
  const int t = i - ps;
  const int piv = w.perm[i];
  const double dpiv = w.dsc[piv];
  const double ljj = sqrt(fmax(dpiv, 0.0));
  if (threadIdx.x < t) lp[threadIdx.x] = w.LT[size_t(threadIdx.x) * n + piv];
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.L[size_t(piv) * k + i] = ljj;
    w.LT[size_t(t) * n + piv] = ljj;
  }
  const double inv = ljj > 0.0 ? 1.0 / ljj : 0.0;
  double bv = -INFINITY;
  int bp = n;
  const double *hrow = w.Hk + size_t(piv) * n;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const int pr = w.pos[r];
    double v = hrow[r];
    double lr[PB];
#pragma unroll
    for (int l = 0; l < PB; ++l) lr[l] = l < t ? w.LT[size_t(l) * n + r] : 0.0;
#pragma unroll
    for (int l = 0; l < PB; ++l) v -= l < t ? lr[l] * lp[l] : 0.0;
    if (pr <= i) continue;
    const double lv = v * inv;
    w.L[size_t(r) * k + i] = lv;
    w.LT[size_t(t) * n + r] = lv;
    const double dn = w.dsc[r] - lv * lv;
    w.dsc[r] = dn;
    if (dn > bv || (dn == bv && pr < bp)) {
      bv = dn;
      bp = pr;
    }
  }
  // dgeqp3 stops after min(k, n) steps: no swap into position k.
  if (i + 1 < k) argmax_publish(bv, bp, i + 1, n, w);
}

// Persistent form of the pivot steps of one panel (steps ps .. pe-1): one
// launch instead of one per pivot.  Thread (block b, lane x) owns rows
// r = (b * 256 + x) + u * G * 256 (u < RPT) and keeps their panel of L in
// registers.  Per step every workgroup publishes its best candidate (Schur
// diagonal, dgeqp3 position, row, and that row's panel of L) with sc1 stores
// and takes an arrival ticket; the last arriver does dgeqp3's swap
// bookkeeping and broadcasts the next pivot (its diagonal, row and L panel)
// plus the swapped pair; the others poll the broadcast flag.  All
// cross-workgroup data moves by sc1 stores + vmcnt(0) + flag/ticket and sc1
// loads (MI355X_MICROARCH.md "Valid forms"), so placement does not matter.
__device__ inline double ld1(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st1(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline int ld1i(const int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st1i(int32_t *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Wave argmax without the LDS crossbar: partner values through
// v_permlane{32,16}_swap (lane ^ 32, ^ 16) and DPP row mirrors / quad perms
// (lane ^ 15, ^ 7, ^ 3, ^ 1); each pairing flips a new lane bit, so after the
// six stages every lane holds the maximum of the strict total order used.
__device__ inline int part32(int x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ inline int part16(int x) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (threadIdx.x & 16) ? r[0] : r[1];
}
template <int CTRL>
__device__ inline int partdpp(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}
template <int S>
__device__ inline int partner(int x) {
  if constexpr (S == 0) return part32(x);
  else if constexpr (S == 1) return part16(x);
  else if constexpr (S == 2) return partdpp<0x140>(x);  // row_mirror: lane ^ 15
  else if constexpr (S == 3) return partdpp<0x141>(x);  // row_half_mirror: lane ^ 7
  else if constexpr (S == 4) return partdpp<0x1B>(x);   // quad_perm [3,2,1,0]: lane ^ 3
  else return partdpp<0xB1>(x);                         // quad_perm [1,0,3,2]: lane ^ 1
}
// (value desc, then p asc, then g asc): the dgeqp3 pivot rule with a
// deterministic workgroup tie-break
template <int S>
__device__ inline void argmax_stage(double &v, int &p, int &g) {
  const double ov = __hiloint2double(partner<S>(__double2hiint(v)), partner<S>(__double2loint(v)));
  const int op = partner<S>(p), og = partner<S>(g);
  if (ov > v || (ov == v && (op < p || (op == p && og < g)))) {
    v = ov;
    p = op;
    g = og;
  }
}
__device__ inline void wave_argmax(double &v, int &p, int &g) {
  argmax_stage<0>(v, p, g);
  argmax_stage<1>(v, p, g);
  argmax_stage<2>(v, p, g);
  argmax_stage<3>(v, p, g);
  argmax_stage<4>(v, p, g);
  argmax_stage<5>(v, p, g);
}

// Worker selection: the launch has at least 8 (G - 1) + 1 workgroups; each
// takes a ticket on its XCD (HW_REG_XCC_ID) and the first XCD to hand out G
// tickets becomes the worker set (pigeonhole: one always does); the others
// exit.  Workers then hand data over through that XCD's L2: plain stores +
// vmcnt(0) + agent atomic ticket, sc1 (L1-bypassing) loads.
#ifdef TG_PIV_PHASES
__device__ unsigned long long g_pivph[8];
#define PVT(i)                                                                 \
  {                                                                            \
    const uint64_t tt = __builtin_amdgcn_s_memrealtime();                      \
    if (i > 0 && tid == 0 && me == 0) atomicAdd(g_pivph + i - 1, tt - pvt_last); \
    pvt_last = tt;                                                             \
  }
#else
#define PVT(i)
#endif

template <int RPT>
__global__ __launch_bounds__(256) void piv_panel_kernel(int n, int k, int ps, int pe, int G,
                                                        unsigned base, PivWs w) {
  extern __shared__ int permL[];  // n: position -> row (every workgroup keeps a copy)
  __shared__ double sv[4], lrow[PB + 1];
  __shared__ int spos[4], swin[4], s_g, s_me;
  __shared__ double s_best;
  __shared__ double slotc[PGMAX * PPS];
  __shared__ double wrow[4][PB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    unsigned *xc = w.flag + 4;  // [0..7] tickets per XCD, [8] chosen XCD + 1
    const unsigned tk = __hip_atomic_fetch_add(xc + (x & 7), 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    int me = -1;
    if (tk < unsigned(G)) {
      if (tk == unsigned(G) - 1) {
        unsigned expect = 0;
        __hip_atomic_compare_exchange_strong(xc + 8, &expect, x + 1, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      unsigned ch;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((ch = __hip_atomic_load(xc + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
      }
      if (ch == x + 1) me = int(tk);
    }
    s_me = me;
  }
  __syncthreads();
  const int me = s_me;
  if (me < 0) return;
  for (int x = tid; x < n; x += 256) permL[x] = w.perm[x];
  // base = arrivals of earlier panel launches (G per step before ps), from the host
  int rows[RPT], posr[RPT];
  double dsr[RPT], lr[RPT][PB];
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    rows[u] = me * 256 + tid + u * G * 256;
    const bool ok = rows[u] < n;
    posr[u] = ok ? w.pos[rows[u]] : n;
    dsr[u] = ok ? w.dsc[rows[u]] : 0.0;
#pragma unroll
    for (int l = 0; l < PB; ++l) lr[u][l] = 0.0;
  }
  __syncthreads();
  int piv = permL[ps];
  double dpiv = w.dsc[piv];
  // H_k[piv][row] for the next step, loaded as soon as the pivot is known
  double hv[RPT];
#pragma unroll
  for (int u = 0; u < RPT; ++u) hv[u] = w.Hk[size_t(piv) * n + min(rows[u], n - 1)];
#ifdef TG_PIV_PHASES
  uint64_t pvt_last = 0;
#endif
  for (int i = ps; i < pe; ++i) {
    const int t = i - ps;
    PVT(0)
    const double ljj = sqrt(fmax(dpiv, 0.0));
    const double inv = ljj > 0.0 ? 1.0 / ljj : 0.0;
    double bv = -INFINITY;
    int bp = n, bu = -1;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int r = rows[u];
      if (r >= n) continue;
      if (r == piv) {  // the pivot row itself
#pragma unroll
        for (int l = 0; l < PB; ++l)
          if (l == t) lr[u][l] = ljj;
        continue;
      }
      if (posr[u] <= i) continue;
      double v = hv[u];
#pragma unroll
      for (int l = 0; l < PB; ++l) v -= l < t ? lr[u][l] * lrow[l] : 0.0;
      const double lv = v * inv;
#pragma unroll
      for (int l = 0; l < PB; ++l)
        if (l == t) lr[u][l] = lv;
      dsr[u] -= lv * lv;
      if (dsr[u] > bv || (dsr[u] == bv && posr[u] < bp)) {
        bv = dsr[u];
        bp = posr[u];
        bu = u;
      }
    }
    PVT(1)
    if (i + 1 >= k) break;  // dgeqp3 stops after k steps: no swap into position k
    // workgroup candidate (largest diagonal, first dgeqp3 position); each
    // wave's winning lane stages its row and L row in LDS
    int bw = tid;
    wave_argmax(bv, bp, bw);
    if (lane == 0) {
      sv[wid] = bv;
      spos[wid] = bp;
      swin[wid] = bw;
    }
    if (tid == bw && bu >= 0) {
#pragma unroll
      for (int u = 0; u < RPT; ++u)
        if (u == bu) {
          wrow[wid][0] = double(rows[u]);
#pragma unroll
          for (int l = 0; l < PB; ++l) wrow[wid][1 + l] = lr[u][l];
        }
    }
    __syncthreads();
    PVT(2)
    int wq = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q)
      if (sv[q] > sv[wq] || (sv[q] == sv[wq] && spos[q] < spos[wq])) wq = q;
    // publish: value, position, row, the row's L panel (slot parity = step parity)
    double *mine = w.pp + (size_t(i & 1) * PGMAX + me) * PPS;
    if (wid == 0) {  // one parallel store: [0] value, [1] position, [2] row, [8 + l] L row
      if (lane < 3) mine[lane] = lane == 0 ? sv[wq] : (lane == 1 ? double(spos[wq]) : wrow[wq][0]);
      else if (lane >= 8 && lane - 8 <= t) mine[lane] = wrow[wq][lane - 7];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    PVT(3)
    // all-to-all: wait for every workgroup's candidate of this step
    // wave 0 as a whole wave (scalar loop, spin.h): arrive, bounded poll; a
    // stall sets flag[15] and ends every later wait of the launch at once
    if (__builtin_amdgcn_readfirstlane(wid) == 0) {
      tg::wave_arrive(w.cnt);
      const unsigned target = base + unsigned(G) * unsigned(t + 1);
      s_me = tg::spin_geq(w.cnt, target, w.flag + 15, 200000000ull) ? 0 : -1;
    }
    __syncthreads();
    if (s_me < 0) return;
    PVT(4)
    // every workgroup's record (value, position, row, L row) in one round of
    // parallel sc1 loads, so the winner's L row needs no second round trip
    const double *slots = w.pp + size_t(i & 1) * PGMAX * PPS;
    {
      const int nrec = G * PPS;
      double tmp[PGMAX * PPS / 256];
#pragma unroll
      for (int u = 0; u < PGMAX * PPS / 256; ++u) {
        const int x = tid + u * 256;
        tmp[u] = x < nrec ? ld1(slots + x) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < PGMAX * PPS / 256; ++u) {
        const int x = tid + u * 256;
        if (x < nrec) slotc[x] = tmp[u];
      }
    }
    __syncthreads();
    PVT(5)
    if (wid == 0) {
      double v = -INFINITY;
      int p2 = n, g = lane;
      if (lane < G) {
        v = slotc[lane * PPS];
        p2 = int(slotc[lane * PPS + 1]);
      }
      wave_argmax(v, p2, g);
      if (lane == 0) {
        s_best = v;
        s_g = g;
        spos[0] = p2;
      }
    }
    __syncthreads();
    const int g = min(max(s_g, 0), G - 1), q = min(max(spos[0], i + 1), n - 1);
    const double *win = slotc + g * PPS;
    if (tid <= t) lrow[tid] = win[8 + tid];
    const int rowb = min(max(int(win[2]), 0), n - 1);
#pragma unroll
    for (int u = 0; u < RPT; ++u) hv[u] = w.Hk[size_t(rowb) * n + min(rows[u], n - 1)];
    const int a = permL[i + 1];
    __syncthreads();
    PVT(6)
    if (tid == 0 && q != i + 1) {  // dgeqp3 swap of positions i+1 and q (every copy)
      permL[i + 1] = rowb;
      permL[q] = a;
      if (me == 0) {
        w.perm[i + 1] = rowb;
        w.perm[q] = a;
        w.pos[rowb] = i + 1;
        w.pos[a] = q;
      }
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      if (rows[u] == rowb) posr[u] = i + 1;
      else if (rows[u] == a && q != i + 1) posr[u] = q;
    }
    dpiv = s_best;
    piv = rowb;
    __syncthreads();
    PVT(7)
  }
  // the panel's L columns, once: row-contiguous into L, coalesced into LT
  const int pw = min(pe, k) - ps;
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const int r = rows[u];
    if (r >= n) continue;
    w.dsc[r] = dsr[u];
#pragma unroll
    for (int l = 0; l < PB; ++l) {
      if (l < pw) {
        w.L[size_t(r) * k + ps + l] = lr[u][l];
        w.LT[size_t(l) * n + r] = lr[u][l];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Candidate-set pivoting: one workgroup picks a whole panel's pivots.
//
// Schur diagonals only decrease.  At the start of a panel the rows with the
// (about) SEL largest diagonals form the candidate set C; every other
// unpivoted row stays <= tau = max of their diagonals at panel start.  Step
// 0 of the panel is a full argmax.  At a later step, if the best candidate
// (diagonal desc, dgeqp3 position asc) is strictly above tau it is the exact
// dgeqp3 choice; otherwise the panel ends there (fewer than PB steps) and the
// next panel re-selects.  Only candidates carry their panel of L (one per
// thread, in registers), so a step costs one H_k load and two workgroup
// barriers instead of an all-to-all across workgroups.  piv_fill_kernel then
// computes the panel's L columns and diagonals of ALL rows with the same
// operation sequence (explicit fma), so candidates and the rest agree bit
// for bit.  Selection: two 11-bit radix passes on the diagonal's bit pattern
// (positive doubles order like their bits), set = rows strictly above the
// crossing bin (|set| <= SEL).
// The candidate-set path keeps H_k compacted: at a panel starting at step ps
// the Schur complement of the unpivoted rows is the leading (n - ps)^2 block,
// row / column x holding the row at position ps + x (leading dimension n).
// Each panel's Schur update writes the next compacted block into the other
// buffer (syrk_compact_kernel), so the update touches (n - ps)^2 entries
// instead of n^2 and a pivot's row is contiguous.
constexpr int SEL = SEL_WS;       // candidates
constexpr int SEL_LDS_N = 8192;  // n up to which piv_sel_kernel stages diagonals in LDS

#ifdef TG_SEL_PHASES
__device__ unsigned long long g_selph[16];
#define SELT(i)                                                     \
  {                                                                 \
    const uint64_t tt = __builtin_amdgcn_s_memtime();               \
    if (i > 0 && threadIdx.x == 0) atomicAdd(g_selph + i - 1, tt - selt_last); \
    selt_last = tt;                                                 \
  }
#else
#define SELT(i)
#endif

__device__ inline unsigned long long dkey(double d) {
  return d > 0.0 ? static_cast<unsigned long long>(__double_as_longlong(d)) : 0ull;
}

// The compacted H_k buffers keep only their lower triangle (the Schur update
// writes no mirror): entry (a, b) is read at (max, min).  The first panel's
// H_k is the full matrix, for which that is the same entry.
__device__ __forceinline__ size_t hk_at(int a, int b, int n) {
  return size_t(max(a, b)) * n + min(a, b);
}

constexpr int STH = 512;        // threads of piv_sel_kernel (8 waves)
constexpr int CPT = SEL / STH;  // candidates per thread

// Block argmax of (v desc, p asc) carrying a row id r (positions are
// unique).  Wave stage: the maximum of v alone through six exchange stages
// (v_permlane{32,16}_swap pairs, DPP row mirrors / quad perms) with v_max_f64,
// then the holder found by a ballot; only a tie on v (rare: exhausted
// candidates at -inf) takes the slower min-position pass.  One barrier; the
// eight wave records are merged by every thread with selects.
// v_max_f64 without the operand canonicalisation fmax() adds for values that
// come out of lane exchanges
__device__ inline double vmax_d(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ inline double sel_pair_max(double x, bool half16) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  if (half16) {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return vmax_d(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
  }
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return vmax_d(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
}
template <int CTRL>
__device__ inline double sel_dpp(double x) {
  return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false),
                          __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false));
}
__device__ inline double wave_max_d(double x) {
  x = sel_pair_max(x, false);
  x = sel_pair_max(x, true);
  x = vmax_d(x, sel_dpp<0x140>(x));  // lane ^ 15
  x = vmax_d(x, sel_dpp<0x141>(x));  // lane ^ 7
  x = vmax_d(x, sel_dpp<0x1B>(x));   // lane ^ 3
  return vmax_d(x, sel_dpp<0xB1>(x));  // lane ^ 1
}
template <int S>
__device__ inline int wave_min_stage(int x) {
  return min(x, partner<S>(x));
}
__device__ inline void block_argmax_sel(double &v, int &p, int &r, int &o, double2 *rec,
                                        int *reco) {
  const double m = wave_max_d(v);
  const bool hold = v == m;
  const unsigned long long b = __ballot(hold);
  int L = __ffsll(static_cast<long long>(b)) - 1;
  // tie on v: smallest position among the holders (uniform branch).  A wave
  // whose candidates are all exhausted (every lane at -inf) skips it: its
  // record cannot win unless every wave's is -inf, and then the panel ends
  if (__popcll(b) > 1 && m != -INFINITY) {
    int pp = hold ? p : INT_MAX;
    pp = wave_min_stage<0>(pp);
    pp = wave_min_stage<1>(pp);
    pp = wave_min_stage<2>(pp);
    pp = wave_min_stage<3>(pp);
    pp = wave_min_stage<4>(pp);
    pp = wave_min_stage<5>(pp);
    L = __ffsll(static_cast<long long>(__ballot(hold & (p == pp)))) - 1;
  }
  const int wp = __builtin_amdgcn_readlane(p, L), wr = __builtin_amdgcn_readlane(r, L);
  const int wo = __builtin_amdgcn_readlane(o, L);
  if ((threadIdx.x & 63) == 0) {
    rec[threadIdx.x >> 6] = make_double2(m, __hiloint2double(wp, wr));
    reco[threadIdx.x >> 6] = wo;
  }
  __syncthreads();
  double2 x[STH / 64];
#pragma unroll
  for (int q = 0; q < STH / 64; ++q) x[q] = rec[q];
  v = x[0].x;
#pragma unroll
  for (int q = 1; q < STH / 64; ++q) v = vmax_d(v, x[q].x);
  p = INT_MAX;
  r = 0;
  o = 0;
#pragma unroll
  for (int q = 0; q < STH / 64; ++q) {
    const int op = __double2hiint(x[q].y);
    const bool take = (x[q].x == v) & (op < p);
    p = take ? op : p;
    r = take ? __double2loint(x[q].y) : r;
    o = take ? reco[q] : o;
  }
}

// Radix-select histograms: 2048 bins padded by one word per 32 (bin b at
// b + b / 32), so the scan's lanes (one 32-bin block each) read conflict-free.
constexpr int HPAD = 2048 + 64;
__device__ inline int hidx(int b) { return b + (b >> 5); }

// Wave-aggregated histogram increment: the exponent bins of one wave's keys
// are few (diagonals of similar scale), so one atomic per distinct bin instead
// of 64 same-address atomics.  Uniform loop over the distinct bins.
__device__ inline void hist_add_agg(unsigned *hist, int bin, bool ok, int lane) {
  unsigned long long pend = __ballot(ok);
  while (pend) {
    const int L = __ffsll(static_cast<long long>(pend)) - 1;
    const int b = __builtin_amdgcn_readlane(bin, L);
    const unsigned long long same = __ballot(ok & (bin == b));
    if (lane == L) atomicAdd(&hist[hidx(b)], unsigned(__popcll(same)));
    pend &= ~same;
  }
}

// Wave 0: crossing bin of the `target`-th largest key (bins scanned top-down;
// lane L holds block 63 - L in registers) and the count strictly above it, to
// out[0..1] (LDS).  Written only when the target is reached.
__device__ inline void hist_scan(const unsigned *hist, int target, int *out) {
  const int lane = threadIdx.x & 63, blk = 63 - lane;
  int c[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) c[j] = int(hist[blk * 33 + 31 - j]);  // bin 32 blk + 31 - j
  int sum = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) sum += c[j];
  int pre = sum;  // inclusive prefix over lanes (top blocks first)
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(pre, off);
    pre += lane >= off ? o : 0;
  }
  int acc = pre - sum;
  if (acc < target && pre >= target) {
    int cb = 0, cbefore = 0;
    bool found = false;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const bool hit = !found & (acc + c[j] >= target);
      cb = hit ? j : cb;
      cbefore = hit ? acc : cbefore;
      found = found | hit;
      acc += c[j];
    }
    out[0] = blk * 32 + 31 - cb;
    out[1] = cbefore;
  }
}

// Modes of piv_sel_kernel.  SEL_FULL: candidate selection, then the panel's
// steps (pivot rows gathered from the compacted H_k).  The candidate-block
// form (the default; TG_PIV_CC=0 keeps SEL_FULL) splits it around the
// previous panel's Schur update (TG_PIV_CC=1; measured no faster, see
// DESIGN.md): SEL_SELECT picks the candidates first and
// maps their compact indices (w.cidx, tagged with the panel start), the
// update then also writes H_k of every candidate pair into the SEL x SEL
// block w.Cc (syrk_compact_p_kernel's epilogue, exact copies of the values it
// stores), and SEL_STEPS runs the steps reading a pivot's row of candidate
// entries as 8 KB contiguous from Cc instead of ~1024 scattered lines of H_k
// (half of them column reads of the lower-triangle storage: the TA-bound
// part of a step).  Same values, same operations: perm and R_x are
// bit-identical.
enum { SEL_FULL = 0, SEL_SELECT = 1, SEL_STEPS = 2 };
constexpr int CC_TAG = 11;  // cidx = (panel start << CC_TAG) | slot
static_assert((1 << CC_TAG) > SEL, "slot field");

template <int MODE>
__global__ __launch_bounds__(STH) void piv_sel_kernel(int n, int k, PivWs w,
                                                      const double *__restrict__ Hc) {
  extern __shared__ int permL[];  // n: position -> row
  __shared__ unsigned hist[HPAD];
  __shared__ int cand[SEL + 1];  // + trash slot for branch-free compaction
  __shared__ double2 rec[STH / 64];
  __shared__ int reco[STH / 64];
  __shared__ double sv[STH / 64];
  __shared__ int scnt[STH / 64];
  __shared__ int sel[4];
  __shared__ double lrow[PB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ps = w.sstate[0];
  if (ps >= k) {
    if (tid == 0 && MODE != SEL_SELECT) w.sstate[1] = 0;
    return;
  }
  const int pe = min(ps + PB, k);
#ifdef TG_SEL_PHASES
  uint64_t selt_last = 0;
#endif
  SELT(0)
  int nset, bp, brow, bo;
  double tau, bv;
  const double *dS;
  const int32_t *pS;
  if constexpr (MODE == SEL_STEPS) {
    // the selection SEL_SELECT made before the Schur update
    for (int x = tid; x < n; x += STH) permL[x] = w.perm[x];
    for (int c = tid; c < SEL; c += STH) cand[c] = w.cand[c];
    nset = w.cand[SEL];
    bp = w.cand[SEL + 1];
    brow = w.cand[SEL + 2];
    bo = w.cand[SEL + 3];
    tau = w.cselv[0];
    bv = w.cselv[1];
    dS = w.dsc;
    pS = w.pos;
    __syncthreads();
  } else {
  // Schur diagonals and positions: staged in LDS once for n <= SEL_LDS_N (the
  // selection passes below read them three times), else read from HBM/L2
  const bool staged = n <= SEL_LDS_N;
  double *dsh = reinterpret_cast<double *>(permL + ((n + 1) & ~1));
  int *posh = reinterpret_cast<int *>(dsh + n);
  if (staged) {
    for (int r0 = tid; r0 < n; r0 += 8 * STH) {
      double dv[8];
      int pv[8], mv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // one batch of loads in flight
        const int r = min(r0 + u * STH, n - 1);
        dv[u] = w.dsc[r];
        pv[u] = w.pos[r];
        mv[u] = w.perm[r];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r0 + u * STH < n) {
          dsh[r0 + u * STH] = dv[u];
          posh[r0 + u * STH] = pv[u];
          permL[r0 + u * STH] = mv[u];
        }
    }
  } else {
    for (int x = tid; x < n; x += STH) permL[x] = w.perm[x];
  }
  for (int x = tid; x < HPAD; x += STH) hist[x] = 0u;
  if (tid == 0) {
    sel[0] = -1;  // b1 (-1: every positive key is a candidate)
    sel[2] = -1;  // b2
  }
  __syncthreads();
  SELT(9)
  dS = staged ? dsh : w.dsc;
  pS = staged ? posh : w.pos;
  // --- candidate set ---------------------------------------------------------
  // one sweep: count of unpivoted rows with positive keys + exponent histogram
  int valid = 0;
  for (int r0 = tid; r0 < n; r0 += 8 * STH) {
    double dv[8];
    int pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = min(r0 + u * STH, n - 1);
      dv[u] = dS[r];
      pv[u] = pS[r];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const unsigned long long key = dkey(dv[u]);
      const bool ok = (r0 + u * STH < n) & (pv[u] >= ps) & (key != 0ull);
      valid += ok;
      hist_add_agg(hist, int(key >> 52), ok, lane);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) valid += __shfl_xor(valid, off);
  if (lane == 0) scnt[wid] = valid;
  __syncthreads();
  valid = 0;
#pragma unroll
  for (int q = 0; q < STH / 64; ++q) valid += scnt[q];
  SELT(10)
  if (valid > SEL) {  // uniform
    if (wid == 0) hist_scan(hist, SEL, sel);  // sel[0] = b1, sel[1] = count above
    __syncthreads();
    for (int x = tid; x < HPAD; x += STH) hist[x] = 0u;
    __syncthreads();
    const int b1 = sel[0];
    for (int r0 = tid; r0 < n; r0 += 8 * STH) {
      double dv[8];
      int pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = min(r0 + u * STH, n - 1);
        dv[u] = dS[r];
        pv[u] = pS[r];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const unsigned long long key = dkey(dv[u]);
        if ((r0 + u * STH < n) & (pv[u] >= ps) & (int(key >> 52) == b1))
          atomicAdd(&hist[hidx(int(key >> 41) & 2047)], 1u);  // mantissa bins: spread
      }
    }
    __syncthreads();
    if (wid == 0) hist_scan(hist, SEL - sel[1], sel + 2);
    __syncthreads();
  }
  SELT(11)
  const int b1 = sel[0], b2 = sel[2];
  // compaction of the set, tau over the rest, full argmax for step 0 (branch-free;
  // membership kept as one bit per row of this thread: n <= 64 STH)
  int mine = 0;
  tau = -INFINITY;
  bv = -INFINITY;
  bp = n;
  brow = 0;
  unsigned long long insm = 0ull;
  for (int r0 = tid, bi = 0; r0 < n; r0 += 8 * STH, bi += 8) {
    double dv[8];
    int pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = min(r0 + u * STH, n - 1);
      dv[u] = dS[r];
      pv[u] = pS[r];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool un = (r0 + u * STH < n) & (pv[u] >= ps);
      const unsigned long long key = dkey(dv[u]);
      const int d1 = int(key >> 52), d2 = int(key >> 41) & 2047;
      const bool ins = un & (key != 0ull) & ((b1 < 0) | (d1 > b1) | ((d1 == b1) & (d2 > b2)));
      mine += ins;
      insm |= static_cast<unsigned long long>(ins) << (bi + u);
      tau = (un & !ins) ? fmax(tau, dv[u]) : tau;
      const bool take = un & ((dv[u] > bv) | ((dv[u] == bv) & (pv[u] < bp)));
      bv = take ? dv[u] : bv;
      bp = take ? pv[u] : bp;
      brow = take ? r0 + u * STH : brow;
    }
  }
  {
    int pre = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(pre, off);
      pre += lane >= off ? o : 0;
    }
    double t2 = tau;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t2 = fmax(t2, __shfl_xor(t2, off));
    __syncthreads();  // scnt reuse
    if (lane == 63) scnt[wid] = pre;
    if (lane == 0) sv[wid] = t2;
    __syncthreads();
    int base = 0;
    tau = -INFINITY;
#pragma unroll
    for (int q = 0; q < STH / 64; ++q) {
      base += q < wid ? scnt[q] : 0;
      tau = fmax(tau, sv[q]);
    }
    int slot = base + pre - mine;
    for (int r0 = tid, bi = 0; r0 < n; r0 += 8 * STH, bi += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ins = (insm >> (bi + u)) & 1ull;
        cand[ins ? slot : SEL] = r0 + u * STH;  // non-members to the trash slot
        slot += ins;
      }
    }
  }
  __syncthreads();
  SELT(12)
  nset = 0;
#pragma unroll
  for (int q = 0; q < STH / 64; ++q) nset += scnt[q];
  bo = bp - ps;  // compact index of the step-0 pivot (positions unchanged so far)
  block_argmax_sel(bv, bp, brow, bo, rec, reco);
  if constexpr (MODE == SEL_SELECT) {
    for (int c = tid; c < nset; c += STH) {
      w.cand[c] = cand[c];
      // compact index (this panel's numbering) -> slot, tagged with the panel
      // start so entries of earlier panels never match (one store per entry)
      w.cidx[pS[cand[c]] - ps] = (ps << CC_TAG) | c;
    }
    if (tid == 0) {
      w.cand[SEL] = nset;
      w.cand[SEL + 1] = bp;
      w.cand[SEL + 2] = brow;
      w.cand[SEL + 3] = bo;
      w.cselv[0] = tau;
      w.cselv[1] = bv;
    }
    return;
  }
  }  // MODE != SEL_STEPS
  int rc[CPT], posc[CPT], oc[CPT];
  double dc[CPT];
  bool done[CPT];
  double lr[CPT][PB];
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int c = tid + u * STH;
    rc[u] = c < nset ? cand[c] : -1;
    posc[u] = rc[u] >= 0 ? pS[rc[u]] : n;
    oc[u] = rc[u] >= 0 ? posc[u] - ps : 0;  // compact index in this panel's H_k
    dc[u] = rc[u] >= 0 ? dS[rc[u]] : -INFINITY;
    done[u] = rc[u] < 0;
#pragma unroll
    for (int l = 0; l < PB; ++l) lr[u][l] = 0.0;
  }
  int piv = brow, q = bp, opiv = bo;
  int cpiv = -1;  // SEL_STEPS: the pivot's candidate slot (step 0: from H_k)
  double dpiv = bv;
  int tdone = 0;
  SELT(1)
  // steps unrolled: the panel column t is a compile-time register index
  bool active = true;  // uniform
  // one instantiation per panel column t: lr[u][t] is a static register index
  auto step = [&]<int t>(std::integral_constant<int, t>) __attribute__((always_inline)) {
    const int i = ps + t;
    active = active && i < pe;
    if (!active) return;
    if (t > 0) {  // candidate argmax; exact only above tau
      double v = -INFINITY;
      int p = n, r = -1, o = 0;
#pragma unroll
      for (int u = 0; u < CPT; ++u) {
        const bool take = !done[u] & ((dc[u] > v) | ((dc[u] == v) & (posc[u] < p)));
        v = take ? dc[u] : v;
        p = take ? posc[u] : p;
        r = take ? rc[u] : r;
        // SEL_STEPS: the candidate slot rides along above the compact index
        o = take ? (MODE == SEL_STEPS ? oc[u] | ((tid + u * STH + 1) << 16) : oc[u]) : o;
      }
      SELT(4)
      block_argmax_sel(v, p, r, o, rec, reco);
      SELT(5)
      active = v > tau;
      if (!active) return;
      dpiv = v;
      q = p;
      piv = r;
      opiv = MODE == SEL_STEPS ? (o & 0xffff) : o;
      cpiv = MODE == SEL_STEPS ? (o >> 16) - 1 : -1;
    }
    double hv[CPT];
    if (MODE == SEL_STEPS && cpiv >= 0) {  // uniform: the pivot's candidate row of Cc
      const double *crow = w.Cc + size_t(cpiv) * SEL;
#pragma unroll
      for (int u = 0; u < CPT; ++u) hv[u] = crow[tid + u * STH];
    } else {
#pragma unroll
      for (int u = 0; u < CPT; ++u)  // H_k[piv][candidate], issued before the hand-off
        hv[u] = Hc[hk_at(opiv, oc[u], n)];  // unconditional; masked below
    }
#pragma unroll
    for (int u = 0; u < CPT; ++u)
      if (rc[u] == piv) {
#pragma unroll
        for (int l = 0; l < t; ++l) lrow[l] = lr[u][l];
      }
    if (tid == 0) {
      const int a = permL[i];
      if (q != i) {
        permL[i] = piv;
        permL[q] = a;
      }
      w.prow[t] = piv;
    }
    SELT(2)
    __syncthreads();
    SELT(3)
    // the pivot's sqrt / reciprocal after the barrier: their latency overlaps
    // the update's fma chains below, which need inv only at their end
    const double ljj = sqrt(fmax(dpiv, 0.0));
    const double inv = ljj > 0.0 ? 1.0 / ljj : 0.0;
    if (tid == 0) w.pinv[t] = inv;
    if (tid <= t) w.Lpp[t * PB + tid] = tid < t ? lrow[tid] : ljj;
    double lrw[PB > 1 ? PB : 1];
#pragma unroll
    for (int l = 0; l < t; ++l) lrw[l] = lrow[l];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {  // branch-free: every slot computes, selects keep
      const bool isp = rc[u] == piv;  // the pivot: dgeqp3 swap of positions i and q
      const bool upd = !done[u] & !isp;
      double v = hv[u];
#pragma unroll
      for (int l = 0; l < t; ++l) v = fma(-lr[u][l], lrw[l], v);
      const double lv = v * inv;
      lr[u][t] = isp ? ljj : (upd ? lv : lr[u][t]);
      dc[u] = upd ? fma(-lv, lv, dc[u]) : dc[u];
      const int pswap = ((posc[u] == i) & (q != i)) ? q : posc[u];
      posc[u] = isp ? i : (upd ? pswap : posc[u]);
      done[u] = done[u] | isp;
    }
    tdone = t + 1;
#ifdef TG_SEL_PHASES
    if (tid == 0) atomicAdd(g_selph + 15, 1ull);
#endif
  };
  [&]<int... Ts>(std::integer_sequence<int, Ts...>) __attribute__((always_inline)) {
    (step(std::integral_constant<int, Ts>{}), ...);
  }(std::make_integer_sequence<int, PB>{});
  SELT(6)
  __syncthreads();
  // compact index (in this panel's H_k) of the row now at position x >= ps:
  // read from the panel-start positions before they are overwritten
  for (int x = ps + tid; x < n; x += STH) w.oidx[x - ps] = pS[permL[x]] - ps;
  __syncthreads();
  for (int x = tid; x < n; x += STH) {
    const int r = permL[x];
    w.perm[x] = r;
    w.pos[r] = x;
  }
  if (tid == 0) {
    w.sstate[0] = ps + tdone;
    w.sstate[1] = tdone;
  }
}

// The last panel's L columns (L row-major by row; LT panel column-major by
// the NEXT panel's compact index) and Schur diagonals of every row still
// unpivoted at the panel start, with piv_sel_kernel's operation sequence.
// One thread per position x >= ps (row perm[x], compact index oidx[x - ps]
// in the panel's H_k block Hc); rows pivoted in the panel (x < ps + tn) get
// their L entries and no LT column.
template <int FT>
__global__ __launch_bounds__(FT) void piv_fill_kernel(int n, int k, PivWs w,
                                                      const double *__restrict__ Hc) {
  __shared__ double lpp[PB][PB + 1];
  __shared__ double pinv[PB];
  __shared__ int prow[PB], poi[PB];
  __shared__ double lst[FT][PB + 1];  // the block's L rows, for row-contiguous stores
  __shared__ int rst[FT];
  const int tid = threadIdx.x;
  const int tn = w.sstate[1];
  if (tn <= 0) return;
  const int ps = w.sstate[0] - tn, ps2 = ps + tn;
  for (int x = tid; x < PB * PB; x += FT) {
    const int i = x / PB, l = x % PB;
    lpp[i][l] = (i < tn && l <= i) ? w.Lpp[x] : 0.0;
  }
  if (tid < PB) {
    pinv[tid] = tid < tn ? w.pinv[tid] : 0.0;
    prow[tid] = tid < tn ? w.prow[tid] : -1;
    poi[tid] = tid < tn ? w.oidx[tid] : 0;  // pivot i sits at position ps + i
  }
  __syncthreads();
  const int x = ps + blockIdx.x * FT + tid;
  const bool valid = x < n;  // no early exit: the L rows go out through LDS below
  const int xc = valid ? x : n - 1;
  const int r = w.perm[xc], oi = w.oidx[xc - ps];
  double hv[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) hv[i] = i < tn ? Hc[hk_at(poi[i], oi, n)] : 0.0;
  double d = w.dsc[r];
  double lr[PB];
  bool done = false;
  // branch-free (selects, no exec-mask regions around each step, so the
  // broadcast LDS reads of row i of the pivots' L are not serialised behind
  // per-step waits): an inactive step (past the panel's steps, or after this
  // row was pivoted) keeps lr = 0 and d, and its fma terms with lr = 0 leave
  // the later sums unchanged -- the same values as the branchy loop
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    double v = hv[i];
#pragma unroll
    for (int l = 0; l < i; ++l) v = fma(-lr[l], lpp[i][l], v);
    const double lv = v * pinv[i];
    const bool act = (i < tn) & !done, isp = prow[i] == r;
    lr[i] = act ? (isp ? lpp[i][i] : lv) : 0.0;
    d = (act & !isp) ? fma(-lv, lv, d) : d;
    done = done | (act & isp);
  }
  if (valid) w.dsc[r] = d;
#pragma unroll
  for (int l = 0; l < PB; ++l) {
    if (valid && x >= ps2) w.LT[size_t(l) * n + (x - ps2)] = lr[l];
    lst[tid][l] = lr[l];
  }
  rst[tid] = valid ? r : -1;
  __syncthreads();
  // L is row-major by row id (rows scattered): 32 lanes write one row's
  // panel segment contiguously instead of every lane striding k apart
  const int hw = tid >> 5, l = tid & 31;
  for (int t = hw; t < FT; t += FT / 32) {
    const int rr = rst[t];
    if (rr >= 0 && l < tn) w.L[size_t(rr) * k + ps + l] = lst[t][l];
  }
}

typedef double doublex4 __attribute__((ext_vector_type(4)));

// Next panel's compacted H_k: Hn[i][j] = Hc[oidx[tn + i]][oidx[tn + j]]
// - sum_l LT[l][i] LT[l][j] for n - ps2 > i >= j (ps2 = steps done after the
// panel, tn its steps) on 64 x 64 lower tiles: the lower triangle only (8
// bytes per entry of the block read and written instead of 12 with the
// mirror; every reader takes (max, min), hk_at).  The entries are the values
// the mirrored form wrote, bit for bit (a diagonal tile's (a, b) and (b, a)
// are the same products summed in the same order).  The grid covers the
// whole n x n lower triangle; tiles past the block exit.
__global__ __launch_bounds__(256) void syrk_compact_kernel(int n, PivWs w,
                                                           const double *__restrict__ Hc,
                                                           double *__restrict__ Hn, int mirror) {
  __shared__ double li[PB][64], lj[PB][64];
  __shared__ double tt[64][65];
  __shared__ int orow[64], ocol[64];
  const int tid = threadIdx.x;
  const int ps2 = w.sstate[0], tn = max(w.sstate[1], 0);
  const int nc = n - ps2;
  const int b = blockIdx.x;
  int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  const int J = b - I * (I + 1) / 2;
  const int i0 = 64 * I, j0 = 64 * J;
  if (i0 >= nc) return;
  if (tid < 64) {
    orow[tid] = w.oidx[tn + min(i0 + tid, nc - 1)];
  } else if (tid < 128) {
    ocol[tid - 64] = w.oidx[tn + min(j0 + tid - 64, nc - 1)];
  }
  for (int e = tid; e < PB * 64; e += 256) {
    const int l = e >> 6, c = e & 63;
    li[l][c] = w.LT[size_t(l) * n + min(i0 + c, nc - 1)];
    lj[l][c] = w.LT[size_t(l) * n + min(j0 + c, nc - 1)];
  }
  __syncthreads();
  // rank-PB update on FP64 MFMA: waves 2 x 2 over the tile, 2 x 2 blocks of
  // 16 x 16 each; the accumulators start from the gathered old values
  const int lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;
  doublex4 acc[2][2];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[ib][jb][q] = Hc[hk_at(orow[wm * 32 + ib * 16 + lk + 4 * q], ocol[wn * 32 + jb * 16 + lr], n)];
#pragma unroll
  for (int kq = 0; kq < PB; kq += 4) {
    double af[2], bf[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) af[ib] = -li[kq + lk][wm * 32 + ib * 16 + lr];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) bf[jb] = lj[kq + lk][wn * 32 + jb * 16 + lr];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
        acc[ib][jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ib], bf[jb], acc[ib][jb], 0, 0, 0);
  }
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = wm * 32 + ib * 16 + lk + 4 * q, cl = wn * 32 + jb * 16 + lr;
        const int gi = i0 + rl, gj = j0 + cl;
        if (gi < nc && gj < nc && (mirror || gi >= gj)) Hn[size_t(gi) * n + gj] = acc[ib][jb][q];
        tt[cl][rl] = acc[ib][jb][q];
      }
  if (I == J || !mirror) return;  // uniform
  __syncthreads();
  // mirror: rows j0 .. j0 + 63 of the block, columns i0 .. i0 + 63, row-contiguous
  for (int e = tid; e < 64 * 64; e += 256) {
    const int rr = e >> 6, cc = e & 63;
    const int gi = j0 + rr, gj = i0 + cc;
    if (gi < nc && gj < nc) Hn[size_t(gi) * n + gj] = tt[rr][cc];
  }
}

// Persistent form of syrk_compact_kernel (the default): two workgroups per
// CU loop over the tiles of the leading (n - ps2)^2 block (its size read on
// the device); the next tile's gathered old values are loaded while this
// tile is multiplied and written (its row / column indices one step earlier
// still), so the memory pipe does not idle through each workgroup's MFMA,
// epilogue and dispatch.  Same arithmetic per entry as syrk_compact_kernel.
// cc: also write H_k of every pair of the next panel's candidates (w.cidx
// entries tagged with this update's ps2) into w.Cc, both triangles, by slot
// (piv_sel_kernel<SEL_STEPS>) -- copies of the values stored to Hn.
__global__ __launch_bounds__(256, 2) void syrk_compact_p_kernel(int n, PivWs w,
                                                                const double *__restrict__ Hc,
                                                                double *__restrict__ Hn,
                                                                int mirror, int cc) {
  __shared__ double li[PB][64], lj[PB][64];
  __shared__ double tt[64][65];
  const int tid = threadIdx.x;
  const int ps2 = w.sstate[0], tn = max(w.sstate[1], 0);
  const int nc = n - ps2;
  if (nc <= 0) return;
  const int ntile = tg::cdiv(nc, 64), tiles = ntile * (ntile + 1) / 2;
  const int lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 15, lk = lane >> 4;
  auto tile_ij = [&](int b, int &i0, int &j0) __attribute__((always_inline)) {
    int I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= b) ++I;
    while (I * (I + 1) / 2 > b) --I;
    i0 = 64 * I;
    j0 = 64 * (b - I * (I + 1) / 2);
  };
  // this thread's gathered rows (ib, q) and columns (jb) of a tile
  auto load_idx = [&](int b, int (&ro)[2][4], int (&co)[2]) __attribute__((always_inline)) {
    int i0, j0;
    tile_ij(b, i0, j0);
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int q = 0; q < 4; ++q) ro[ib][q] = w.oidx[tn + min(i0 + wm * 32 + ib * 16 + lk + 4 * q, nc - 1)];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) co[jb] = w.oidx[tn + min(j0 + wn * 32 + jb * 16 + lr, nc - 1)];
  };
  auto load_old = [&](const int (&ro)[2][4], const int (&co)[2], double (&o)[2][2][4])
      __attribute__((always_inline)) {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 4; ++q) o[ib][jb][q] = Hc[hk_at(ro[ib][q], co[jb], n)];
  };
  int b = blockIdx.x;
  if (b >= tiles) return;
  int ro[2][4], co[2];
  double old[2][2][4], nold[2][2][4];
  load_idx(b, ro, co);
  load_old(ro, co, old);
  const int G = int(gridDim.x);
  if (b + G < tiles) load_idx(b + G, ro, co);
  const int ctag = ps2 << CC_TAG;
  for (; b < tiles; b += G) {
    int i0, j0;
    tile_ij(b, i0, j0);
    // candidate slots of this thread's rows and columns (-1: not a candidate
    // of the next panel); loads in flight through the tile's MFMA
    int crs[2][4], ccs[2];
    if (cc) {
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          crs[ib][q] = w.cidx[min(i0 + wm * 32 + ib * 16 + lk + 4 * q, nc - 1)];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) ccs[jb] = w.cidx[min(j0 + wn * 32 + jb * 16 + lr, nc - 1)];
    }
    __syncthreads();  // the previous tile's reads of li, lj, tt are done
    double lv[8][2];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + u * 256, l = e >> 6, c = e & 63;
      lv[u][0] = w.LT[size_t(l) * n + min(i0 + c, nc - 1)];
      lv[u][1] = w.LT[size_t(l) * n + min(j0 + c, nc - 1)];
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool more = b + G < tiles;
    if (more) load_old(ro, co, nold);  // in flight through this tile
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + u * 256, l = e >> 6, c = e & 63;
      li[l][c] = lv[u][0];
      lj[l][c] = lv[u][1];
    }
    __syncthreads();
    if (b + 2 * G < tiles) load_idx(b + 2 * G, ro, co);
    doublex4 acc[2][2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[ib][jb][q] = old[ib][jb][q];
#pragma unroll
    for (int kq = 0; kq < PB; kq += 4) {
      double af[2], bf[2];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) af[ib] = -li[kq + lk][wm * 32 + ib * 16 + lr];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) bf[jb] = lj[kq + lk][wn * 32 + jb * 16 + lr];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
          acc[ib][jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ib], bf[jb], acc[ib][jb], 0, 0, 0);
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = wm * 32 + ib * 16 + lk + 4 * q, cl = wn * 32 + jb * 16 + lr;
          const int gi = i0 + rl, gj = j0 + cl;
          if (gi < nc && gj < nc && (mirror || gi >= gj)) Hn[size_t(gi) * n + gj] = acc[ib][jb][q];
          tt[cl][rl] = acc[ib][jb][q];
          if (cc && gi < nc && gj < nc && gi >= gj && (crs[ib][q] & ~(SEL_WS * 2 - 1)) == ctag &&
              (ccs[jb] & ~(SEL_WS * 2 - 1)) == ctag) {
            const int a = crs[ib][q] & (SEL_WS * 2 - 1), c2 = ccs[jb] & (SEL_WS * 2 - 1);
            w.Cc[size_t(a) * SEL + c2] = acc[ib][jb][q];
            w.Cc[size_t(c2) * SEL + a] = acc[ib][jb][q];
          }
        }
    if (i0 != j0 && mirror) {  // uniform: mirror rows j0 .. j0 + 63, columns i0 .. i0 + 63
      __syncthreads();
      for (int e = tid; e < 64 * 64; e += 256) {
        const int rr = e >> 6, cc = e & 63;
        const int gi = j0 + rr, gj = i0 + cc;
        if (gi < nc && gj < nc) Hn[size_t(gi) * n + gj] = tt[rr][cc];
      }
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int q = 0; q < 4; ++q) old[ib][jb][q] = nold[ib][jb][q];
  }
}

// dsc = diag(Hk), perm = pos = identity, no pivot chosen yet.
__global__ __launch_bounds__(256) void piv_init2_kernel(int n, PivWs w) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    w.dsc[j] = w.Hk[size_t(j) * n + j];
    w.perm[j] = j;
    w.pos[j] = j;
  }
  if (blockIdx.x == 0 && threadIdx.x < 16) w.sstate[threadIdx.x] = 0;
}

// Rx[t][j] = L[perm[j]][t] for j >= t (upper trapezoidal), perm64 = perm.
__global__ void rx_gather_kernel(int n, int k, PivWs w, double *__restrict__ Rx, int ldr,
                                 int64_t *__restrict__ perm64) {
  const int t = blockIdx.y;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const int r = w.perm[j];
    if (t == 0) perm64[j] = r;
    if (Rx) Rx[size_t(t) * ldr + j] = j >= t ? w.L[size_t(r) * k + t] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// U
// ---------------------------------------------------------------------------
// A[t][j] = (1/S[t]) * Vh[t][perm[j]]     (gptq_utils.py:111, 118-119)
__global__ void gather_scale_kernel(const double *__restrict__ Vh, int ldv, const double *__restrict__ S,
                                    const int64_t *__restrict__ perm, int n, double *__restrict__ A) {
  const int t = blockIdx.y;
  const double sinv = 1.0 / S[t];
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    A[size_t(t) * n + j] = sinv * Vh[size_t(t) * ldv + perm[j]];
}

// Upper Cholesky of the pb x pb diagonal block at U[p][p] (in place), LDS.
// Diagonal block of the U Cholesky (NU x NU, in LDS): U11 = chol_upper(G11)
// written to U, and W = U11^-T (lower) to Wout, so the panel's off-diagonal
// rows become one MFMA GEMM U12 = W G12.  X = U11^-1 by back substitution,
// one column per thread group.
constexpr int NU = 64;
// Diagonal NU x NU block of the U Cholesky: U11 = chol_upper(G11) written to
// U and W = U11^-T (lower) to Wout, so the panel's off-diagonal rows become
// one MFMA GEMM U12 = W G12.  Four waves: lane c = column c, wave
// g holds rows 16g .. 16g + 15 (a[q] = A[16g + q][c]), so each wave issues a
// quarter of the update (a one-wave form, measured and removed, issued ≈17k
// instructions per block: 50 us against 31).  Step j: the owner wave publishes row j (columns < j as 0,
// so the update needs no mask: rows above j take multiplier 0, finished
// columns factor 0), one barrier, every wave updates its rows.  The inverse
// runs right-looking over U's columns: step l (descending) finalises row l of
// X = U^-1 in its owner, publishes it, and every wave subtracts
// U[i][l] X[l][:] from its rows i < l (U's diagonal held apart as 1/U_ll, so
// the stored column has zeros at i >= l).  Broadcast rows double-buffered:
// one barrier per step.
struct PotrfSm {
  double rowb[2][NU];
  double ut[NU][NU + 2];  // ut[l][i] = U[i][l] for i < l (0 elsewhere); then W = U11^-T
  double rinv[NU];
};
// The factor and the inverse of one diagonal block by the four waves of the
// calling workgroup (the steps described above): U11 ends in a[] (row RW g +
// q, column c, upper), W = U11^-T in sm.ut (ut[r][c] = W[r][c], lower), and
// the return value says a pivot of the block's pb rows was not positive.
// INV = false: the factor only (sm.ut then holds U's strict upper part).
// (Two pivots per barrier -- every thread forming the second pivot's row
// from the first's with the owner's fma, bit-identical -- measured no
// faster: the pivots' rsq / Newton chain, not the barriers, sets the pace.)
template <int NWV, bool INV>
__device__ __forceinline__ bool potrf_inv_block(const double *__restrict__ base, int ldu, int pb,
                                                PotrfSm &sm, double (&a)[NU / NWV]) {
  constexpr int RW = NU / NWV;  // rows per wave
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  {
    const int cc = min(c, pb - 1);
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int r = RW * g + q;
      const double v = base[size_t(min(r, pb - 1)) * ldu + cc];  // clamped: no guarded loads
      a[q] = (r < pb && c < pb) ? v : (r == c ? 1.0 : 0.0);
    }
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NU; ++j) {
    const int gj = j / RW, qj = j % RW;
    if (g == gj) sm.rowb[j & 1][c] = c >= j ? a[qj] : 0.0;
    __syncthreads();
    const double d = sm.rowb[j & 1][j];
    const double vc = sm.rowb[j & 1][c];
    double rv[RW];
    const double2 *r2 = reinterpret_cast<const double2 *>(&sm.rowb[j & 1][RW * g]);
#pragma unroll
    for (int q = 0; q < RW / 2; ++q) {
      const double2 t = r2[q];
      rv[2 * q] = t.x;
      rv[2 * q + 1] = t.y;
    }
    // 1/sqrt(d) by v_rsq_f64 + two Newton steps (the IEEE sqrt and division
    // are ~30 dependent instructions on the chain)
    double inv = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    inv = inv * fma(-hd * inv, inv, 1.5);
    inv = inv * fma(-hd * inv, inv, 1.5);
    const double piv = d * inv;
    bad |= !(d > 0.0) && j < pb;
    const double ujc = vc * inv;  // U[j][c] for c > j, 0 for c < j
    const double f = ujc * inv;
#pragma unroll
    for (int q = 0; q < RW; ++q) a[q] = fma(-rv[q], f, a[q]);  // rows <= j: rv = 0 or reset below
    if (g == gj) {
      a[qj] = c > j ? ujc : (c == j ? piv : 0.0);
      sm.ut[c][j] = c > j ? ujc : 0.0;  // column c of U at row j (diagonal apart)
    }
    if (c == j && g == 0) sm.rinv[j] = inv;
  }
  if constexpr (INV) {
    // X = U^-1: s = I, then for l = 63 .. 0: X[l] = s[l] / U_ll (owner), s[i] -= U[i][l] X[l]
    double x[RW];
#pragma unroll
    for (int q = 0; q < RW; ++q) x[q] = (RW * g + q == c) ? 1.0 : 0.0;
    __syncthreads();
#pragma unroll
    for (int l = NU - 1; l >= 0; --l) {
      const int gl = l / RW, ql = l % RW;
      if (g == gl) {
        x[ql] *= sm.rinv[l];
        sm.rowb[l & 1][c] = x[ql];
      }
      __syncthreads();
      const double xl = sm.rowb[l & 1][c];
      double uv[RW];
      const double2 *u2 = reinterpret_cast<const double2 *>(&sm.ut[l][RW * g]);
#pragma unroll
      for (int q = 0; q < RW / 2; ++q) {
        const double2 t = u2[q];
        uv[2 * q] = t.x;
        uv[2 * q + 1] = t.y;
      }
#pragma unroll
      for (int q = 0; q < RW; ++q) x[q] = fma(-uv[q], xl, x[q]);  // U[i][l] = 0 for i >= l
    }
    __syncthreads();  // ut is reused as the W buffer
    // W = X^T (lower): ut[c][r] = X[r][c]
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int r = RW * g + q;
      sm.ut[c][r] = (r < pb && c < pb) ? x[q] : 0.0;
    }
    __syncthreads();
  }
  return bad;
}

template <int NWV>
__global__ __launch_bounds__(64 * NWV) void potrf_inv_4w_kernel(double *__restrict__ U, int ldu,
                                                                int p, int pb,
                                                                double *__restrict__ Wout,
                                                                int *__restrict__ info) {
  constexpr int RW = NU / NWV;
  __shared__ PotrfSm sm;
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  double a[RW];
  double *base = U + size_t(p) * ldu + p;
  const bool bad = potrf_inv_block<NWV, true>(base, ldu, pb, sm, a);
  if (threadIdx.x == 0 && bad) atomicAdd(info, 1);
  // U block (upper) back in place
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int r = RW * g + q;
    if (r < pb && c < pb) base[size_t(r) * ldu + c] = c >= r ? a[q] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int r = RW * g + q;
    Wout[r * NU + c] = sm.ut[r][c];
  }
}

// X = U11^-1 (64 x 64 upper) from potrf_inv_block<.., false>'s factor (U's
// strict upper part in sm.ut[l][i] = U[i][l], 1 / U_ll in sm.rinv) by
// blocks instead of 64 dependent row steps: the eight 8 x 8 diagonal blocks
// by back substitution (one thread per column, all at once), then three
// levels of X12 = -X11 (U12 X22) over blocks of 16, 32, 64 -- 7 barriers.
// xs: X (lower part zero); tmp: U12 X22 of the level.
__device__ __forceinline__ void trinv64_blocked(PotrfSm &sm, double (*xs)[NU + 1],
                                                double (*tmp)[NU + 1]) {
  const int tid = threadIdx.x;
  auto U = [&](int r, int c) { return r < c ? sm.ut[c][r] : 0.0; };  // strict upper
  for (int e = tid; e < NU * NU; e += 256) xs[e >> 6][e & 63] = 0.0;
  __syncthreads();
  if (tid < NU) {
    const int bb = 8 * (tid >> 3), c = tid & 7;
    double x[8];
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      double acc = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int kk = i + 1; kk < 8; ++kk) acc = fma(-U(bb + i, bb + kk), x[kk], acc);
      x[i] = (i <= c) ? acc * sm.rinv[bb + i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) xs[bb + i][bb + c] = x[i];
  }
  __syncthreads();
#pragma unroll
  for (int h = 8; h < NU; h *= 2) {
    const int nb = NU / (2 * h), cnt = nb * h * h;
    for (int t = tid; t < cnt; t += 256) {  // T = U12 X22 (X22 upper: k <= c)
      const int blk = t / (h * h), r = (t / h) % h, c = t % h, o = blk * 2 * h;
      double acc = 0.0;
      for (int kk = 0; kk <= c; ++kk) acc = fma(U(o + r, o + h + kk), xs[o + h + kk][o + h + c], acc);
      tmp[o + r][o + h + c] = acc;
    }
    __syncthreads();
    for (int t = tid; t < cnt; t += 256) {  // X12 = -X11 T (X11 upper: kk >= r)
      const int blk = t / (h * h), r = (t / h) % h, c = t % h, o = blk * 2 * h;
      double acc = 0.0;
      for (int kk = r; kk < h; ++kk) acc = fma(xs[o + r][o + kk], tmp[o + kk][o + h + c], acc);
      xs[o + r][o + h + c] = -acc;
    }
    __syncthreads();
  }
}

// Fused panel step of chol_upper_rows (TG_CHOL_FUSED, the default): workgroup
// t factors the panel's diagonal block itself (every workgroup the same
// operations on the same block, so the same U11 and W in each) and forms its
// 64-column tile of the panel rows, P = W G12[:, tile], on FP64 MFMA, in
// place -- one launch where the potrf kernel, a GEMM launch and the gap
// between them were.  U11 is NOT written here (another workgroup may still
// be reading the block): chol_diag_kernel factors every panel's block again
// at the end (the blocks stay as they were factored: no later step of the
// factorisation writes them) and writes U11 and the pivot count.
__global__ __launch_bounds__(256) void chol_panel_kernel(double *__restrict__ U, int ldu, int p,
                                                         int pb, int c0, int n) {
  constexpr int RW = NU / 4;
  __shared__ PotrfSm sm;
  __shared__ double gs[NU][NU + 1];  // the tile of G12 (row l, column j)
  __shared__ double xs[NU][NU + 1];  // X = U11^-1
  __shared__ double xt[NU][NU + 1];  // the inverse's level products
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6, lr = lane >> 4, lc = lane & 15;
  const int col0 = c0 + NU * int(blockIdx.x);
  // the tile first (its loads in flight through the factorisation)
  double tv[NU * NU / 256];
#pragma unroll
  for (int u = 0; u < NU * NU / 256; ++u) {
    const int e = tid + 256 * u, r = e >> 6, cc = e & 63;
    tv[u] = U[size_t(p + min(r, pb - 1)) * ldu + min(col0 + cc, n - 1)];
  }
  double a[RW];
  (void)potrf_inv_block<4, false>(U + size_t(p) * ldu + p, ldu, pb, sm, a);
  __syncthreads();  // sm.ut / sm.rinv complete
  trinv64_blocked(sm, xs, xt);
#pragma unroll
  for (int u = 0; u < NU * NU / 256; ++u) {
    const int e = tid + 256 * u, r = e >> 6, cc = e & 63;
    gs[r][cc] = (r < pb) ? tv[u] : 0.0;
  }
  __syncthreads();
  // wave g: rows 16 g .. 16 g + 15 of P, four 16-column blocks, K = 64;
  // W = X^T restricted to the block's pb rows and columns
  doublex4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < NU; k0 += 4) {
    const int wi = 16 * g + lc, wk = k0 + lr;
    const double av = (wi < pb && wk < pb) ? xs[wk][wi] : 0.0;  // W[row][k] = X[k][row]
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, gs[k0 + lr][16 * cb + lc], acc[cb], 0, 0, 0);
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * g + lr + 4 * q, cc = col0 + 16 * cb + lc;
      if (r < pb && cc < n) U[size_t(p + r) * ldu + cc] = acc[cb][q];
    }
}

// U11 of every panel of chol_upper_rows' fused form (one workgroup each, the
// panels' blocks as they were factored) and the count of non-positive pivots.
__global__ __launch_bounds__(256) void chol_diag_kernel(double *__restrict__ U, int ldu, int k,
                                                        int *__restrict__ info) {
  constexpr int RW = NU / 4;
  __shared__ PotrfSm sm;
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int p = NU * int(blockIdx.x), pb = min(NU, k - p);
  double a[RW];
  double *base = U + size_t(p) * ldu + p;
  const bool bad = potrf_inv_block<4, false>(base, ldu, pb, sm, a);
  if (threadIdx.x == 0 && bad) atomicAdd(info, 1);
  __syncthreads();  // every wave's reads of the block are done
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int r = RW * g + q;
    if (r < pb && c < pb) base[size_t(r) * ldu + c] = c >= r ? a[q] : 0.0;
  }
}

// Row-panel triangular solve: X = Ubb^{-T} G[p:p+pb, c] for c in [c0, n).
// One thread per column; the column's pb unknowns live in LDS (xs[j][tid]).
__global__ __launch_bounds__(256) void trsm_rows_kernel(double *__restrict__ U, int ldu, int p, int pb,
                                                        int c0, int n) {
  __shared__ double ub[CB][CB + 1];
  __shared__ double xs[CB][256];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < CB * CB; idx += blockDim.x) {
    const int r = idx / CB, c = idx % CB;
    ub[r][c] = (r < pb && c < pb) ? U[size_t(p + r) * ldu + p + c] : (r == c ? 1.0 : 0.0);
  }
  const int c = c0 + blockIdx.x * blockDim.x + tid;
  const bool act = c < n;
  for (int j = 0; j < pb; ++j) xs[j][tid] = act ? U[size_t(p + j) * ldu + c] : 0.0;
  __syncthreads();
  for (int j = 0; j < pb; ++j) {
    double v = xs[j][tid];
    for (int l = 0; l < j; ++l) v -= ub[l][j] * xs[l][tid];
    xs[j][tid] = v / ub[j][j];
  }
  if (act)
    for (int j = 0; j < pb; ++j) U[size_t(p + j) * ldu + c] = xs[j][tid];
}

__global__ void zero_lower_kernel(double *__restrict__ U, int ldu, int k) {
  const int r = blockIdx.y;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < r && c < k; c += gridDim.x * blockDim.x)
    U[size_t(r) * ldu + c] = 0.0;
}


// Right-looking blocked upper Cholesky of the first k rows of the symmetric
// n x n matrix in U (upper triangle read): U[:k, :] <- R with R^T R = G
// restricted to those rows (k = n: the full factor).  NU-row panels: the
// diagonal block and its inverse (potrf_inv_4w_kernel), the panel rows as
// one MFMA GEMM U12 = U11^-T G12, the trailing update as a second GEMM.
// info[0] counts non-positive pivots.
// Diagonal-block factor + inverse: the four-wave kernel.
static void launch_potrf_inv(hipStream_t st, double *U, int ldu, int p, int pb, double *Wb,
                             int *info) {
  hipLaunchKernelGGL(potrf_inv_4w_kernel<4>, dim3(1), dim3(256), 0, st, U, ldu, p, pb, Wb, info);
}

// Two-level blocking: NU-row panels inside strips of CS = 256 rows.  A
// panel's rank-NU update only reaches the rest of its strip; the rows below
// the strip get one rank-CS update per strip (a quarter of the passes over
// the trailing matrix, and at K = 256 the update is MFMA-bound instead of
// HBM-bound: at k = 12,288 the 192 rank-64 updates streamed ~150 GB).  When
// k == n the trailing matrix is symmetric and that update is a SYRK on the
// lower tiles, mirrored (half the flops of the square).  The strip update
// writes the whole trailing square (lower tiles mirrored): later panels read
// only its upper triangle.
constexpr int CS = 256;

hipError_t chol_upper_rows(hipStream_t st, double *U, int ldu, int k, int n, double *Wb,
                           int *info) {
  // (a depth-1 look-ahead on a side stream measured +0.4 ms: the event
  // waits cost more than the overlap; removed)
  // TG_CHOL_FUSED=0: the potrf kernel and a GEMM launch per panel (the
  // panel's U11 written at once) instead of chol_panel_kernel + chol_diag_kernel
  const char *cf = getenv("TG_CHOL_FUSED");  // development switch, read per call
  const bool fused = !(cf && cf[0] == '0');
  for (int s0 = 0; s0 < k; s0 += CS) {
    const int se = std::min(k, s0 + CS);
    for (int p = s0; p < se; p += NU) {
      const int pb = std::min(NU, se - p);
      const int c0 = p + pb;
      hipError_t e = hipSuccess;
      if (fused) {
        if (c0 < n)
          hipLaunchKernelGGL(chol_panel_kernel, dim3(tg::cdiv(n - c0, NU)), dim3(256), 0, st, U, ldu,
                             p, pb, c0, n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
      } else {
        launch_potrf_inv(st, U, ldu, p, pb, Wb, info);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (c0 < n) {
          // in place: one 64-row tile covers the panel's rows, so each workgroup
          // reads its columns of G12 fully before writing them
          double *P = U + size_t(p) * ldu + c0;
          e = tg::dgemm(st, false, false, pb, n - c0, pb, 1.0, Wb, NU, P, ldu, 0.0, P, ldu);
          if (e != hipSuccess) return e;
        }
      }
      if (c0 < se) {  // the rest of the strip
        const double *P = U + size_t(p) * ldu + c0;
        e = tg::dgemm(st, true, false, se - c0, n - c0, pb, -1.0, P, ldu, P, ldu, 1.0,
                      U + size_t(c0) * ldu + c0, ldu);
        if (e != hipSuccess) return e;
      }
    }
    if (se < k) {  // rows below the strip: one rank-(se - s0) update
      const double *Q = U + size_t(s0) * ldu + se;
      const hipError_t e =
          k == n ? tg::dsyrk_tn(st, n - se, se - s0, -1.0, Q, ldu, 1.0, U + size_t(se) * ldu + se,
                                ldu)
                 : tg::dgemm(st, true, false, k - se, n - se, se - s0, -1.0, Q, ldu, Q, ldu, 1.0,
                             U + size_t(se) * ldu + se, ldu);
      if (e != hipSuccess) return e;
    }
  }
  if (fused && k > 0) {
    hipLaunchKernelGGL(chol_diag_kernel, dim3(tg::cdiv(k, NU)), dim3(256), 0, st, U, ldu, k, info);
    return hipGetLastError();
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// GPTQ comparator factor (process_hessian, gptq_utils.py:129-165):
// R = chol_upper(inv(H_p + damp I)), H_p = H[perm][:, perm].  With J the
// reversal, chol_upper(J H_p J) = U' gives H_p = Ut Ut^T for the upper
// Ut = J U'^T J, hence inv(H_p) = Ut^-T Ut^-1 and R = Ut^-1 = J (U'^-1)^T J:
// one Cholesky and one triangular inverse instead of the reference's
// cholesky -> cholesky_inverse -> cholesky (same matrix, other rounding).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void diag_mean_kernel(const double *__restrict__ H, int64_t ldh,
                                                        int n, double *__restrict__ mean) {
  __shared__ double part[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += H[i * ldh + i];
  part[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += part[i];  // fixed order: deterministic
    t /= double(n);
    mean[0] = (t == 0.0) ? 1.0 : t;              // :144-145
  }
}

// A[i][j] = H[p(n-1-i)][p(n-1-j)] + (i == j) damp * mean
__global__ void flip_damp_kernel(const double *__restrict__ H, int64_t ldh, int n,
                                 const int64_t *__restrict__ perm, double damp,
                                 const double *__restrict__ mean, double *__restrict__ A) {
  // Entry (i, j) of A = J H_p J is H_p[n-1-i][n-1-j]; it is always read from
  // H_p's LOWER triangle (row n-1-min(i,j) >= column n-1-max(i,j)), the only
  // triangle the reference's torch.linalg.cholesky(H_damped) reads
  // (gptq_utils.py:152), so an H that is not bit-symmetric factors the same
  // way.  A itself is then exactly symmetric, whichever triangle
  // chol_upper_rows' panels and strip SYRKs read.
  const int i = blockIdx.y;
  const double dm = damp * mean[0];
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const int r = n - 1 - min(i, j), c = n - 1 - max(i, j);
    const int64_t pr = perm ? perm[r] : r, pc = perm ? perm[c] : c;
    double v = H[pr * ldh + pc];
    if (i == j) v += dm;
    A[int64_t(i) * n + j] = v;
  }
}

// Y_bb = U_bb^-1 for every NU x NU diagonal block b (one workgroup each);
// the rest of Y is left to the caller (zeroed, then filled by GEMMs).
__global__ __launch_bounds__(256) void trinv_diag_kernel(const double *__restrict__ U, int ldu,
                                                         int n, double *__restrict__ Y, int ldy) {
  __shared__ double a[NU][NU + 1];
  __shared__ double x[NU][NU + 1];
  const int p = blockIdx.x * NU, pb = min(NU, n - p), tid = threadIdx.x;
  for (int idx = tid; idx < NU * NU; idx += blockDim.x) {
    const int r = idx / NU, c = idx % NU;
    a[r][c] = (r < pb && c < pb) ? (c >= r ? U[size_t(p + r) * ldu + p + c] : 0.0)
                                 : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  const int c = tid >> 2, part = tid & 3;
  for (int i = NU - 1; i >= 0; --i) {
    double sacc = 0.0;
    if (i < c)
      for (int l = i + 1 + part; l <= c; l += 4) sacc += a[i][l] * x[l][c];
    sacc += __shfl_xor(sacc, 1);
    sacc += __shfl_xor(sacc, 2);
    if (part == 0) x[i][c] = i > c ? 0.0 : ((i == c ? 1.0 : 0.0) - sacc) / a[i][i];
    __syncthreads();
  }
  for (int idx = tid; idx < pb * pb; idx += blockDim.x) {
    const int r = idx / pb, cc = idx % pb;
    Y[size_t(p + r) * ldy + p + cc] = x[r][cc];
  }
}

// Off-diagonal blocks of Y = U^-1 (upper; the NU x NU diagonal blocks are
// already in Y, everything below the diagonal is zero).  Bottom-up: at block
// size b = NU, 2NU, ... each pair of adjacent solved blocks merges with
// Y12 = -(Y11 U12) Y22.  All full-size pairs of a level are independent and
// go out as two batched GEMMs, which skip the zero triangles of Y11 and Y22
// (half their flops); a pair whose second block is the ragged tail gets two
// plain GEMMs.  T holds >= n*n/4 doubles.
// bmax: stop before merging blocks of bmax rows (the diagonal bmax x bmax
// blocks of Y are then the inverses of U's, the rest untouched).
hipError_t trinv_offdiag(hipStream_t st, const double *U, int ldu, double *Y, int ldy, int n,
                         double *T, int bmax = 1 << 30) {
  for (int b = NU; b < n && b < bmax; b *= 2) {
    const int nblk = tg::cdiv(n, b), npair = nblk / 2;
    const bool ragged = npair > 0 && 2 * npair * b > n;
    const int nfull = ragged ? npair - 1 : npair;
    hipError_t e = hipSuccess;
    if (nfull > 0) {
      const int64_t bb = int64_t(b) * b, dy = int64_t(ldy) + 1, du = int64_t(ldu) + 1;
      const tg::ChunkSpec c1{2 * b, nfull, 2 * b * nfull, dy, 0, du, 0, 0, bb, b, b, b};
      e = tg::dgemm_chunked(st, false, false, c1, 1.0, Y, ldy, U + b, ldu, 0.0, T, b, 1);
      if (e != hipSuccess) return e;
      const tg::ChunkSpec c2{2 * b, nfull, 2 * b * nfull, 0, bb, dy, 0, dy, 0, b, b, b};
      e = tg::dgemm_chunked(st, false, false, c2, -1.0, T, b, Y + size_t(b) * ldy + b, ldy, 0.0,
                            Y + b, ldy, 2);
      if (e != hipSuccess) return e;
    }
    if (ragged) {
      const size_t s = size_t(2) * (npair - 1) * b;
      const int b2 = n - int(s) - b;
      e = tg::dgemm(st, false, false, b, b2, b, 1.0, Y + s * ldy + s, ldy, U + s * ldu + s + b,
                    ldu, 0.0, T, b2);
      if (e != hipSuccess) return e;
      e = tg::dgemm(st, false, false, b, b2, b2, -1.0, T, b2, Y + (s + b) * ldy + s + b, ldy, 0.0,
                    Y + s * ldy + s + b, ldy);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// R[i][j] = Y[n-1-j][n-1-i] (j >= i), 0 below the diagonal
__global__ void flip_transpose_kernel(const double *__restrict__ Y, int n, double *__restrict__ R,
                                      int64_t ldr) {
  const int i = blockIdx.y;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    R[i * ldr + j] = j >= i ? Y[int64_t(n - 1 - j) * n + (n - 1 - i)] : 0.0;
}

__global__ void identity_kernel(int n, double *__restrict__ R, int64_t ldr) {
  const int i = blockIdx.y;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    R[i * ldr + j] = i == j ? 1.0 : 0.0;
}

// ---------------------------------------------------------------------------
// Conditioning guard of the Gram-matrix (CholeskyQR) factors of U.
// tg_u_factor and tg_u_factor_rx take R from the Cholesky factor of a Gram
// matrix Y^T Y, which squares Y's condition number (the reference runs a
// Householder QR, gptq_utils.py:120).  After the first Cholesky the host reads
// the factor's info count and diagonal range; when a pivot broke down, or
// (max/min diag)^2 * eps puts the factor's error above ~1e-9, the factor is
// refined by CholeskyQR passes on the explicit Q = Y R^-1 (CholeskyQR2), with
// a shifted first factorisation when the plain one broke down (shifted
// CholeskyQR3: G + s I, s = 11 (k^2 + k (k+1)) u ||Y||_F^2).
// ---------------------------------------------------------------------------
// out[0] = max |d_i|, out[1] = min d_i (0 when any is non-positive or not
// finite), diagonal of the k x k upper factor U
__global__ __launch_bounds__(256) void diag_range_kernel(const double *__restrict__ U, int64_t ldu,
                                                         int k, double *__restrict__ out) {
  __shared__ double mx[256], mn[256];
  double a = 0.0, b = DBL_MAX;
  for (int i = threadIdx.x; i < k; i += 256) {
    const double d = U[i * ldu + i];
    const bool ok = d > 0.0 && d <= DBL_MAX;
    a = ok ? fmax(a, d) : a;
    b = ok ? fmin(b, d) : 0.0;
  }
  mx[threadIdx.x] = a;
  mn[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      mx[threadIdx.x] = fmax(mx[threadIdx.x], mx[threadIdx.x + s]);
      mn[threadIdx.x] = fmin(mn[threadIdx.x], mn[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = mx[0];
    out[1] = mn[0];
  }
}

// out[0] = trace of the k x k matrix G (fixed summation order)
__global__ __launch_bounds__(256) void diag_sum_kernel(const double *__restrict__ G, int64_t ldg,
                                                       int k, double *__restrict__ out) {
  __shared__ double part[256];
  double acc = 0.0;
  for (int i = threadIdx.x; i < k; i += 256) acc += G[i * ldg + i];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0];
}

__global__ void add_diag_kernel(double *__restrict__ G, int64_t ldg, int k, double s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k) G[i * ldg + i] += s;
}

struct CholStat {
  double dmax, dmin, trace;
  int info;
};

// stats[0..2] = {max diag, min diag, trace}, info -> host (one sync)
static hipError_t read_stat(hipStream_t st, const double *stats, const int *info, CholStat &h) {
  double v[3];
  hipError_t e = hipMemcpyAsync(v, stats, sizeof(v), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(&h.info, info, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  h.dmax = v[0];
  h.dmin = v[1];
  h.trace = v[2];
  return e;
}

// 0: never refine, 1: always refine, 2 (default): refine when the guard asks
static int refine_mode() {
  const char *e = getenv("TG_U_REFINE");
  return (e && e[0] == '0') ? 0 : (e && e[0] == '1') ? 1 : 2;
}

// the first factor is not trusted: breakdown (always handled), or
// (dmax/dmin)^2 eps > 1e-9 (TG_U_REFINE=0 / 1 disable / force this part)
static bool needs_refine(const CholStat &h) {
  if (h.info > 0 || !(h.dmin > 0.0)) return true;
  const int mode = refine_mode();
  if (mode != 2) return mode == 1;
  const double r = h.dmax / h.dmin;
  return r * r * DBL_EPSILON > 1e-9;
}

// Y = R^-1 (k x k upper, ld k); T: trinv_offdiag scratch
static hipError_t trinv(hipStream_t st, const double *R, int ldr, int k, double *Y, double *T) {
  hipError_t e = hipMemsetAsync(Y, 0, sizeof(double) * size_t(k) * k, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(trinv_diag_kernel, dim3(tg::cdiv(k, NU)), dim3(256), 0, st, R, ldr, k, Y, k);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return trinv_offdiag(st, R, ldr, Y, k, k, T);
}

static hipError_t zero_lower(hipStream_t st, double *U, int ldu, int k) {
  hipLaunchKernelGGL(zero_lower_kernel, dim3(tg::cdiv(k, 256) < 16 ? tg::cdiv(k, 256) : 16, k),
                     dim3(256), 0, st, U, ldu, k);
  return hipGetLastError();
}

// Scratch of the refinement: Ri, Q, G (k x k each), T (trinv), stats.
struct RefineWs {
  double *Ri, *Q, *G, *T, *stats;
};

// Shifted first factor: R (k x k, ld k) = chol(Y^T Y + s I), s from trace(Y^T Y).
static int shifted_factor(hipStream_t st, const double *Y, int64_t ldy, int k, double *R,
                          RefineWs &w, double *Wb, int *info, CholStat &h) {
  TG_HIP(tg::dsyrk_tn(st, k, k, 1.0, Y, ldy, 0.0, R, k));
  hipLaunchKernelGGL(diag_sum_kernel, dim3(1), dim3(256), 0, st, R, int64_t(k), k, w.stats + 2);
  TG_LAUNCHED();
  TG_HIP(read_stat(st, w.stats, info, h));
  const double kk = double(k);
  const double s = 11.0 * (kk * kk + kk * (kk + 1.0)) * (DBL_EPSILON / 2) * h.trace;
  hipLaunchKernelGGL(add_diag_kernel, dim3(tg::cdiv(k, 256)), dim3(256), 0, st, R, int64_t(k), k, s);
  TG_LAUNCHED();
  TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
  TG_HIP(chol_upper_rows(st, R, k, k, k, Wb, info));
  TG_HIP(zero_lower(st, R, k, k));
  hipLaunchKernelGGL(diag_range_kernel, dim3(1), dim3(256), 0, st, R, int64_t(k), k, w.stats);
  TG_LAUNCHED();
  TG_HIP(read_stat(st, w.stats, info, h));
  if (h.info > 0 || !(h.dmin > 0.0)) {
    tg::set_error("U factor: shifted Cholesky of the Gram matrix broke down (%d pivots; "
                  "input not of full rank k = %d)", h.info, k);
    return int(hipErrorUnknown);
  }
  return 0;
}

// One CholeskyQR pass: Q = Y R^-1, Q^T Q = R'^T R', R <- R' R.
static int cholqr_pass(hipStream_t st, const double *Y, int64_t ldy, int k, double *R,
                       RefineWs &w, double *Wb, int *info) {
  TG_HIP(trinv(st, R, k, k, w.Ri, w.T));
  TG_HIP(tg::dgemm(st, false, false, k, k, k, 1.0, Y, ldy, w.Ri, k, 0.0, w.Q, k));
  TG_HIP(tg::dsyrk_tn(st, k, k, 1.0, w.Q, k, 0.0, w.G, k));
  TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
  TG_HIP(chol_upper_rows(st, w.G, k, k, k, Wb, info));
  TG_HIP(zero_lower(st, w.G, k, k));
  TG_HIP(tg::dgemm(st, false, false, k, k, k, 1.0, w.G, k, R, k, 0.0, w.Ri, k));  // R' R
  TG_HIP(hipMemcpyAsync(R, w.Ri, sizeof(double) * size_t(k) * k, hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(diag_range_kernel, dim3(1), dim3(256), 0, st, R, int64_t(k), k, w.stats);
  TG_LAUNCHED();
  CholStat h{};
  TG_HIP(read_stat(st, w.stats, info, h));
  if (h.info > 0 || !(h.dmin > 0.0)) {
    tg::set_error("U factor: CholeskyQR refinement broke down (%d pivots, k = %d)", h.info, k);
    return int(hipErrorUnknown);
  }
  return 0;
}

// Refined R (k x k, ld k) of Y (k x k, ld ldy), given the first factor in R
// and its statistics h: shifted restart on breakdown, then 1 (2 after a
// shift) CholeskyQR passes.
static int refine_factor(hipStream_t st, const double *Y, int64_t ldy, int k, double *R,
                         RefineWs &w, double *Wb, int *info, CholStat h) {
  int passes = 1;
  if (h.info > 0 || !(h.dmin > 0.0)) {
    const int e = shifted_factor(st, Y, ldy, k, R, w, Wb, info, h);
    if (e != 0) return e;
    passes = 2;
  }
  for (int p = 0; p < passes; ++p) {
    const int e = cholqr_pass(st, Y, ldy, k, R, w, Wb, info);
    if (e != 0) return e;
  }
  return 0;
}

}  // namespace

extern "C" size_t tg_pivot_workspace_size(int n, int k) {
  tg::Sizer s;
  piv_layout(s, n, k, nullptr);
  return s.off + 256;
}

// Greedy diagonal pivoting on w.Hk (filled by the caller) -> perm, R_x.
// Candidate-set pivot order (piv_sel_kernel + piv_fill_kernel per panel).
// Panels end early when the candidate bound fails, so the host launches the
// panels full panels would need, reads the step count once, and continues
// while steps remain.  The Schur update of a round's last panel is issued
// only once more steps are known to follow.
static int pivot_core_sel(hipStream_t st, PivWs &w, int n, int k) {
#ifdef TG_SEL_PHASES
  static bool reg = false;
  if (!reg) {
    reg = true;
    atexit([] {
      unsigned long long h[16];
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_selph), sizeof(h));
      const char *nm[12] = {"sel:argmax+cand", "head", "barrier2", "compute+wargmax", "blockargmax",
                            "?", "tail", "?", "sel:stage", "sel:count", "sel:radix", "sel:compact"};
      fprintf(stderr, "sel phases (cycles, thread 0):");
      for (int q = 0; q < 12; ++q) fprintf(stderr, " %s %.3g", nm[q], double(h[q]));
      fprintf(stderr, " steps %llu", h[15]);
      fprintf(stderr, "\n");
    });
  }
#endif
  hipLaunchKernelGGL(piv_init2_kernel, dim3(std::min(64, tg::cdiv(n, 256))), dim3(256), 0, st, n, w);
  TG_LAUNCHED();
  const size_t lds = sizeof(int) * size_t((n + 1) & ~1) +
                     (n <= SEL_LDS_N ? (sizeof(double) + sizeof(int)) * size_t(n) : 0);
  if (lds > 48 * 1024) {
    TG_HIP(hipFuncSetAttribute((const void *)piv_sel_kernel<SEL_FULL>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    TG_HIP(hipFuncSetAttribute((const void *)piv_sel_kernel<SEL_SELECT>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    TG_HIP(hipFuncSetAttribute((const void *)piv_sel_kernel<SEL_STEPS>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  }
  // TG_SYR2K_PERSIST=0: one tile per workgroup (development switch, per call)
  const char *ps = getenv("TG_SYR2K_PERSIST");
  const bool persist = !(ps && ps[0] == '0');
  // TG_SCHUR_MIRROR=1: the Schur updates also write the upper triangle
  // (development switch; the readers take (max, min) either way)
  const char *sm = getenv("TG_SCHUR_MIRROR");
  const int mirror = (sm && sm[0] == '1') ? 1 : 0;
  const tg::XcdInfo xi = tg::xcd_info();
  const int ncu = std::max(1, xi.xcds * xi.cus_per_xcd);
  // compacted Schur complements alternate between the two buffers
  const double *hc = w.Hk;
  double *hn = w.Hk2;
  // TG_PIV_CC=1: the steps gather pivot rows from the candidate block instead
  // of H_k (development switch, per call; the block needs the persistent
  // Schur update).  Measured at n = 4096: the pivot class 9.0 -> 8.9 ms but
  // the phase 10.6 -> 11.0 ms (the extra selection launch and the block's
  // writes in every update), so it is off by default
  const char *pc = getenv("TG_PIV_CC");
  const bool ccb = persist && pc && pc[0] == '1';
  auto schur_compact = [&](int rows, int cc = 0) -> hipError_t {
    const int nt = tg::cdiv(rows, 64);
    if (persist)
      hipLaunchKernelGGL(syrk_compact_p_kernel, dim3(std::min(nt * (nt + 1) / 2, 2 * ncu)),
                         dim3(256), 0, st, n, w, hc, hn, mirror, cc);
    else
      hipLaunchKernelGGL(syrk_compact_kernel, dim3(nt * (nt + 1) / 2), dim3(256), 0, st, n, w, hc,
                         hn, mirror);
    const hipError_t e = hipGetLastError();
    double *t = const_cast<double *>(hc);
    hc = hn;
    hn = t;
    return e;
  };
  if (ccb) TG_HIP(hipMemsetAsync(w.cidx, 0xff, sizeof(int32_t) * size_t(n), st));  // no tags
  int done = 0;
  // a panel's Schur update runs at the head of the next panel: with the
  // candidate block, between that panel's selection and its steps
  int pend_rows = 0;  // rows of the pending update (0: none)
  for (int round = 0;; ++round) {
    if (round > 4 * (k / PB + 2)) {
      tg::set_error("pivot order: no progress after %d rounds (%d of %d steps)", round, done, k);
      return int(hipErrorUnknown);
    }
    const int P = tg::cdiv(k - done, PB);
    // every panel starts at or after `done + p` steps: grids sized for that bound
    for (int p = 0; p < P; ++p) {
      const int rows = n - (done + p);
      if (ccb && pend_rows > 0) {
        auto tk = tg::prof_begin(st, tg::PROF_PIVSTEP, 8.0 * double(n) * 2, 0.0);
        hipLaunchKernelGGL(piv_sel_kernel<SEL_SELECT>, dim3(1), dim3(STH), lds, st, n, k, w, hc);
        tg::prof_end(st, tk);
        TG_LAUNCHED();
        TG_HIP(schur_compact(pend_rows, 1));
      } else if (pend_rows > 0) {
        TG_HIP(schur_compact(pend_rows));
      }
      auto tok = tg::prof_begin(st, tg::PROF_PIVSTEP, 8.0 * double(n) * PB * 3, 0.0);
      if (ccb && pend_rows > 0)
        hipLaunchKernelGGL(piv_sel_kernel<SEL_STEPS>, dim3(1), dim3(STH), lds, st, n, k, w, hc);
      else
        hipLaunchKernelGGL(piv_sel_kernel<SEL_FULL>, dim3(1), dim3(STH), lds, st, n, k, w, hc);
      // one wave per workgroup: the gathers of the pivots' columns spread
      // over 4x the CUs of 256-thread groups (n = 12,288: -1.4 ms per solve)
      hipLaunchKernelGGL(piv_fill_kernel<64>, dim3(tg::cdiv(rows, 64)), dim3(64), 0, st, n, k, w, hc);
      tg::prof_end(st, tok);
      TG_LAUNCHED();
      pend_rows = rows;
    }
    int32_t h = 0;
    TG_HIP(hipMemcpyAsync(&h, w.sstate, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    TG_HIP(hipStreamSynchronize(st));
    if (h >= k) break;
    pend_rows = n - (done + P - 1);  // the round's last panel, updated at the next one's head
    done = h;
  }
  return 0;
}

static int pivot_core(hipStream_t st, PivWs &w, int n, int k, int64_t *perm, double *Rx, int ldr) {
  if (compact_pivot(n)) {
    const int e = pivot_core_sel(st, w, n, k);
    if (e != 0) return e;
    hipLaunchKernelGGL(rx_gather_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, k),
                       dim3(256), 0, st, n, k, w, Rx, ldr, perm);
    TG_LAUNCHED();
    return 0;
  }
  const int g0 = std::min(PGMAX, tg::cdiv(n, 256));
  hipLaunchKernelGGL(piv_init_kernel, dim3(g0), dim3(256), 0, st, n, w);
  TG_LAUNCHED();
  const int G = std::max(1, std::min(PGMAX, tg::cdiv(n, 256)));
  const int rpt = tg::cdiv(n, G * 256);
  const bool persistent = rpt <= 2 && n <= 32768 && getenv("TG_PIVOT_STEPWISE") == nullptr;
#ifdef TG_PIV_PHASES
  static bool reg = false;
  if (!reg) {
    reg = true;
    atexit([] {
      unsigned long long h[8];
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pivph), sizeof(h));
      double tot = 0;
      for (int q = 0; q < 7; ++q) tot += h[q];
      fprintf(stderr, "pivot phases (share of step time, workgroup 0):");
      const char *nm[7] = {"local", "wgargmax", "publish", "poll", "slotcopy", "argmax+lrow",
                           "swap"};
      for (int q = 0; q < 7; ++q) fprintf(stderr, " %s %.2f", nm[q], h[q] / tot);
      fprintf(stderr, "\n");
    });
  }
#endif
  if (persistent && n * sizeof(int) > 64 * 1024) {
    TG_HIP(hipFuncSetAttribute((const void *)piv_panel_kernel<1>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(n * sizeof(int))));
    TG_HIP(hipFuncSetAttribute((const void *)piv_panel_kernel<2>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(n * sizeof(int))));
  }
  TG_HIP(hipMemsetAsync(w.flag, 0, 16 * sizeof(unsigned), st));
  // the arrival counter of the panel kernels starts at 0 after piv_init
  for (int ps = 0; ps < k; ps += PB) {
    const int pe = std::min(ps + PB, k);
    if (persistent) {
      // per-panel: n rows x (PB/2 + 3) doubles of H row, L panel and diagonal
      auto tok = tg::prof_begin(st, tg::PROF_PIVSTEP, 8.0 * double(n) * (pe - ps) * 3, 0.0);
      const size_t lds = sizeof(int) * size_t(n);
      TG_HIP(hipMemsetAsync(w.flag + 4, 0, 9 * sizeof(unsigned), st));
      const int grid = 8 * G;  // >= 8 (G - 1) + 1: some XCD always collects G tickets
      if (rpt == 1)
        hipLaunchKernelGGL(piv_panel_kernel<1>, dim3(grid), dim3(256), lds, st, n, k, ps, pe, G,
                           unsigned(G) * unsigned(ps), w);
      else
        hipLaunchKernelGGL(piv_panel_kernel<2>, dim3(grid), dim3(256), lds, st, n, k, ps, pe, G,
                           unsigned(G) * unsigned(ps), w);
      tg::prof_end(st, tok);
      TG_LAUNCHED();
    } else {
      for (int i = ps; i < pe; ++i) {
        auto tok = tg::prof_begin(st, tg::PROF_PIVSTEP, 8.0 * double(n - i) * (i - ps + 3), 0.0);
        hipLaunchKernelGGL(piv_step_kernel, dim3(G), dim3(256), 0, st, n, k, i, ps, w);
        tg::prof_end(st, tok);
        TG_LAUNCHED();
      }
    }
    if (pe < k)  // Schur update with this panel's columns (all rows, original order)
      TG_HIP(tg::dsyrk_tn(st, n, pe - ps, -1.0, w.LT, n, 1.0, w.Hk, n));
  }
  hipLaunchKernelGGL(rx_gather_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, k),
                     dim3(256), 0, st, n, k, w, Rx, ldr, perm);
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_pivoted_factor(void *stream, const double *Vh, int ldv, const double *S, int n,
                                 int k, int64_t *perm, double *Rx, int ldr, void *ws,
                                 size_t ws_bytes) {
  TG_ARG(Vh, 2, "null Vh");
  TG_ARG(ldv >= n, 3, "ldv < n");
  TG_ARG(S, 4, "null S");
  TG_ARG(n >= 1, 5, "n < 1");
  TG_ARG(k >= 1 && k <= n, 6, "k must be in [1, n]");
  TG_ARG(perm, 7, "null perm");
  TG_ARG(!Rx || ldr >= n, 9, "ldr < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  PivWs w{};
  piv_layout(ar, n, k, &w);
  TG_WS(ar);
  TG_HIP(hipMemsetAsync(w.cnt, 0, 16 * sizeof(unsigned), st));
  TG_HIP(hipMemsetAsync(w.LT, 0, sizeof(double) * PB * size_t(n), st));
  hipLaunchKernelGGL(scale_rows_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, k),
                     dim3(256), 0, st, Vh, ldv, S, n, k, w.B);
  TG_LAUNCHED();
  TG_HIP(tg::dsyrk_tn(st, n, k, 1.0, w.B, n, 0.0, w.Hk, n));  // H_k = H_sqrt^T H_sqrt
  return pivot_core(st, w, n, k, perm, Rx, ldr);
}

// Complement form: H_k = H - B_c^T B_c with B_c = diag(S_c) Vc, the nc
// dropped eigenpairs that are not at rounding level (k < j < k + nc in
// descending order).  Equal to V_k L_k V_k^T up to the dropped eigenvalues
// below the rounding threshold; nc may be 0.
extern "C" int tg_pivoted_factor_complement(void *stream, const double *H, int ldh,
                                            const double *Vc, int ldvc, const double *Sc, int nc,
                                            int n, int k, int64_t *perm, double *Rx, int ldr,
                                            void *ws, size_t ws_bytes) {
  TG_ARG(H, 2, "null H");
  TG_ARG(ldh >= n, 3, "ldh < n");
  TG_ARG(nc == 0 || Vc, 4, "null Vc");
  TG_ARG(nc == 0 || ldvc >= n, 5, "ldvc < n");
  TG_ARG(nc == 0 || Sc, 6, "null Sc");
  TG_ARG(nc >= 0 && nc <= k && k + nc <= n, 7, "nc must be in [0, min(k, n - k)]");
  TG_ARG(n >= 1, 8, "n < 1");
  TG_ARG(k >= 1 && k <= n, 9, "k must be in [1, n]");
  TG_ARG(perm, 10, "null perm");
  TG_ARG(!Rx || ldr >= n, 12, "ldr < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  PivWs w{};
  piv_layout(ar, n, k, &w);
  TG_WS(ar);
  TG_HIP(hipMemsetAsync(w.cnt, 0, 16 * sizeof(unsigned), st));
  TG_HIP(hipMemsetAsync(w.LT, 0, sizeof(double) * PB * size_t(n), st));
  TG_HIP(hipMemcpy2DAsync(w.Hk, sizeof(double) * n, H, sizeof(double) * ldh, sizeof(double) * n,
                          n, hipMemcpyDeviceToDevice, st));
  if (nc > 0) {
    hipLaunchKernelGGL(scale_rows_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, nc),
                       dim3(256), 0, st, Vc, ldvc, Sc, n, nc, w.B);
    TG_LAUNCHED();
    TG_HIP(tg::dsyrk_tn(st, n, nc, -1.0, w.B, n, 1.0, w.Hk, n));
  }
  return pivot_core(st, w, n, k, perm, Rx, ldr);
}

template <class Ar>
static void refine_layout(Ar &ar, int k, RefineWs *w) {
  RefineWs d{};
  RefineWs &q = w ? *w : d;
  const size_t h = size_t(NU) * ((tg::cdiv(k, NU) + 1) / 2);
  auto t = [&](double *&dst, size_t cnt) {
    if constexpr (std::is_same_v<Ar, tg::Arena>) dst = ar.template take<double>(cnt);
    else ar.template take<double>(cnt);
  };
  t(q.Ri, size_t(k) * k);
  t(q.Q, size_t(k) * k);
  t(q.G, size_t(k) * k);
  t(q.T, h * h);
  t(q.stats, 8);
}

template <class Ar>
static void ufac_layout(Ar &ar, int n, int k, double **A, int **info, double **Wb, double **Rk,
                        RefineWs *w) {
  auto t = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<Ar, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  double *d[3];
  int *i0;
  t(A ? *A : d[0], size_t(k) * n);
  t(info ? *info : i0, 16);
  t(Wb ? *Wb : d[1], NU * NU);
  t(Rk ? *Rk : d[2], size_t(k) * k);
  refine_layout(ar, k, w);
}

extern "C" size_t tg_ufactor_workspace_size(int n, int k) {
  tg::Sizer s;
  ufac_layout(s, n, k, nullptr, nullptr, nullptr, nullptr, nullptr);
  return s.off + 256;
}

extern "C" int tg_u_factor(void *stream, const double *Vh, int ldv, const double *S,
                           const int64_t *perm, int n, int k, double *U, int ldu, void *ws,
                           size_t ws_bytes) {
  TG_ARG(Vh, 2, "null Vh");
  TG_ARG(ldv >= n, 3, "ldv < n");
  TG_ARG(S, 4, "null S");
  TG_ARG(perm, 5, "null perm");
  TG_ARG(n >= 1, 6, "n < 1");
  TG_ARG(k >= 1 && k <= n, 7, "k must be in [1, n]");
  TG_ARG(U, 8, "null U");
  TG_ARG(ldu >= n, 9, "ldu < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  double *A, *Wb, *Rk;
  int *info;
  RefineWs rw{};
  ufac_layout(ar, n, k, &A, &info, &Wb, &Rk, &rw);
  TG_WS(ar);
  TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
  hipLaunchKernelGGL(gather_scale_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, k),
                     dim3(256), 0, st, Vh, ldv, S, perm, n, A);
  TG_LAUNCHED();
  // G[:k, :] = A[:, :k]^T A   (k x n) into U
  TG_HIP(tg::dgemm(st, true, false, k, n, k, 1.0, A, n, A, n, 0.0, U, ldu));
  TG_HIP(chol_upper_rows(st, U, ldu, k, n, Wb, info));
  TG_HIP(zero_lower(st, U, ldu, k));
  hipLaunchKernelGGL(diag_range_kernel, dim3(1), dim3(256), 0, st, U, int64_t(ldu), k, rw.stats);
  TG_LAUNCHED();
  CholStat h{};
  TG_HIP(read_stat(st, rw.stats, info, h));
  if (!needs_refine(h)) return 0;
  // Refined: R11 by CholeskyQR passes on A1 = A[:, :k], then R12 = Q^T A2
  // with the explicit Q = A1 R11^-1 (not R11^-T G12, whose error grows with
  // cond(A1)^2).
  if (h.info == 0 && h.dmin > 0.0)
    TG_HIP(hipMemcpy2DAsync(Rk, sizeof(double) * k, U, sizeof(double) * ldu, sizeof(double) * k,
                            k, hipMemcpyDeviceToDevice, st));
  const int e = refine_factor(st, A, n, k, Rk, rw, Wb, info, h);
  if (e != 0) return e;
  TG_HIP(trinv(st, Rk, k, k, rw.Ri, rw.T));
  TG_HIP(tg::dgemm(st, false, false, k, k, k, 1.0, A, n, rw.Ri, k, 0.0, rw.Q, k));
  TG_HIP(hipMemcpy2DAsync(U, sizeof(double) * ldu, Rk, sizeof(double) * k, sizeof(double) * k, k,
                          hipMemcpyDeviceToDevice, st));
  if (n > k) TG_HIP(tg::dgemm(st, true, false, k, n - k, k, 1.0, rw.Q, k, A + k, n, 0.0, U + k, ldu));
  return 0;
}

// U from R_x alone (complement path, no kept eigenvectors):
// P^T H_k P = L L^T with L = R_x^T (n x k, full column rank), so
// P^T H_k^+ P = L (L^T L)^-2 L^T = A^T A with A = S^-1 R_x, S = R_x R_x^T,
// and U is the R factor of A (positive diagonal).
//
// Default (one serial Cholesky).  With R_x = [R11 R12] (R11 k x k upper
// triangular, invertible) and C = R11^-1 R12:
//   S = R11 (I + C C^T) R11^T,  Z := R11^-1 S = R11^T + C R12^T,
//   A = S^-1 R_x = Z^-1 R11^-1 R_x = Z^-1 [I C].
// With N = Z Z^T = V V^T (V upper triangular, positive diagonal),
//   A^T A = [I C]^T N^-1 [I C] = (V^-1 [I C])^T (V^-1 [I C]),
// and V^-1 [I C] is upper trapezoidal with positive diagonal, so by
// uniqueness of the R factor  U = [V^-1, V^-1 C].  V comes from the upper
// Cholesky of the reversed N' = J N J = R^T R:  V = J R^T J, V^-1 = J R^-T J.
// Work: two triangular inverses (parallel recursive GEMMs), four GEMMs and
// ONE k x k blocked Cholesky, against two Choleskys (one over k x n rows) for
// the form below (TG_URX_TWOCHOL=1): S = T^T T, Y = T^-1, A = Y (Y^T R_x),
// U = first k rows of the upper Cholesky of A^T A.
// N has the conditioning of A[:, :k]^T A[:, :k], the same matrix the second
// Cholesky of the two-Cholesky form factors.
template <class Ar>
static void urx_layout(Ar &ar, int n, int k, double **S, double **Y, double **Bm, double **A,
                       double **Tt, double **Wb, int **info, double **Rq, RefineWs *rw) {
  const size_t h = size_t(NU) * ((tg::cdiv(k, NU) + 1) / 2);
  auto t = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<Ar, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  double *d[7];
  int *i0;
  t(S ? *S : d[0], size_t(k) * k);
  t(Y ? *Y : d[1], size_t(k) * k);
  t(Bm ? *Bm : d[2], size_t(k) * n);
  t(A ? *A : d[3], size_t(k) * n);
  t(Tt ? *Tt : d[4], h * h);
  t(Wb ? *Wb : d[5], size_t(NU) * NU);
  t(info ? *info : i0, 16);
  t(Rq ? *Rq : d[6], size_t(k) * k);
  refine_layout(ar, k, rw);
}


// N'[i][j] = N[k-1-i][k-1-j]
__global__ void flip_both_kernel(const double *__restrict__ N, int k, double *__restrict__ Np) {
  const int i = blockIdx.y;
  const double *src = N + size_t(k - 1 - i) * k + (k - 1);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < k; j += gridDim.x * blockDim.x)
    Np[size_t(i) * k + j] = src[-j];
}

extern "C" size_t tg_ufactor_rx_workspace_size(int n, int k) {
  tg::Sizer s;
  urx_layout(s, n, k, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
             nullptr);
  return s.off + 256;
}

// C = R11^-1 B for the upper-triangular R11 (k x k, ld ldr; its strict lower
// triangle zero) and B (k x m, ld ldr): back substitution by TB-row blocks
// from the bottom, block i = Dinv_i (Cw_i) then Cw[0:p] -= R11[0:p, i] C_i;
// Dinv (ld ldd) holds the inverses of the TB x TB diagonal blocks.
// Cw: k x m scratch (ld m); C: k x m (ld m).  k^2 m flops against the
// explicit R11^-1's k^3 / 3 (the near-full-rank layers' m = n - k is tiny).
constexpr int TB = 256;
static int trsm_upper_blocks(hipStream_t st, const double *R, int ldr, int k, const double *B,
                             int m, const double *Dinv, int ldd, double *Cw, double *C, int ldc) {
  TG_HIP(hipMemcpy2DAsync(Cw, sizeof(double) * ldc, B, sizeof(double) * ldr, sizeof(double) * m,
                          k, hipMemcpyDeviceToDevice, st));
  for (int bi = tg::cdiv(k, TB) - 1; bi >= 0; --bi) {
    const int p = bi * TB, pb = std::min(TB, k - p);
    TG_HIP(tg::dgemm(st, false, false, pb, m, pb, 1.0, Dinv + size_t(p) * ldd + p, ldd,
                     Cw + size_t(p) * ldc, ldc, 0.0, C + size_t(p) * ldc, ldc));
    if (p > 0)
      TG_HIP(tg::dgemm(st, false, false, p, m, pb, -1.0, R + p, ldr, C + size_t(p) * ldc, ldc, 1.0,
                       Cw, ldc));
  }
  return 0;
}

// The small-m form of the U factor (below): m * 16 <= k by default;
// TG_URX_SMALLM=0 / 1 forces the explicit-inverse form / this one.
static bool urx_small_m(int k, int m) {
  const char *e = getenv("TG_URX_SMALLM");
  if (e) return e[0] == '1';
  return int64_t(m) * 16 <= int64_t(k);
}

// Stages of the explicit form (below), shared with the column-sharded entry
// points (tg_urx_c / tg_urx_u11 / tg_urx_u12, gptq_svd_amd.dist.
// u_factor_rx_sharded): each column of C = R11^-1 R12 and of U12 = V^-1 C
// depends on its own column of R12 / C only (block back substitution and
// GEMMs with a fixed k order per entry), so a rank computing a column block
// gets the single-call values bit for bit.
// (a) the 256-block diagonal inverses of R11 into Yr (k x k, zeroed first)
static int urx_diag_inverses(hipStream_t st, const double *Rx, int ldr, int k, double *Yr,
                             double *Tt) {
  TG_HIP(hipMemsetAsync(Yr, 0, sizeof(double) * size_t(k) * k, st));
  hipLaunchKernelGGL(trinv_diag_kernel, dim3(tg::cdiv(k, NU)), dim3(256), 0, st, Rx, ldr, k, Yr,
                     k);
  TG_LAUNCHED();
  TG_HIP(trinv_offdiag(st, Rx, ldr, Yr, k, k, Tt, TB));
  return 0;
}
// (b) from the full C (k x m, ld ldc): Z^T = R11 + R12 C^T, N = Z Z^T, the
// Cholesky of N' = J N J (refined when ill-conditioned) and U11 = V^-1 into
// U; Yr, ZT, Nm, Rq: k x k scratch
static int urx_u11_from_c(hipStream_t st, const double *Rx, int ldr, int n, int k, const double *C,
                          int ldc, double *U, int ldu, double *Yr, double *ZT, double *Nm,
                          double *Rq, double *Tt, double *Wb, int *info, RefineWs &rw) {
  const int m = n - k;
  const dim3 gk(tg::cdiv(k, 256) < 16 ? tg::cdiv(k, 256) : 16, k);
  auto form_zt = [&](bool scratch_free) -> int {  // Z^T = R11 + R12 C^T
    TG_HIP(hipMemcpy2DAsync(ZT, sizeof(double) * k, Rx, sizeof(double) * ldr, sizeof(double) * k,
                            k, hipMemcpyDeviceToDevice, st));
    if (m <= 0) return 0;
    // the DGEMM stages 16-byte vectors only from 16-byte-aligned rows: with
    // an odd k R12's rows start mid-vector, so it is copied to an even-ld
    // buffer first (Y, when the caller says it is not live; C has an even
    // ld already)
    const int mp = m + (m & 1);
    const bool pad = scratch_free && ((k & 1) || (ldr & 1)) && mp <= k;
    if (pad) {
      double *R12p = Yr;
      TG_HIP(hipMemcpy2DAsync(R12p, sizeof(double) * mp, Rx + k, sizeof(double) * ldr,
                              sizeof(double) * m, k, hipMemcpyDeviceToDevice, st));
      TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, R12p, mp, C, ldc, 1.0, ZT, k));
    } else {
      TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, Rx + k, ldr, C, ldc, 1.0, ZT, k));
    }
    return 0;
  };
  if (const int e = form_zt(true)) return e;
  TG_HIP(tg::dsyrk_tn(st, k, k, 1.0, ZT, k, 0.0, Nm, k));         // N = Z Z^T
  hipLaunchKernelGGL(flip_both_kernel, gk, dim3(256), 0, st, Nm, k, Rq);  // N' = J N J
  TG_LAUNCHED();
  TG_HIP(chol_upper_rows(st, Rq, k, k, k, Wb, info));               // N' = R^T R
  hipLaunchKernelGGL(diag_range_kernel, dim3(1), dim3(256), 0, st, Rq, int64_t(k), k, rw.stats);
  TG_LAUNCHED();
  CholStat h{};
  TG_HIP(read_stat(st, rw.stats, info, h));
  if (needs_refine(h)) {
    double *Yq = Nm;
    TG_HIP(zero_lower(st, Rq, k, k));
    hipLaunchKernelGGL(flip_both_kernel, gk, dim3(256), 0, st, ZT, k, Yq);
    TG_LAUNCHED();
    const int e = refine_factor(st, Yq, k, k, Rq, rw, Wb, info, h);
    if (e != 0) return e;
  }
  TG_HIP(trinv(st, Rq, k, k, Yr, Tt));                              // Yr = R^-1
  hipLaunchKernelGGL(flip_transpose_kernel, gk, dim3(256), 0, st, Yr, k, U, int64_t(ldu));
  TG_LAUNCHED();                                                    // U11 = V^-1 = J R^-T J
  return 0;
}

extern "C" int tg_u_factor_rx(void *stream, const double *Rx, int ldr, int n, int k, double *U,
                              int ldu, void *ws, size_t ws_bytes) {
  TG_ARG(Rx, 2, "null Rx");
  TG_ARG(ldr >= n, 3, "ldr < n");
  TG_ARG(n >= 1, 4, "n < 1");
  TG_ARG(k >= 1 && k <= n, 5, "k must be in [1, n]");
  TG_ARG(U, 6, "null U");
  TG_ARG(ldu >= n, 7, "ldu < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  double *S, *Y, *Bm, *A, *Tt, *Wb, *Rq;
  int *info;
  RefineWs rw{};
  urx_layout(ar, n, k, &S, &Y, &Bm, &A, &Tt, &Wb, &info, &Rq, &rw);
  TG_WS(ar);
  TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
  const bool two_chol = getenv("TG_URX_TWOCHOL") != nullptr;  // read per call (tests set it)
  if (!two_chol) {
    const int m = n - k;
    const dim3 gk(tg::cdiv(k, 256) < 16 ? tg::cdiv(k, 256) : 16, k);
    const bool small_m = urx_small_m(k, m);
    // C: k x m; the explicit form keeps its ld even so the DGEMMs that read
    // it stage 16-byte vectors
    const int ldc = small_m ? m : m + (m & 1);
    double *Yr = Y, *C = Bm, *ZT = S, *Nm = A;
    TG_HIP(hipMemsetAsync(Yr, 0, sizeof(double) * size_t(k) * k, st));
    hipLaunchKernelGGL(trinv_diag_kernel, dim3(tg::cdiv(k, NU)), dim3(256), 0, st, Rx, ldr, k, Yr,
                       k);
    TG_LAUNCHED();
    auto form_zt = [&](bool scratch_free) -> int {  // Z^T = R11 + R12 C^T
      TG_HIP(hipMemcpy2DAsync(ZT, sizeof(double) * k, Rx, sizeof(double) * ldr,
                              sizeof(double) * k, k, hipMemcpyDeviceToDevice, st));
      if (m <= 0) return 0;
      // the DGEMM stages 16-byte vectors only from 16-byte-aligned rows: with
      // an odd k R12's rows start mid-vector, so it is copied to an even-ld
      // buffer first (Y, when the caller says it is not live; C has an even
      // ld already)
      const int mp = m + (m & 1);
      const bool pad = scratch_free && ((k & 1) || (ldr & 1)) && mp <= k;
      if (pad) {
        double *R12p = Yr;
        TG_HIP(hipMemcpy2DAsync(R12p, sizeof(double) * mp, Rx + k, sizeof(double) * ldr,
                                sizeof(double) * m, k, hipMemcpyDeviceToDevice, st));
        TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, R12p, mp, C, ldc, 1.0, ZT, k));
      } else {
        TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, Rx + k, ldr, C, ldc, 1.0, ZT, k));
      }
      return 0;
    };
    if (small_m) {
      // C = R11^-1 R12 by block back substitution (no explicit inverse), and
      // N = Z Z^T = (R11 + R12 C^T)^T (R11 + R12 C^T) as
      //   R11^T R11 + V C^T + C V^T,  V = R11^T R12 + C (R12^T R12) / 2,
      // the first term a triangular SYRK (a third of the square's flops)
      if (m > 0) {
        TG_HIP(trinv_offdiag(st, Rx, ldr, Yr, k, k, Tt, TB));          // 256-block inverses
        if (const int e = trsm_upper_blocks(st, Rx, ldr, k, Rx + k, m, Yr, k, Nm, C, ldc)) return e;
        double *V = ZT, *G = Rq;  // k x m and m x m (ld m)
        TG_HIP(tg::dgemm(st, true, false, k, m, k, 1.0, Rx, ldr, Rx + k, ldr, 0.0, V, m));
        TG_HIP(tg::dgemm(st, true, false, m, m, k, 1.0, Rx + k, ldr, Rx + k, ldr, 0.0, G, m));
        TG_HIP(tg::dgemm(st, false, false, k, m, m, 0.5, C, m, G, m, 1.0, V, m));
      }
      TG_HIP(tg::dsyrk_tn_upper(st, k, 1.0, Rx, ldr, 0.0, Nm, k));     // R11^T R11
      if (m > 0) {
        TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, ZT, m, C, m, 1.0, Nm, k));  // + V C^T
        TG_HIP(tg::dgemm(st, false, true, k, k, m, 1.0, C, m, ZT, m, 1.0, Nm, k));  // + C V^T
      }
    } else {
      // C = R11^-1 R12 by block back substitution over 256-row blocks, as in
      // the small-m form (k^2 m flops, no k^3 / 3 inverse: n = 12,288 at
      // 3n/4 rank -14 ms); TG_URX_INV=1 (development switch, read per call)
      // keeps the explicit inverse and its triangular product
      const char *ui = getenv("TG_URX_INV");
      if (ui && ui[0] == '1') {
        TG_HIP(trinv_offdiag(st, Rx, ldr, Yr, k, k, Tt));             // Yr = R11^-1
        if (m > 0) TG_HIP(tg::dgemm_upper_a(st, k, m, k, 1.0, Yr, k, Rx + k, ldr, 0.0, C, ldc));
      } else if (m > 0) {
        TG_HIP(trinv_offdiag(st, Rx, ldr, Yr, k, k, Tt, TB));         // 256-block inverses
        if (const int e = trsm_upper_blocks(st, Rx, ldr, k, Rx + k, m, Yr, k, Nm, C, ldc)) return e;
      }
      if (const int e = urx_u11_from_c(st, Rx, ldr, n, k, C, ldc, U, ldu, Yr, ZT, Nm, Rq, Tt, Wb,
                                       info, rw))
        return e;
      if (m > 0)
        TG_HIP(tg::dgemm_upper_a(st, k, m, k, 1.0, U, ldu, C, ldc, 0.0, U + k, ldu));  // V^-1 C
      return 0;
    }
    hipLaunchKernelGGL(flip_both_kernel, gk, dim3(256), 0, st, Nm, k, Rq);  // N' = J N J
    TG_LAUNCHED();
    TG_HIP(chol_upper_rows(st, Rq, k, k, k, Wb, info));               // N' = R^T R
    hipLaunchKernelGGL(diag_range_kernel, dim3(1), dim3(256), 0, st, Rq, int64_t(k), k, rw.stats);
    TG_LAUNCHED();
    CholStat h{};
    TG_HIP(read_stat(st, rw.stats, info, h));
    if (needs_refine(h)) {
      // R is the R factor of Yq = J Z^T J (Yq^T Yq = N'): CholeskyQR passes on Yq
      double *Yq = Nm;
      TG_HIP(zero_lower(st, Rq, k, k));
      if (small_m) {  // ZT held V
        if (const int e = form_zt(false)) return e;
      }
      hipLaunchKernelGGL(flip_both_kernel, gk, dim3(256), 0, st, ZT, k, Yq);
      TG_LAUNCHED();
      const int e = refine_factor(st, Yq, k, k, Rq, rw, Wb, info, h);
      if (e != 0) return e;
    }
    TG_HIP(trinv(st, Rq, k, k, Yr, Tt));                              // Yr = R^-1
    hipLaunchKernelGGL(flip_transpose_kernel, gk, dim3(256), 0, st, Yr, k, U, int64_t(ldu));
    TG_LAUNCHED();                                                    // U11 = V^-1 = J R^-T J
    if (m > 0)
      TG_HIP(tg::dgemm_upper_a(st, k, m, k, 1.0, U, ldu, C, ldc, 0.0, U + k, ldu));  // V^-1 C
    return 0;
  }
  CholStat h{};
  TG_HIP(tg::dsyrk_nt(st, k, n, 1.0, Rx, ldr, 0.0, S, k));        // S = R_x R_x^T
  TG_HIP(chol_upper_rows(st, S, k, k, k, Wb, info));                // S <- T, T^T T = S
  TG_HIP(read_stat(st, rw.stats, info, h));
  if (h.info > 0) {
    tg::set_error("U factor (two-Cholesky form): R_x R_x^T is not positive definite (%d pivots)",
                  h.info);
    return int(hipErrorUnknown);
  }
  TG_HIP(hipMemsetAsync(Y, 0, sizeof(double) * size_t(k) * k, st));
  hipLaunchKernelGGL(trinv_diag_kernel, dim3(tg::cdiv(k, NU)), dim3(256), 0, st, S, k, k, Y, k);
  TG_LAUNCHED();
  TG_HIP(trinv_offdiag(st, S, k, Y, k, k, Tt));                     // Y = T^-1
  TG_HIP(tg::dgemm(st, true, false, k, n, k, 1.0, Y, k, Rx, ldr, 0.0, Bm, n));  // T^-T R_x
  TG_HIP(tg::dgemm(st, false, false, k, n, k, 1.0, Y, k, Bm, n, 0.0, A, n));    // S^-1 R_x
  TG_HIP(tg::dgemm(st, true, false, k, n, k, 1.0, A, n, A, n, 0.0, U, ldu));    // G[:k, :]
  TG_HIP(chol_upper_rows(st, U, ldu, k, n, Wb, info));
  TG_HIP(zero_lower(st, U, ldu, k));
  TG_HIP(read_stat(st, rw.stats, info, h));
  if (h.info > 0) {
    tg::set_error("U factor (two-Cholesky form): Gram matrix not positive definite (%d pivots)",
                  h.info);
    return int(hipErrorUnknown);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// The explicit-form U factor in column-sharded pieces (multi-GPU,
// gptq_svd_amd.dist.u_factor_rx_sharded): rank r computes C[:, c0:c1] =
// R11^-1 R12[:, c0:c1] (tg_urx_c), the ranks all-gather C, every rank forms
// U11 = V^-1 from the whole C (tg_urx_u11: Z, N, one k x k Cholesky, the
// triangular inverse -- replicated), then rank r its U12 columns V^-1 C[:,
// c0:c1] (tg_urx_u12) and the ranks all-gather U12.  Every C and U12 entry
// depends on its own column only (block back substitution, GEMMs with a
// fixed k order per entry), so the gathered U equals tg_u_factor_rx's
// explicit form bit for bit (tests/test_gpu_urx_sharded.py).  Workspace:
// tg_ufactor_rx_workspace_size(n, k).  The small-m form (m * 16 <= k, the
// near-full-rank layers) is not sharded: its C is a sliver.
// ---------------------------------------------------------------------------
extern "C" int tg_urx_c(void *stream, const double *Rx, int ldr, int n, int k, int c0, int c1,
                        double *C, int ldc, void *ws, size_t ws_bytes) {
  TG_ARG(Rx, 2, "null Rx");
  TG_ARG(ldr >= n, 3, "ldr < n");
  TG_ARG(k >= 1 && k <= n, 5, "k must be in [1, n]");
  TG_ARG(c0 >= 0 && c0 <= c1 && c1 <= n - k, 6, "column range outside [0, n - k]");
  TG_ARG(C || c1 == c0, 8, "null C");
  TG_ARG(ldc >= c1 - c0, 9, "ldc < c1 - c0");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  double *S, *Y, *Bm, *A, *Tt, *Wb, *Rq;
  int *info;
  RefineWs rw{};
  urx_layout(ar, n, k, &S, &Y, &Bm, &A, &Tt, &Wb, &info, &Rq, &rw);
  TG_WS(ar);
  if (c1 == c0) return 0;
  if (const int e = urx_diag_inverses(st, Rx, ldr, k, Y, Tt)) return e;
  return trsm_upper_blocks(st, Rx, ldr, k, Rx + k + c0, c1 - c0, Y, k, A, C, ldc);
}

extern "C" int tg_urx_u11(void *stream, const double *Rx, int ldr, int n, int k, const double *C,
                          int ldc, double *U, int ldu, void *ws, size_t ws_bytes) {
  TG_ARG(Rx, 2, "null Rx");
  TG_ARG(ldr >= n, 3, "ldr < n");
  TG_ARG(k >= 1 && k <= n, 5, "k must be in [1, n]");
  TG_ARG(C || n == k, 6, "null C");
  TG_ARG(ldc >= n - k, 7, "ldc < n - k");
  TG_ARG(U, 8, "null U");
  TG_ARG(ldu >= n, 9, "ldu < n");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  double *S, *Y, *Bm, *A, *Tt, *Wb, *Rq;
  int *info;
  RefineWs rw{};
  urx_layout(ar, n, k, &S, &Y, &Bm, &A, &Tt, &Wb, &info, &Rq, &rw);
  TG_WS(ar);
  TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
  return urx_u11_from_c(st, Rx, ldr, n, k, C, ldc, U, ldu, Y, S, A, Rq, Tt, Wb, info, rw);
}

extern "C" int tg_urx_u12(void *stream, const double *U, int ldu, int k, const double *C, int ldc,
                          int ncols, double *out, int ldo) {
  TG_ARG(U, 2, "null U");
  TG_ARG(ldu >= k, 3, "ldu < k");
  TG_ARG(k >= 1, 4, "k < 1");
  TG_ARG(ncols >= 0, 7, "ncols < 0");
  TG_ARG((C && out) || ncols == 0, 5, "null C / out");
  TG_ARG(ldc >= ncols && ldo >= ncols, 6, "ldc / ldo < ncols");
  if (ncols == 0) return 0;
  TG_HIP(tg::dgemm_upper_a((hipStream_t)stream, k, ncols, k, 1.0, U, ldu, C, ldc, 0.0, out, ldo));
  return 0;
}

namespace {
template <class A>
void hinv_layout(A &ar, int n, double **Aw, double **Yw, double **Tw, double **Wb, double **mean,
                 int **info) {
  const size_t h = size_t(NU) * ((tg::cdiv(n, NU) + 1) / 2);
  auto t = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<A, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  double *d0, *d1, *d2, *d3, *d4;
  int *i0;
  t(Aw ? *Aw : d0, size_t(n) * n);
  t(Yw ? *Yw : d1, size_t(n) * n);
  t(Tw ? *Tw : d2, h * h);
  t(Wb ? *Wb : d3, size_t(NU) * NU);
  t(mean ? *mean : d4, 1);
  t(info ? *info : i0, 16);
}
}  // namespace

extern "C" size_t tg_hinv_chol_workspace_size(int n) {
  tg::Sizer s;
  hinv_layout(s, n, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  return s.off + 256;
}

extern "C" int tg_hinv_chol(void *stream, const double *H, int n, int ldh, const int64_t *perm,
                            double damp_percent, int max_tries, double *R, int ldr,
                            int *tries_used, void *ws, size_t ws_bytes) {
  TG_ARG(H, 2, "null H");
  TG_ARG(n >= 1, 3, "n < 1");
  TG_ARG(ldh >= n, 4, "ldh < n");
  TG_ARG(max_tries >= 1, 7, "max_tries < 1");
  TG_ARG(R, 8, "null R");
  TG_ARG(ldr >= n, 9, "ldr < n");
  TG_ARG(tries_used, 10, "null tries_used");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  double *A, *Y, *T, *Wb, *mean;
  int *info;
  hinv_layout(ar, n, &A, &Y, &T, &Wb, &mean, &info);
  TG_WS(ar);
  const dim3 g2(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, n);
  hipLaunchKernelGGL(diag_mean_kernel, dim3(1), dim3(256), 0, st, H, int64_t(ldh), n, mean);
  TG_LAUNCHED();
  // damping ladder of gptq_utils.py:148-160: damp = 10^e * damp_percent
  double scale = 1.0;
  for (int e = 0; e < max_tries; ++e, scale *= 10.0) {
    hipLaunchKernelGGL(flip_damp_kernel, g2, dim3(256), 0, st, H, int64_t(ldh), n, perm,
                       scale * damp_percent, mean, A);
    TG_LAUNCHED();
    TG_HIP(hipMemsetAsync(info, 0, sizeof(int), st));
    TG_HIP(chol_upper_rows(st, A, n, n, n, Wb, info));
    int h_info = 0;
    TG_HIP(hipMemcpyAsync(&h_info, info, sizeof(int), hipMemcpyDeviceToHost, st));
    TG_HIP(hipStreamSynchronize(st));
    if (h_info != 0) continue;  // not positive definite at this damping: next rung
    TG_HIP(hipMemsetAsync(Y, 0, sizeof(double) * size_t(n) * n, st));
    hipLaunchKernelGGL(trinv_diag_kernel, dim3(tg::cdiv(n, NU)), dim3(256), 0, st, A, n, n, Y, n);
    TG_LAUNCHED();
    TG_HIP(trinv_offdiag(st, A, n, Y, n, n, T));
    hipLaunchKernelGGL(flip_transpose_kernel, g2, dim3(256), 0, st, Y, n, R, int64_t(ldr));
    TG_LAUNCHED();
    *tries_used = e;
    return 0;
  }
  // every rung failed: identity (the reference's intended fallback, :162-164)
  hipLaunchKernelGGL(identity_kernel, g2, dim3(256), 0, st, n, R, int64_t(ldr));
  TG_LAUNCHED();
  *tries_used = max_tries;
  return 0;
}
