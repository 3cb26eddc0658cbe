// Panel QR of the two-stage band reduction (band.hip, sy2sb): for the
// panel P = A[r0:r0+m, p:p+32] it forms ONE compact-WY block,
//   P = H [R; 0],  H = I - Y T Y^T  (Y m x 32 unit lower trapezoidal),
// and writes [R; 0] (and its transpose) back into A.
//
// Replaces the per-panel Householder QR of the reduction inside
// `torch.linalg.eigh` (/root/reference/src/TruncGPTQ/gptq_utils.py:93).
// One persistent launch per panel: NW workgroups (launched 8 NW, the ones
// with blockIdx % 8 == 0 work, so they share one XCD's L2 under round-robin
// dispatch; correctness does not depend on it), each holding 256 rows of P in
// LDS, an in-launch grid barrier between phases (cdna_hip_programming.md §6
// Guideline 16: write-through sc1 payload stores, every storing wave drains
// vmcnt, one relaxed counter add per workgroup, bounded relaxed poll, sc1
// payload loads):
//  1. CholeskyQR2 (Yamamoto et al. 2015): G = Q^T Q on FP64 MFMA (partials
//     per workgroup, summed in workgroup order by workgroup 0), L = chol(G)
//     by one wave, Q <- Q L^-T by row-wise forward substitution (backward
//     stable).  The first pass is shifted (Fukaya et al. 2020) when its
//     pivots show a condition number near 1/sqrt(eps); passes repeat until
//     the Gram matrix of the current Q is within 0.1 of I (at most NPASS).
//  2. Householder reconstruction (Ballard et al. 2015): LU of I - Q1 S
//     (S_jj = -sign chosen during the elimination, pivots 1 + |.| >= 1)
//     gives Y1 = L and U; Y2 = -Q2 S U^-1 (forward substitution with U),
//     T = U Y1^-T, R = S (L_g^T ... L_1^T).
//  3. Fallback (rank-deficient or numerically singular panels, m < 64):
//     Householder column by column over the grid, one barrier per column
//     (one reduction gives the column norm and every w = P^T v entry).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <utility>

#include "band.h"
#include "common.h"
#include "spin.h"
#include "lanes.h"

namespace {

using tg::SB_B;
constexpr int PT = 256;    // threads per workgroup (4 waves) = rows per workgroup
constexpr int XS = 34;     // row stride of the LDS row block (16-B aligned rows)
constexpr int NPASS = 4;   // Gram passes before the Householder fallback
constexpr int FB_MIN_M = 64;
constexpr double SERIES_TOL = 1e-5;  // |G - I| below which the last factor is a series

enum Dec { DEC_CONTINUE = 1, DEC_ACCEPT = 2, DEC_FALLBACK = 3 };

// broadcast block layout (doubles)
constexpr int BC_DEC = 0, BC_L = 64, BC_RINV = BC_L + 1024, BC_T = BC_RINV + 64,
              BC_PROW = BC_T + 1024, BC_MB = BC_PROW + 128, BC_SIZE = BC_MB + 2048;
static_assert(BC_SIZE <= tg::PQR_BC_DOUBLES, "broadcast block");

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;

struct PqrArgs {
  double *A;
  int64_t lda;
  int p, r0, m, nw;
  double *Y, *YT, *T;  // outputs (Y, YT: m x 32 row-major)
  double *part;        // partials: Gram nw x 1024 | fallback 2 x nw x 32
  double *bc;          // broadcast block
  unsigned *cnt;       // [0] barrier counter, [1] path record (zeroed before the launch)
  unsigned *tmo;       // timeout flag (shared by all panels)
  unsigned long long timeout;
  unsigned long long *stats;  // TG_PQR_STATS: per-phase clock stamps of workgroup 0 (or null)
  int force_fb;               // TG_PQR_FALLBACK=1: every panel through the Householder path (tests)
  int wstride;                // blocks per worker: the XCD count (workers on one XCD) or 1
};

struct PqrSm {
  double Xs[PT][XS];          // this workgroup's rows (panel row 256 w + t in Xs[t])
  double Gs[32][33];          // workgroup 0: Gram sum; HR: U^-1; fallback: reduce rows
  double Lt[32][33];          // this pass's L (Lt[c][i] = L[i][c], i.e. L^T)
  double Ra[32][33];          // workgroup 0: R = L_g^T ... L_1^T
  double Ut[32][33], Tm[32][33];
  double Cq[32][33];          // Q top rows -> Y1 (HR); fallback: T recurrence input
  double RgI[32][33];         // (L_g^T)^-1; scratch of the R update
  double MB[32][65];          // [M1 | M1 T] of the final CholeskyQR pass
  double rinv[32], uinv[32], sv[32];
  double dsum[32], prow[32], taus[32];
  double delta;
  double bcast[4][128];        // one-wave broadcast rows (+ a trash slot per lane), 2 x double-buffered
  int dec;
  PqrArgs ga;                 // the launch arguments (read by the out-of-line phases)
};

// Per-workgroup state at file scope, so the out-of-line phases below address
// it as LDS without pointer arguments.  The phases are kept out of line so
// that their unrolled address arithmetic is not hoisted across the pass loop
// (it once held ~700 SGPRs and spilled).
__shared__ PqrSm s_pq;

#ifdef TG_PQR_DBG
__device__ unsigned long long g_pq_dbg[64];
#define DBG_STAMP(k) \
  if (threadIdx.x == 0) g_pq_dbg[(k)] += __builtin_amdgcn_s_memrealtime();
#define DBG_STAMP_T(k, t) \
  if (threadIdx.x == (t)) g_pq_dbg[(k)] += __builtin_amdgcn_s_memrealtime();
#else
#define DBG_STAMP(k)
#define DBG_STAMP_T(k, t)
#endif

// threadIdx.x through an empty asm: every phase derives its lane indices and
// LDS addresses from its own opaque copy, so the compiler neither hoists them
// out of the pass loop nor shares them between inlined phases (which held
// hundreds of registers live across the kernel and spilled).
__device__ __forceinline__ int otid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

typedef __attribute__((address_space(1))) double gf64;
__device__ __forceinline__ void st_sc1(double *p, double v) {
  __hip_atomic_store((gf64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
  return __hip_atomic_load((gf64 *)const_cast<double *>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double rsq_nr(double x) {  // 1/sqrt(x), ~1 ulp
  double r = __builtin_amdgcn_rsq(x);
  r = r * fma(-0.5 * x * r, r, 1.5);
  return r * fma(-0.5 * x * r, r, 1.5);
}
__device__ __forceinline__ double rcp_nr(double x) {  // 1/x, ~1 ulp
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Grid barrier (counter form): every wave's sc1 stores drained, one arrival
// per workgroup and a bounded poll, both by wave 0 as a whole wave (scalar
// loop, spin.h); a stalled barrier sets *tmo and later ones return at once.
__device__ __forceinline__ void grid_bar(const PqrArgs &g, unsigned &ep) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ++ep;
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    tg::wave_arrive(g.cnt);
    tg::spin_geq(g.cnt, unsigned(g.nw) * ep, g.tmo, g.timeout);
  }
  __syncthreads();
}

// Panel row i (zeros past m) into registers.
__device__ __forceinline__ void load_row(const PqrArgs &g, int i, double (&x)[32]) {
  const int ic = min(i, g.m - 1);
  const double *s = g.A + (g.r0 + int64_t(ic)) * g.lda + g.p;
  double2 v[16];
  if ((g.lda & 1) == 0 && (g.p & 1) == 0) {
    const double2 *s2 = reinterpret_cast<const double2 *>(s);
#pragma unroll
    for (int l = 0; l < 16; ++l) v[l] = s2[l];
  } else {
#pragma unroll
    for (int l = 0; l < 16; ++l) v[l] = make_double2(s[2 * l], s[2 * l + 1]);
  }
  const bool ok = i < g.m;
#pragma unroll
  for (int l = 0; l < 16; ++l) {
    x[2 * l] = ok ? v[l].x : 0.0;
    x[2 * l + 1] = ok ? v[l].y : 0.0;
  }
}
__device__ __forceinline__ void row_to_lds(double *dst, const double (&x)[32]) {
  double2 *d = reinterpret_cast<double2 *>(dst);
#pragma unroll
  for (int l = 0; l < 16; ++l) d[l] = make_double2(x[2 * l], x[2 * l + 1]);
}
__device__ __forceinline__ void row_from_lds(const double *src, double (&x)[32]) {
  const double2 *s = reinterpret_cast<const double2 *>(src);
#pragma unroll
  for (int l = 0; l < 16; ++l) {
    const double2 v = s[l];
    x[2 * l] = v.x;
    x[2 * l + 1] = v.y;
  }
}

// x <- x L^-T (forward substitution; Lt[c][l] = L[l][c] = R[c][l]).  Row
// c + 1 of Lt is loaded while column c is applied; the empty asm with a
// memory clobber keeps the compiler from hoisting all 528 uniform LDS loads
// to the top (they then spill).
__device__ __forceinline__ void trsm_row(double (&x)[32], const double (*Lt)[33], const double *rinv) {
  double cur[32], nxt[32];
#pragma unroll
  for (int l = 1; l < 32; ++l) cur[l] = Lt[0][l];
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    const double rc = rinv[c];
#pragma unroll
    for (int l = c + 2; l < 32; ++l) nxt[l] = Lt[c + 1 < 32 ? c + 1 : 31][l];
    x[c] *= rc;
#pragma unroll
    for (int l = c + 1; l < 32; ++l) x[l] = fma(-x[c], cur[l], x[l]);
#pragma unroll
    for (int l = c + 2; l < 32; ++l) cur[l] = nxt[l];
    asm volatile("" ::: "memory");
  }
}

// C = A diag(d) B for 32 x 32 LDS matrices on FP64 MFMA (d = null: no
// scaling): wave w computes the 16 x 16 block (w >> 1, w & 1), K = 32.
// C may not alias A or B.  All four waves of the workgroup must call it.
template <int LDA, int LDB, int LDC>
__device__ __forceinline__ void mm32(double *C, const double *A, const double *B, const double *d) {
  const int tid = otid(), lane = tid & 63, wid = tid >> 6, lr = lane >> 4, lc = lane & 15;
  const int bi = 16 * (wid >> 1), bj = 16 * (wid & 1);
  doublex4 acc = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 4) {
    double a = A[(bi + lc) * LDA + k0 + lr];
    if (d) a *= d[k0 + lr];
    const double b = B[(k0 + lr) * LDB + bj + lc];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) C[(bi + lr + 4 * q) * LDC + bj + lc] = acc[q];
}

// This workgroup's Gram partial of its LDS rows -> part[w]: waves 0, 1, 2
// take the 16 x 16 blocks (0,0), (0,1), (1,1) over all 256 rows (no
// cross-wave reduction); (1,0) is the transpose of (0,1).
__device__ __forceinline__ void gram_publish(const PqrArgs &g, PqrSm &sm, int w) {
  const int tid = otid(), lane = tid & 63, wid = tid >> 6, lr = lane >> 4, lc = lane & 15;
  if (wid >= 3) return;
  const int ia = wid == 2 ? 16 : 0, cb = wid == 0 ? 0 : 16;
  doublex4 acc[2] = {doublex4{0.0, 0.0, 0.0, 0.0}, doublex4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll 4
  for (int k0 = 0; k0 < PT; k0 += 8) {
    const double a0 = sm.Xs[k0 + lr][ia + lc], b0 = sm.Xs[k0 + lr][cb + lc];
    const double a1 = sm.Xs[k0 + 4 + lr][ia + lc], b1 = sm.Xs[k0 + 4 + lr][cb + lc];
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1], 0, 0, 0);
  }
  double *out = g.part + int64_t(w) * 1024;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double v = acc[0][q] + acc[1][q];
    const int r = ia + lr + 4 * q, c = cb + lc;
    st_sc1(out + r * 32 + c, v);
    if (wid == 1) st_sc1(out + c * 32 + r, v);
  }
}

// Workgroup 0: G = sum of the partials in workgroup order -> Gs.
__device__ __forceinline__ void gram_reduce(const PqrArgs &g, PqrSm &sm) {
  const int tid = otid();
  constexpr int NB = 16;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int w0 = 0; w0 < g.nw; w0 += NB) {
    double v[4][NB];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        v[u][b] = ld_sc1(g.part + int64_t(min(w0 + b, g.nw - 1)) * 1024 + tid + PT * u);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[u] += (w0 + b < g.nw) ? v[u][b] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + PT * u;
    sm.Gs[e >> 5][e & 31] = acc[u];
  }
}

// One wave: L = chol(Gs + shift I) into Lt (Lt[c][i] = L[i][c]) and rinv;
// lane (i = lane & 31, h = lane >> 5) holds row i, columns 16h .. 16h + 15;
// column j is broadcast through LDS at each step.  The pivot chain is kept
// free of compares and selects (lanes above the pivot compute unused upper
// entries); ok (every pivot positive and finite) and minrat = min_j
// pivot_j / (G_jj + shift) are evaluated once at the end from L's diagonal.
__device__ __forceinline__ bool chol32_ool(double shift, double &minrat) {
  PqrSm &sm = s_pq;
  const int lane = otid() & 63, i = lane & 31, h = lane >> 5;
  double gr[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) gr[c] = sm.Gs[i][16 * h + c] + (16 * h + c == i ? shift : 0.0);
  // Software-pipelined: column 0 is published and read up front; step j
  // updates column j + 1 first, publishes it (double-buffered LDS) and issues
  // the next step's reads before the rest of its own update, so the LDS round
  // trip overlaps the remaining fma.
  auto read_col = [&](int j, double &piv, double &gij, double (&col)[16]) {
    const double *buf = sm.bcast[j & 1];
    wave_lds_sync();
    piv = buf[j];
    gij = buf[i];
    const double2 *b2 = reinterpret_cast<const double2 *>(buf + 16 * h);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const double2 v = b2[c];
      col[2 * c] = v.x;
      col[2 * c + 1] = v.y;
    }
  };
  double piv, gij, col[16];
  DBG_STAMP(24)
  sm.bcast[0][h == 0 ? i : 32 + lane] = gr[0];
  read_col(0, piv, gij, col);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int hj = j >> 4, cj = j & 15;
    const double r = rsq_nr(piv);
    const double lij = gij * r;  // L[i][j] for i >= j (i == j: sqrt(piv)); 0 above
    const double mlr = -lij * r;
    double pn = 0.0, gn = 0.0, cn2[16];
    if (j + 1 < 32) {
      // lanes of column j + 1 publish its rows >= j + 1 (rows above as 0, so
      // that the update needs no per-entry mask: those rows get l = 0 and no
      // row's finished columns are touched); the others write a slot nobody reads
      const int hn = (j + 1) >> 4, cn = (j + 1) & 15;
      gr[cn] = fma(mlr, col[cn], gr[cn]);
      sm.bcast[(j + 1) & 1][h == hn ? i : 32 + lane] = i >= j + 1 ? gr[cn] : 0.0;
      read_col(j + 1, pn, gn, cn2);
    }
#pragma unroll
    for (int c = 0; c < 16; ++c)  // column j itself: reset below
      if (c != ((j + 1) & 15) || j + 1 >= 32) gr[c] = fma(mlr, col[c], gr[c]);
    if (h == hj) gr[cj] = lij;
    if (j + 1 < 32) {
      piv = pn;
      gij = gn;
#pragma unroll
      for (int c = 0; c < 16; ++c) col[c] = cn2[c];
    }
  }
  DBG_STAMP(25)
  double dg = 1.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    sm.Lt[16 * h + c][i] = (16 * h + c <= i) ? gr[c] : 0.0;
    dg = (16 * h + c == i) ? gr[c] : dg;
  }
  // lane i (its diagonal half): L_ii > 0 finite, pivot ratio L_ii^2 / (G_ii + shift)
  const bool mine = (i >> 4) == h;
  if (mine) sm.rinv[i] = rcp_nr(dg);
  const bool good = !mine || (dg > 0.0 && dg <= DBL_MAX);
  double rat = mine ? dg * dg / (sm.Gs[i][i] + shift) : 1.0;
  if (!(rat == rat)) rat = 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) rat = fmin(rat, __shfl_xor(rat, off));
  minrat = rat;
  const bool allgood = __all(good);
  DBG_STAMP(26)
  return allgood;
}

// X = R^-1 for a 32 x 32 upper triangular R = get(i, k) (i <= k) with
// reciprocal diagonal rd (unit: rd = null), by blocks: the four 8 x 8
// diagonal blocks by back substitution (one thread per column), then two
// levels of  X12 = -A^-1 B D^-1.  All threads of the workgroup; X is LDS
// (stride 33), lower part zeroed; `tmp` is 32 x 33 LDS scratch.
template <class Get>
__device__ __forceinline__ void trinv_upper32(Get get, const double *rd, double (*X)[33],
                                              double (*tmp)[33]) {
  const int tid = otid();
  for (int e = tid; e < 1024; e += PT) X[e >> 5][e & 31] = 0.0;
  __syncthreads();
  if (tid < 32) {
    const int bb = 8 * (tid >> 3), c = tid & 7;
    double x[8];
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      double acc = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int k = i + 1; k < 8; ++k) acc = fma(-get(bb + i, bb + k), x[k], acc);
      x[i] = (i <= c) ? acc * (rd ? rd[bb + i] : 1.0) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) X[bb + i][bb + c] = x[i];
  }
  __syncthreads();
  // level 1 (16 x 16 blocks at 0 and 16): T1 = B D^-1, then X12 = -A^-1 T1
#pragma unroll
  for (int lev = 0; lev < 2; ++lev) {
    const int hb = lev == 0 ? 8 : 16;        // half block size
    const int nblk = lev == 0 ? 2 : 1;       // blocks of size 2 hb
    const int cnt = nblk * hb * hb;
    if (tid < cnt) {
      const int blk = tid / (hb * hb), r = (tid / hb) % hb, c = tid % hb;
      const int o = blk * 2 * hb;
      double acc = 0.0;
      for (int k = 0; k <= c; ++k) acc = fma(get(o + r, o + hb + k), X[o + hb + k][o + hb + c], acc);
      tmp[o + r][o + hb + c] = acc;
    }
    __syncthreads();
    if (tid < cnt) {
      const int blk = tid / (hb * hb), r = (tid / hb) % hb, c = tid % hb;
      const int o = blk * 2 * hb;
      double acc = 0.0;
      for (int k = r; k < hb; ++k) acc = fma(X[o + r][o + k], tmp[o + k][o + hb + c], acc);
      X[o + r][o + hb + c] = -acc;
    }
    __syncthreads();
  }
}

// Two independent inverses at once (the Householder reconstruction's U^-1 and
// Y1^-T): the same blocked steps with matrix A on waves 0-1 and B on waves 2-3
// where a step has at most 128 items, both per thread where it has 256, so the
// two share every barrier and their dependent fma chains overlap.
template <class GetA, class GetB>
__device__ __forceinline__ void trinv2_upper32(GetA geta, const double *rda, double (*XA)[33],
                                               double (*tmpA)[33], GetB getb, const double *rdb,
                                               double (*XB)[33], double (*tmpB)[33]) {
  const int tid = otid();
  for (int e = tid; e < 1024; e += PT) {
    XA[e >> 5][e & 31] = 0.0;
    XB[e >> 5][e & 31] = 0.0;
  }
  __syncthreads();
  auto diag = [&](auto get, const double *rd, double (*X)[33], int t) {
    const int bb = 8 * (t >> 3), c = t & 7;
    double x[8];
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      double acc = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int k = i + 1; k < 8; ++k) acc = fma(-get(bb + i, bb + k), x[k], acc);
      x[i] = (i <= c) ? acc * (rd ? rd[bb + i] : 1.0) : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) X[bb + i][bb + c] = x[i];
  };
  if (tid < 32) diag(geta, rda, XA, tid);
  else if (tid >= 128 && tid < 160) diag(getb, rdb, XB, tid - 128);
  __syncthreads();
#pragma unroll
  for (int lev = 0; lev < 2; ++lev) {
    const int hb = lev == 0 ? 8 : 16;
    auto prod1 = [&](auto get, double (*X)[33], double (*tmp)[33], int t) {
      const int blk = t / (hb * hb), r = (t / hb) % hb, c = t % hb;
      const int o = blk * 2 * hb;
      double acc = 0.0;
      for (int k = 0; k <= c; ++k) acc = fma(get(o + r, o + hb + k), X[o + hb + k][o + hb + c], acc);
      tmp[o + r][o + hb + c] = acc;
    };
    auto prod2 = [&](double (*X)[33], double (*tmp)[33], int t) {
      const int blk = t / (hb * hb), r = (t / hb) % hb, c = t % hb;
      const int o = blk * 2 * hb;
      double acc = 0.0;
      for (int k = r; k < hb; ++k) acc = fma(X[o + r][o + k], tmp[o + k][o + hb + c], acc);
      X[o + r][o + hb + c] = -acc;
    };
    if (lev == 0) {  // 2 blocks of 8 x 8: 128 items per matrix
      if (tid < 128) prod1(geta, XA, tmpA, tid);
      else prod1(getb, XB, tmpB, tid - 128);
      __syncthreads();
      if (tid < 128) prod2(XA, tmpA, tid);
      else prod2(XB, tmpB, tid - 128);
    } else {  // one 16 x 16 block: 256 items per matrix
      prod1(geta, XA, tmpA, tid);
      prod1(getb, XB, tmpB, tid);
      __syncthreads();
      prod2(XA, tmpA, tid);
      prod2(XB, tmpB, tid);
    }
    __syncthreads();
  }
}

// Workgroup 0: LU of I - Cq S (Householder reconstruction) into Ut (U), Cq
// (Y1, unit lower), sv (S), uinv.  All four waves: thread t holds row t >> 3,
// columns 4 (t & 7) .. + 3, so a step is a few dozen instructions per wave (a
// single wave holding 16 entries per lane spent ~1.5k cycles per pivot pair,
// issue-bound).  Two pivots per barrier: step j (even) reads rows j, j + 1 and
// columns j, j + 1 as left by step j - 2; every thread forms L_{j+1,j}, the
// updated pivot U_{j+1,j+1} and its row's updated column j + 1 entry itself
// (the same fma a sequential step does, so the factors are bit-identical),
// then applies both rank-1 terms.  Columns j + 2, j + 3 are published before
// the rest of the update, rows j + 2, j + 3 after it (double-buffered).
__device__ __forceinline__ void lu_hr() {
  PqrSm &sm = s_pq;
  const int tid = otid();
  const int i = tid >> 3, g = tid & 7;
  double c[4], lw[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    c[l] = sm.Cq[i][4 * g + l];
    lw[l] = 0.0;
  }
  double svr = 0.0;  // thread j < 32: S_jj
  // parity p: rows j, j + 1 at bcast[2p][0..31], [32..63]; columns j, j + 1 at
  // bcast[2p + 1][0..31], [32..63] (entry of row i at i)
  auto put_rows = [&](int j2, double *rb) {
    if (i == j2 || i == j2 + 1) {
      double2 *d2 = reinterpret_cast<double2 *>(rb + 32 * (i - j2) + 4 * g);
      d2[0] = make_double2(c[0], c[1]);
      d2[1] = make_double2(c[2], c[3]);
    }
  };
  auto put_cols = [&](int j2, double *cb) {
    if (g == (j2 >> 2)) {
      cb[i] = c[j2 & 3];
      cb[32 + i] = c[(j2 & 3) + 1];
    }
  };
  put_cols(0, sm.bcast[1]);
  put_rows(0, sm.bcast[0]);
  // L_ij = -S_jj C^(j)_ij / U_jj, U_jj = 1 + |C^(j)_jj|, S_jj = -sign(C^(j)_jj),
  // C^(j+1)_il = C^(j)_il - L_ij C^(j)_jl.  No per-entry masks: rows <= j take
  // l = 0; the working columns < j (and j, once L_ij is in lw) are dead and
  // only ever feed dead columns.
#pragma unroll
  for (int j = 0; j < 32; j += 2) {
    const double *rb = sm.bcast[2 * ((j >> 1) & 1)], *cb = sm.bcast[2 * ((j >> 1) & 1) + 1];
    __syncthreads();
    const double qjj = cb[j], cj1j = cb[j + 1];            // C_jj, C_{j+1,j}
    const double cjj1 = cb[32 + j], cj1j1 = cb[32 + j + 1];  // C_{j,j+1}, C_{j+1,j+1}
    const double cij = cb[i], cij1 = cb[32 + i];           // C_ij, C_{i,j+1}
    double r0[4], r1[4];
    {
      const double2 *a2 = reinterpret_cast<const double2 *>(rb + 4 * g);
      const double2 *b2 = reinterpret_cast<const double2 *>(rb + 32 + 4 * g);
      const double2 a = a2[0], b = a2[1], u = b2[0], v = b2[1];
      r0[0] = a.x; r0[1] = a.y; r0[2] = b.x; r0[3] = b.y;
      r1[0] = u.x; r1[1] = u.y; r1[2] = v.x; r1[3] = v.y;
    }
    const double ms0 = copysign(1.0, qjj);
    const double ru0 = rcp_nr(1.0 + fabs(qjj));
    const double lij = i > j ? ms0 * cij * ru0 : 0.0;
    const double lj1 = ms0 * cj1j * ru0;  // row j + 1's (as its own thread forms it)
    const double piv1 = fma(-lj1, cjj1, cj1j1);
    const double cij1u = fma(-lij, cjj1, cij1);
    const double ms1 = copysign(1.0, piv1);
    const double ru1 = rcp_nr(1.0 + fabs(piv1));
    const double lij1 = i > j + 1 ? ms1 * cij1u * ru1 : 0.0;
    svr = tid == j ? -ms0 : (tid == j + 1 ? -ms1 : svr);
    if (g == (j >> 2)) {
      lw[j & 3] = lij;
      lw[(j & 3) + 1] = lij1;
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) r1[l] = fma(-lj1, r0[l], r1[l]);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      c[l] = fma(-lij, r0[l], c[l]);
      c[l] = fma(-lij1, r1[l], c[l]);
    }
    if (j + 2 < 32) {
      const int np = ((j >> 1) + 1) & 1;
      put_cols(j + 2, sm.bcast[2 * np + 1]);
      put_rows(j + 2, sm.bcast[2 * np]);
    }
  }
  if (tid < 32) sm.sv[tid] = svr;
  __syncthreads();
  DBG_STAMP_T(20, 0)
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const int col = 4 * g + l;
    sm.Ut[i][col] = (col == i) ? 1.0 + fabs(c[l]) : (col > i ? -sm.sv[col] * c[l] : 0.0);
    sm.Cq[i][col] = (col < i) ? lw[l] : (col == i ? 1.0 : 0.0);
    if (col == i) sm.uinv[i] = rcp_nr(1.0 + fabs(c[l]));
  }
}

// Workgroup 0 after acceptance (Lt = this pass's factor L_g, Ra = L_g^T ...
// L_1^T, the LDS rows = Q_{g-1}):
//   RgI = (L_g^T)^-1 (trinv_upper32), Cq = the final Q's top rows = Xs[0:32] RgI;
//   wave 0: LU of I - Cq S (Householder reconstruction): U, Y1 (into Cq), S;
//   U^-1 and Y1^-T (trinv_upper32), T = U Y1^-T, the band block S R written
//   to A, MB = [M1 | M1 T] with M1 = RgI (-S) U^-1, and Y1 T (into Ut)
// so that a row q of the previous pass gives Y = q M1, Y T = q M1 T.
__device__ __forceinline__ void hr_top_ool() {
  PqrSm &sm = s_pq;
  const PqrArgs &g = sm.ga;
  const int tid = otid();
  double(*UI)[33] = sm.Gs;
  double(*Tmp)[33] = reinterpret_cast<double(*)[33]>(&sm.MB[0][0]);  // MB is written last
  DBG_STAMP(16)
  if (sm.delta <= SERIES_TOL) {
    // R = I + F with |F| <= ~1e-5: R^-1 = I - F + F^2 - F^3 (error |F|^4)
    for (int e = tid; e < 1024; e += PT) {
      const int i2 = e >> 5, j2 = e & 31;
      sm.Ut[i2][j2] = sm.Lt[i2][j2] - (i2 == j2 ? 1.0 : 0.0);  // F
    }
    __syncthreads();
    mm32<33, 33, 33>(&sm.Cq[0][0], &sm.Ut[0][0], &sm.Ut[0][0], nullptr);  // F^2
    __syncthreads();
    mm32<33, 33, 33>(&Tmp[0][0], &sm.Cq[0][0], &sm.Ut[0][0], nullptr);  // F^3
    __syncthreads();
    for (int e = tid; e < 1024; e += PT) {
      const int i2 = e >> 5, j2 = e & 31;
      sm.RgI[i2][j2] = (i2 == j2 ? 1.0 : 0.0) - sm.Ut[i2][j2] + sm.Cq[i2][j2] - Tmp[i2][j2];
    }
    __syncthreads();
  } else {
    trinv_upper32([&](int i, int k) { return sm.Lt[i][k]; }, sm.rinv, sm.RgI, Tmp);
  }
  mm32<XS, 33, 33>(&sm.Cq[0][0], &sm.Xs[0][0], &sm.RgI[0][0], nullptr);
  __syncthreads();
  lu_hr();
  __syncthreads();
  DBG_STAMP(17)
  // the band block S R (lower storage: the upper part of A is never read again)
  for (int e = tid; e < 1024; e += PT) {
    const int i2 = e >> 5, cc = e & 31;
    g.A[(g.r0 + int64_t(i2)) * g.lda + g.p + cc] = (i2 <= cc) ? sm.sv[i2] * sm.Ra[i2][cc] : 0.0;
  }
  // U^-1 and Y1^-T = (Y1^T)^-1 (unit upper, into Tm); Lt (this pass's factor,
  // already folded into RgI and Ra) is the second scratch
  trinv2_upper32([&](int i, int k) { return sm.Ut[i][k]; }, sm.uinv, UI, Tmp,
                 [&](int i, int k) { return sm.Cq[k][i]; }, nullptr, sm.Tm, sm.Lt);
  DBG_STAMP(18)
  if (tid < 32) sm.dsum[tid] = -sm.sv[tid];
  // T = U Y1^-T (into Tmp, then Tm), M1 = RgI (-S) U^-1
  mm32<33, 33, 33>(&Tmp[0][0], &sm.Ut[0][0], &sm.Tm[0][0], nullptr);
  __syncthreads();
  for (int e = tid; e < 1024; e += PT) sm.Tm[e >> 5][e & 31] = Tmp[e >> 5][e & 31];
  __syncthreads();
  mm32<33, 33, 65>(&sm.MB[0][0], &sm.RgI[0][0], &UI[0][0], sm.dsum);
  mm32<33, 33, 33>(&sm.Ut[0][0], &sm.Cq[0][0], &sm.Tm[0][0], nullptr);  // Y1 T (U done)
  __syncthreads();
  mm32<65, 33, 65>(&sm.MB[0][32], &sm.MB[0][0], &sm.Tm[0][0], nullptr);
  __syncthreads();
  DBG_STAMP(19)
}

// Final pass of the CholeskyQR path: [Y | Y T] = Q_prev [M1 | M1 T] on FP64
// MFMA (Q_prev = the LDS rows), rows >= 32; workgroup 0's rows < 32 are Y1
// (from the LU) and Y1 T.  Also zeroes the panel rows >= 32 in A.
__device__ __forceinline__ void final_rows(const PqrArgs &g, PqrSm &sm, int w) {
  const int tid = otid(), lane = tid & 63, wid = tid >> 6, lr = lane >> 4, lc = lane & 15;
  doublex4 acc[4][4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = doublex4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < 32; k0 += 4) {
    double bf[4], af[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) bf[cb] = sm.MB[k0 + lr][16 * cb + lc];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) af[rb] = sm.Xs[64 * wid + 16 * rb + lc][k0 + lr];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[rb][cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[rb], bf[cb], acc[rb][cb], 0, 0, 0);
  }
  const int base = w * PT + 64 * wid;
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = base + 16 * rb + lr + 4 * q;
      if (i < SB_B || i >= g.m) continue;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        (cb < 2 ? g.Y : g.YT)[int64_t(i) * SB_B + 16 * (cb & 1) + lc] = acc[rb][cb][q];
    }
  // (the panel's rows below the band block are never read again: A is destroyed)
  if (w == 0 && tid < 2 * SB_B) {
    // rows 0..31: Y1 (from the LU) and Y1 T (hr_top), 32 columns per lane
    const int i2 = tid & 31;
    const double *src = (tid < SB_B) ? &sm.Cq[i2][0] : &sm.Ut[i2][0];
    double *dst = ((tid < SB_B) ? g.Y : g.YT) + i2 * SB_B;
#pragma unroll
    for (int c = 0; c < 32; ++c) dst[c] = src[c];
  }
}

// Fallback: Householder QR over the grid, one barrier per column, from the
// original panel row of each thread (registers); writes Y, Y T, T and [R; 0].
__device__ __forceinline__ void householder(const PqrArgs &g, PqrSm &sm, int w, unsigned &ep) {
  const int tid = otid(), lane = tid & 63, wid = tid >> 6;
  const int row = w * PT + tid;
  double a[32];
  load_row(g, row, a);
  double(*red)[32] = reinterpret_cast<double(*)[32]>(&sm.Gs[0][0]);
  double *fpart = g.part + int64_t(g.nw) * 1024;
  auto step = [&](auto jc) {
    constexpr int j = decltype(jc)::value;
    double d[32];
    const double x = (row > j) ? a[j] : 0.0;  // rows >= m hold zeros
#pragma unroll
    for (int l = 0; l < 32; ++l) d[l] = x * a[l];
    const double s = tg::lanes::reduce_scatter32(d, lane);
    if ((lane & 1) == 0) red[wid][tg::lanes::rs_col(lane)] = s;
    __syncthreads();
    if (tid < 32)
      st_sc1(fpart + (int64_t(j & 1) * g.nw + w) * 32 + tid,
             (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]));
    if (w == 0 && tid == j) {
#pragma unroll
      for (int l = 0; l < 32; ++l) st_sc1(g.bc + BC_PROW + (j & 1) * 32 + l, a[l]);
    }
    grid_bar(g, ep);
    if (tid < 32) {
      constexpr int NB = 32;
      double v[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b)
        v[b] = (b < g.nw) ? ld_sc1(fpart + (int64_t(j & 1) * g.nw + b) * 32 + tid) : 0.0;
      double acc = 0.0;
#pragma unroll
      for (int b = 0; b < NB; ++b) acc += v[b];
      sm.dsum[tid] = acc;
      sm.prow[tid] = ld_sc1(g.bc + BC_PROW + (j & 1) * 32 + tid);
    }
    __syncthreads();
    const double sig = sm.dsum[j], alpha = sm.prow[j];
    double tau = 0.0, scal = 0.0, beta = alpha;
    if (sig != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sig), alpha);
      tau = (beta - alpha) / beta;
      scal = 1.0 / (alpha - beta);
    }
    const double v = a[j] * scal;
    const double tv = row > j ? tau * v : (row == j ? tau : 0.0);
    a[j] = row > j ? v : (row == j ? beta : a[j]);
#pragma unroll
    for (int l = j + 1; l < 32; ++l) a[l] = fma(-tv, fma(scal, sm.dsum[l], sm.prow[l]), a[l]);
    if (w == 0) {
      if (tid < j) sm.Cq[tid][j] = fma(scal, sm.dsum[tid], sm.prow[tid]);  // (Y^T v_j)_tid
      if (tid == 0) sm.taus[j] = tau;
    }
  };
  [&]<int... J>(std::integer_sequence<int, J...>) {
    (step(std::integral_constant<int, J>{}), ...);
  }(std::make_integer_sequence<int, SB_B>{});
  __syncthreads();
  if (w == 0 && tid < 32) {
    // T (dlarft forward columnwise), row tid; R rows of the band block
    double trow[32];
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) {
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < jj; ++c) acc = fma(trow[c], sm.Cq[c][jj], acc);
      const double tj = sm.taus[jj];
      trow[jj] = (tid < jj) ? -tj * acc : (tid == jj ? tj : 0.0);
    }
#pragma unroll
    for (int l = 0; l < 32; ++l) {
      st_sc1(g.bc + BC_T + tid * 32 + l, trow[l]);
      g.T[tid * 32 + l] = trow[l];
    }
    if (tid < g.m) {
#pragma unroll
      for (int l = 0; l < 32; ++l) {
        const double rv = (l >= tid) ? a[l] : 0.0;
        g.A[(g.r0 + int64_t(tid)) * g.lda + g.p + l] = rv;
        g.A[(g.p + int64_t(l)) * g.lda + g.r0 + tid] = rv;
      }
    }
  }
  if (w == 0 && tid == 0)
    tg::ctl_record(g.cnt + 1, unsigned(DEC_FALLBACK * 16));
  grid_bar(g, ep);
  {
    double t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = ld_sc1(g.bc + BC_T + tid + PT * u);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + PT * u;
      sm.Tm[e >> 5][e & 31] = t[u];
    }
    __syncthreads();
  }
  if (row < g.m) {
    double y[32];
#pragma unroll
    for (int l = 0; l < 32; ++l) y[l] = (row > l) ? a[l] : (row == l ? 1.0 : 0.0);
    double2 *yo = reinterpret_cast<double2 *>(g.Y + int64_t(row) * SB_B);
    double2 *to = reinterpret_cast<double2 *>(g.YT + int64_t(row) * SB_B);
#pragma unroll
    for (int c = 0; c < 32; c += 2) {
      double t0 = 0.0, t1 = 0.0;
#pragma unroll
      for (int l = 0; l <= c + 1; ++l) {
        if (l <= c) t0 = fma(y[l], sm.Tm[l][c], t0);
        t1 = fma(y[l], sm.Tm[l][c + 1], t1);
      }
      yo[c / 2] = make_double2(y[c], y[c + 1]);
      to[c / 2] = make_double2(t0, t1);
    }
    if (row >= SB_B) {
      double *ad = g.A + (g.r0 + int64_t(row)) * g.lda + g.p;
#pragma unroll
      for (int l = 0; l < 32; ++l) ad[l] = 0.0;
#pragma unroll
      for (int l = 0; l < 32; ++l) g.A[(g.p + int64_t(l)) * g.lda + g.r0 + row] = 0.0;
    }
  }
}

// Out-of-line phases (state in s_pq).  Phase 1: this workgroup's Gram partial.
__device__ __forceinline__ void ph_gram(int w) { gram_publish(s_pq.ga, s_pq, w); }

__device__ __forceinline__ void ph_bar(unsigned ep) {
  unsigned e = ep - 1;
  grid_bar(s_pq.ga, e);
}

// Workgroup 0 after Gram pass `npass`: sum, Cholesky, decision; on accept the
// Householder reconstruction and [M1 | M1 T]; publishes what the other
// workgroups need.  Returns the decision.
__device__ __forceinline__ int ph_decide(int npass) {
  PqrSm &sm = s_pq;
  const PqrArgs &g = sm.ga;
  const int tid = otid(), lane = tid & 63, wid = tid >> 6;
  [[maybe_unused]] const int dk = npass == 1 ? 0 : 8;
  DBG_STAMP(dk + 0)
  gram_reduce(g, sm);
  __syncthreads();
  DBG_STAMP(dk + 1)
  if (wid == 0) {
    double delta = 0.0;
    if (npass >= 2) {
      for (int e = lane; e < 1024; e += 64)
        delta = fmax(delta, fabs(sm.Gs[e >> 5][e & 31] - ((e >> 5) == (e & 31) ? 1.0 : 0.0)));
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) delta = fmax(delta, __shfl_xor(delta, off));
    }
    if (lane == 0) sm.delta = delta;
  }
  __syncthreads();
  // G within 1e-5 of I (the usual second pass): its Cholesky factor by the
  // series R = I + F, F = Phi(E - F^T F), E = G - I (Phi: strict upper + half
  // diagonal), two terms: error O(|E|^3) <= 1e-15, all 32 x 32 products on
  // MFMA instead of a 32-step pivot chain.
  const bool series = npass >= 2 && sm.delta <= SERIES_TOL;
  if (series) {
    for (int e = tid; e < 1024; e += PT) {
      const int i2 = e >> 5, j2 = e & 31;
      const double ev = sm.Gs[i2][j2] - (i2 == j2 ? 1.0 : 0.0);
      const double f = (i2 < j2) ? ev : (i2 == j2 ? 0.5 * ev : 0.0);
      sm.RgI[i2][j2] = f;  // F1
      sm.Ut[j2][i2] = f;   // F1^T
    }
    __syncthreads();
    mm32<33, 33, 33>(&sm.Cq[0][0], &sm.Ut[0][0], &sm.RgI[0][0], nullptr);  // F1^T F1
    __syncthreads();
    for (int e = tid; e < 1024; e += PT) {
      const int i2 = e >> 5, j2 = e & 31;
      const double ev = sm.Gs[i2][j2] - (i2 == j2 ? 1.0 : 0.0) - sm.Cq[i2][j2];
      const double f = (i2 < j2) ? ev : (i2 == j2 ? 0.5 * ev : 0.0);
      sm.Lt[i2][j2] = (i2 == j2 ? 1.0 : 0.0) + f;  // R = L^T (upper)
      if (i2 == j2) sm.rinv[i2] = rcp_nr(1.0 + f);
    }
    if (tid == 0) sm.dec = DEC_ACCEPT;
  } else if (wid == 0) {
    const double delta = sm.delta;
    double mr = 0.0;
    bool ok = chol32_ool(0.0, mr);
    if (npass == 1 && (!ok || mr < 1e-12)) {
      double tr = 0.0;
      for (int c = 0; c < 32; ++c) tr += sm.Gs[c][c];
      const double shift = 11.0 * (double(g.m) * 32.0 + 32.0 * 33.0) * (0.5 * DBL_EPSILON) * tr;
#ifdef TG_PQR_DBG
      if (lane == 0) g_pq_dbg[30] += 1;
#endif
      ok = chol32_ool(shift, mr);
    }
    const int d = !ok ? DEC_FALLBACK
                      : (npass >= 2 && delta < 0.1) ? DEC_ACCEPT
                                                    : (npass >= NPASS ? DEC_FALLBACK : DEC_CONTINUE);
    if (lane == 0) sm.dec = d;
  }
  __syncthreads();
  DBG_STAMP(dk + 2)
  const int d = sm.dec;
  if (d != DEC_FALLBACK) {
    // Ra <- L^T Ra (upper triangular product; Lt is L^T), via RgI
    if (npass == 1) {
      for (int e = tid; e < 1024; e += PT) sm.Ra[e >> 5][e & 31] = sm.Lt[e >> 5][e & 31];
    } else {
      mm32<33, 33, 33>(&sm.RgI[0][0], &sm.Lt[0][0], &sm.Ra[0][0], nullptr);
      __syncthreads();
      for (int e = tid; e < 1024; e += PT) sm.Ra[e >> 5][e & 31] = sm.RgI[e >> 5][e & 31];
    }
    __syncthreads();
  }
  DBG_STAMP(dk + 3)
  if (d == DEC_ACCEPT) {
    DBG_STAMP(dk + 4)
    hr_top_ool();
    DBG_STAMP(dk + 5)
    for (int e = tid; e < 2048; e += PT) st_sc1(g.bc + BC_MB + e, sm.MB[e >> 6][e & 63]);
    for (int e = tid; e < 1024; e += PT) g.T[e] = sm.Tm[e >> 5][e & 31];
  }
  if (d == DEC_CONTINUE) {
    for (int e = tid; e < 1024; e += PT) st_sc1(g.bc + BC_L + e, sm.Lt[e >> 5][e & 31]);
    if (tid < 32) st_sc1(g.bc + BC_RINV + tid, sm.rinv[tid]);
  }
  DBG_STAMP(dk + 6)
  if (tid == 0) {
    st_sc1(g.bc + BC_DEC, double(d));
    tg::ctl_record(g.cnt + 1, unsigned(d * 16 + npass));
  }
  return d;
}

// Every workgroup but 0: this pass's L; then Q <- Q L^-T on the LDS rows.
__device__ __forceinline__ void ph_apply(int w) {
  PqrSm &sm = s_pq;
  const PqrArgs &g = sm.ga;
  const int tid = otid();
  if (w != 0) {
    double t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = ld_sc1(g.bc + BC_L + tid + PT * u);
    const double ri = tid < 32 ? ld_sc1(g.bc + BC_RINV + tid) : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + PT * u;
      sm.Lt[e >> 5][e & 31] = t[u];
    }
    if (tid < 32) sm.rinv[tid] = ri;
    __syncthreads();
  }
  double x[32];
  row_from_lds(&sm.Xs[tid][0], x);
  trsm_row(x, sm.Lt, sm.rinv);
  row_to_lds(&sm.Xs[tid][0], x);
  __syncthreads();
}

__device__ __forceinline__ void ph_final(int w) {
  PqrSm &sm = s_pq;
  const PqrArgs &g = sm.ga;
  const int tid = otid();
  if (w != 0) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = ld_sc1(g.bc + BC_MB + tid + PT * u);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + PT * u;
      sm.MB[e >> 6][e & 63] = t[u];
    }
    __syncthreads();
  }
  final_rows(g, sm, w);
}

__device__ __noinline__ void ph_householder(int w, unsigned ep) {
  unsigned e = ep;
  householder(s_pq.ga, s_pq, w, e);
}

__global__ __launch_bounds__(PT) void pqr_kernel(PqrArgs ga) {
  PqrSm &sm = s_pq;
  if (blockIdx.x % ga.wstride != 0) return;  // workers: one per XCD count (one XCD under round-robin)
  const int w = blockIdx.x / ga.wstride;
  const int tid = otid();
  if (tid == 0) sm.ga = ga;
  unsigned ep = 0;
  int nst = 0;
  auto stamp = [&]() {
    if (ga.stats && w == 0 && tid == 0 && nst < 15) ga.stats[nst] = __builtin_amdgcn_s_memrealtime();
    ++nst;
  };
  stamp();
  int dec = (ga.m < FB_MIN_M || ga.force_fb) ? DEC_FALLBACK : DEC_CONTINUE;
  if (dec == DEC_CONTINUE) {
    double x[32];
    load_row(ga, w * PT + tid, x);
    row_to_lds(&sm.Xs[tid][0], x);
  }
  __syncthreads();
  int npass = 0;
  while (dec == DEC_CONTINUE) {
    ph_gram(w);
    stamp();
    ph_bar(++ep);
    stamp();
    ++npass;
    if (w == 0) ph_decide(npass);
    stamp();
    ph_bar(++ep);
    stamp();
    dec = int(ld_sc1(ga.bc + BC_DEC));
    if (dec == DEC_ACCEPT) {
      ph_final(w);
      stamp();
      return;
    }
    if (dec == DEC_CONTINUE) ph_apply(w);
  }
  ph_householder(w, ep);
}

}  // namespace

namespace tg {

// One row per thread, 256 rows per workgroup, every workgroup resident (one
// per CU: the row block and the factor tiles fill its LDS): panels of up to
// 256 x 256 rows (n <= 65,568), the largest down_proj (n = 28,672) needs 112.
// The workers meet at grid barriers, so all cdiv(m, PT) of them must be
// resident at once: the single-level path is only taken when they fit the
// device's CUs at the kernel's occupancy (a smaller device or partition falls
// back to the TSQR band reduction instead of stalling into the spin timeout).
static int pqr_resident_workers() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cached[dev] == 0) {
    int ncu = 0, occ = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pqr_kernel, PT, 0) != hipSuccess)
      occ = 0;
    cached[dev] = std::max(0, ncu) * std::max(0, occ);
    if (cached[dev] == 0) cached[dev] = -1;
  }
  return std::max(0, cached[dev]);
}

int pqr_rows_per_thread(int m) {
  return m <= PQR_NWMAX * PT && cdiv(m, PT) <= pqr_resident_workers() ? 1 : 0;
}

hipError_t panel_qr(hipStream_t st, double *A, int lda, int p, int r0, int m, double *Y,
                    double *YT, double *T, double *part, double *bc, unsigned *cnt,
                    unsigned *tmo) {
  if (m < 1 || pqr_rows_per_thread(m) == 0) return hipErrorInvalidValue;
  PqrArgs g{};
  g.A = A;
  g.lda = lda;
  g.p = p;
  g.r0 = r0;
  g.m = m;
  g.nw = cdiv(m, PT);
  g.Y = Y;
  g.YT = YT;
  g.T = T;
  g.part = part;
  g.bc = bc;
  g.cnt = cnt;
  g.tmo = tmo;
  static const unsigned long long tmo_ticks = spin_timeout_ticks("TG_PQR_TIMEOUT_TICKS");
  g.timeout = tmo_ticks;
  {
    const char *fb = getenv("TG_PQR_FALLBACK");
    g.force_fb = (fb && fb[0] == '1') ? 1 : 0;
  }
  static unsigned long long *stats = nullptr;
  static int nstat = 0;
  static double acc[16] = {0};
  if (getenv("TG_PQR_STATS")) {
    if (!stats) {
      (void)hipMalloc(&stats, 16 * sizeof(unsigned long long));
      atexit([] {
        if (nstat == 0) return;
        fprintf(stderr, "pqr phases (us, mean of %d accepted 2-pass panels):", nstat);
        for (int i = 1; i < 10; ++i) fprintf(stderr, " %.2f", acc[i] / nstat / 100.0);
        fprintf(stderr, "\n");
      });
    }
    (void)hipMemsetAsync(stats, 0, 16 * sizeof(unsigned long long), st);
    g.stats = stats;
  }
  // 2 Gram passes + the row solve and the final [Y | YT] product: ~10 m 32^2 flops
  auto tok = prof_begin(st, PROF_TSQR, 8.0 * m * SB_B * 3, 10.0 * m * SB_B * SB_B);
  // up to 32 workers share one XCD (launched x8, blockIdx % 8 == 0: one XCD
  // under round-robin dispatch -- speed only: the hand-offs are sc1 stores and
  // loads, correct across XCDs); more are spread over the chip
  const XcdInfo xi = xcd_info();
  g.wstride = g.nw <= xi.cus_per_xcd ? xi.xcds : 1;
  hipLaunchKernelGGL(pqr_kernel, dim3(g.wstride * g.nw), dim3(PT), 0, st, g);
  prof_end(st, tok);
  if (g.stats) {
    unsigned long long h[16];
    (void)hipMemcpyAsync(h, g.stats, sizeof(h), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    if (h[9] != 0 && h[10] == 0) {
      for (int i = 1; i < 10; ++i) acc[i] += double(h[i] - h[i - 1]);
      ++nstat;
    }
#ifdef TG_PQR_DBG
    static int ndbg = 0;
    if (++ndbg == 250) {
      unsigned long long d[64];
      (void)hipMemcpyFromSymbol(d, HIP_SYMBOL(g_pq_dbg), sizeof(d));
      fprintf(stderr, "pqr decide sub-phases (us, sums over launches): p1 reduce %.1f chol %.1f ra %.1f pub %.1f | p2 reduce %.1f chol %.1f ra %.1f cq %.1f hr %.1f pub %.1f\n",
              (d[1] - d[0]) / 100.0, (d[2] - d[1]) / 100.0, (d[3] - d[2]) / 100.0, (d[6] - d[3]) / 100.0,
              (d[9] - d[8]) / 100.0, (d[10] - d[9]) / 100.0, (d[11] - d[10]) / 100.0,
              (d[12] - d[11]) / 100.0, (d[13] - d[12]) / 100.0, (d[14] - d[13]) / 100.0);
      fprintf(stderr, "  shifted first passes: %llu; chol32: loop %.1f tail %.1f (sums)\n", d[30],
              (d[25] - d[24]) / 100.0, (d[26] - d[25]) / 100.0);
      fprintf(stderr, "  hr: LU||RgI %.1f  T||UI||R %.1f  M1+Y1T %.1f  (sums); LU %.1f RgI %.1f\n",
              (d[17] - d[16]) / 100.0, (d[18] - d[17]) / 100.0, (d[19] - d[18]) / 100.0,
              (d[20] - d[16]) / 100.0, (d[21] - d[16]) / 100.0);
    }
#endif
  }
  return hipGetLastError();
}

}  // namespace tg
