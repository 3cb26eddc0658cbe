// Stage 1 of the two-stage symmetric eigensolver: full -> band reduction
// (sy2sb) with TSQR panel factorisations, and its back-transformation.
#pragma once
#include <algorithm>
#include <type_traits>
#include <vector>

#include "common.h"

namespace tg {

constexpr int SB_B = 32;    // half-bandwidth of the band matrix (= panel width)
constexpr int SB_C = 256;   // TSQR leaf height (last leaf of a level absorbs < SB_C rows)
constexpr int SB_LV = 6;    // max TSQR levels
constexpr int PQR_NWMAX = 256;       // panel-QR workgroups (pqr.hip): 256 rows each, one per CU
constexpr int PQR_BC_DOUBLES = 8192; // panel-QR broadcast block

// One TSQR level of one panel: `rows` stacked rows split in `nc` chunks.
struct SbLevel {
  int rows, nc;
  size_t yoff, toff;  // offsets of this level's Y (rows x 32) and T (nc x 32 x 32)
};
struct SbPanel {
  int p, r0, m, nl;
  SbLevel L[SB_LV];
};

// single: one compact-WY block per panel (Y m x 32, one T; pqr.hip panel
// QR), the default while the panel QR takes the first panel's rows
// (pqr_rows_per_thread); otherwise (or TG_SB_TSQR=1) the TSQR tree of leaves
// of SB_C rows.  A panel's levels are then one level of one chunk
// of m rows (P.L[0] = {m, 1, ...}).
struct SbPlan {
  std::vector<SbPanel> panels;
  size_t ytotal = 0, ttotal = 0;
  int ncmax = 1;
  bool single = false;
  explicit SbPlan(int n);
};

// Device buffers (carved by the caller from the eigensolver workspace).
struct SbBufs {
  double *Y, *T;          // reflector storage for all panels (persist until back-transform)
  double *YT, *X, *G, *M; // per-panel temporaries
  double *YTl[SB_LV];     // Y T of TSQR levels >= 1 (computed on a side stream)
  double *R[2];           // TSQR R stacks (ping-pong between levels)
  double *Gr, *U;         // gathered rows / symmetric update (ncmax*32 x n)
  double *Xs;             // gathered rows of X (ncmax*32 x ncmax*32)
  double *Zg, *P, *Mz;    // back-transformation temporaries (ncmax*32 x k)
  // stage 2 (bulge.hip)
  double *Bst;            // band storage n x 2b
  double *V2;             // bulge-chasing reflector records (tau, v_1..v_{b-1}), (n-2) x smax x b
  double *T2;             // Q2 block T factors
  unsigned *prog;         // pipeline progress per sweep group
  // panel QR (pqr.hip): partials, broadcast block, per-panel control words
  double *pq_part, *pq_bc;
  unsigned *pq_ctl;       // [0] timeout flag, [1] M-kernel ticket, [4 + 4 i] panel i counters
  unsigned *xm_tick;      // X / M kernel tickets (band.hip xm_kernel), xm_tick_words(n)
  double *xm_xpart;       // X / M K-split partial X blocks, xm_xpart_doubles(n)
};

int pqr_rows_per_thread(int m);
// Panel A[r0:r0+m, p:p+32] -> Y (m x 32), YT = Y T, T (32 x 32); writes
// [R; 0] and its transpose into A.  cnt: 2 words zeroed before the launch.
hipError_t panel_qr(hipStream_t st, double *A, int lda, int p, int r0, int m, double *Y,
                    double *YT, double *T, double *part, double *bc, unsigned *cnt,
                    unsigned *tmo);

int sb_smax(int n);
size_t sb2st_prog_words(int n);
size_t sb2st_t2_count(int n);

// control words: 4 + 4 per panel, padded to a multiple of 16 bytes
inline size_t pq_ctl_words(int n) { return 4 + 4 * size_t(std::max(1, n / SB_B + 1)); }
// X / M kernel: one ticket per group of 32 row blocks of 16 rows, + 1
// X / M control words: group tickets [0, n / 256 + 7), the fused-W flag at
// n / 256 + 7, the K-split column-block tickets from n / 256 + 8 (n / 16 + 2)
inline size_t xm_mflag_off(int n) { return size_t(n) / 256 + 7; }
inline size_t xm_cbt_off(int n) { return size_t(n) / 256 + 8; }
inline size_t xm_tick_words(int n) { return xm_cbt_off(n) + size_t(n) / 16 + 2; }
// K-split partial X blocks: at most 8 splits of every 32-row block
inline size_t xm_xpart_doubles(int n) { return 8 * (size_t(n) + 32) * 32; }

template <class A>
void sb_layout(A &ar, int n, int kmax, const SbPlan &pl, SbBufs *bp) {
  SbBufs d{};
  SbBufs &b = bp ? *bp : d;
  const size_t w = size_t(pl.ncmax) * SB_B;
  auto take = [&](double *&dst, size_t cnt) {
    if constexpr (std::is_same_v<A, Arena>) dst = ar.template take<double>(cnt);
    else ar.template take<double>(cnt);
  };
  take(b.Y, pl.ytotal + 1);
  take(b.T, pl.ttotal + 1);
  take(b.YT, size_t(n) * SB_B);
  for (int l = 1; l < SB_LV; ++l) take(b.YTl[l], w * SB_B);
  take(b.X, size_t(n) * w);
  take(b.G, w * w);
  take(b.M, w * w);
  take(b.R[0], w * SB_B);
  take(b.R[1], w * SB_B);
  take(b.Gr, w * n);
  // X partials: one m x 32 slab per 256-row block of A22 (TSQR path); the
  // single path's X / M partials (n / 16 + n / 256 blocks of 1024; with the
  // panel-pair products n / 32 + n / 1024 blocks of 5 x 1024) fit too
  take(b.U, std::max({w * n, (size_t(n) / 16 + size_t(n) / 256 + 2) * 1024,
                      (size_t(n) / 32 + size_t(n) / 1024 + 2) * 5 * 1024}));
  take(b.Xs, w * w);
  take(b.Zg, w * kmax);
  take(b.P, w * kmax);
  take(b.Mz, w * kmax);
  const size_t nsw = size_t(std::max(1, n - 2)), smax = size_t(sb_smax(n));
  take(b.Bst, size_t(n) * 2 * SB_B);
  take(b.V2, nsw * smax * SB_B);
  take(b.T2, sb2st_t2_count(n));
  // per-group progress + 4 control words (XCD, group queue, stall flag)
  if constexpr (std::is_same_v<A, Arena>) b.prog = ar.template take<unsigned>(sb2st_prog_words(n));
  else ar.template take<unsigned>(sb2st_prog_words(n));
  // partials: panel QR (2 per worker), X row blocks, M (one per 128 rows)
  const size_t npart = std::max<size_t>(std::max<size_t>(2 * PQR_NWMAX + 2, size_t(n) / SB_C + 2),
                                        size_t(n) / 128 + 2) * 1024;
  take(b.pq_part, npart);
  take(b.pq_bc, PQR_BC_DOUBLES);
  if constexpr (std::is_same_v<A, Arena>) b.pq_ctl = ar.template take<unsigned>(pq_ctl_words(n));
  else ar.template take<unsigned>(pq_ctl_words(n));
  if constexpr (std::is_same_v<A, Arena>) b.xm_tick = ar.template take<unsigned>(xm_tick_words(n));
  else ar.template take<unsigned>(xm_tick_words(n));
  take(b.xm_xpart, xm_xpart_doubles(n));
}

// A (n x n symmetric, full storage, lda) -> band matrix of half-bandwidth
// SB_B in place (full storage, zeros outside the band); reflectors in bufs.
hipError_t sy2sb(hipStream_t st, double *A, int lda, int n, const SbPlan &pl, const SbBufs &b);
// Single-level plans: reads the panel-QR timeout flag (one D2H copy + sync).
hipError_t sy2sb_timed_out(hipStream_t st, const SbPlan &pl, const SbBufs &b, bool *tmo);
// Band (in A after sy2sb) -> tridiagonal (d, e) by bulge chasing.
// A stalled hand-off (a wait beyond the timeout, TG_BULGE_TIMEOUT_TICKS of the
// 100 MHz clock, default 2 s) poisons d and e with NaN; the stall flag stays
// in prog and is read back by sb2st_stalled (one D2H copy + stream sync).
hipError_t sb2st(hipStream_t st, const double *A, int lda, int n, double *Bst, double *V2,
                 unsigned *prog, double *d, double *e);
// *broken: the tridiagonal guard fired (trace / Frobenius norm of the band not
// preserved by the chase; d and e poisoned).  TG_TRI_GUARD_PRINT=1 prints the
// guard's residuals.
hipError_t sb2st_stalled(hipStream_t st, int n, const unsigned *prog, bool *stalled,
                         bool *broken = nullptr);
// Z (n x k row-major) <- Q2 Z.
hipError_t sb_apply_q2(hipStream_t st, int n, double *Z, int k, const double *V2,
                       double *T2);
// Q2 block T factors only (T2), for sb_apply_few.
hipError_t sb_q2_tfactors(hipStream_t st, int n, const double *V2, double *T2);
// side stream of the band reduction: fork after the work queued on st, join back into st
hipError_t side_fork(hipStream_t st, hipStream_t *side);
hipError_t side_join(hipStream_t st);
// Z (n x k row-major) <- Q1 Q2 Z with Z resident on chip (backtr.hip): k <= 32,
// or up to 128 in 16-column slabs when sb_apply_few_ok; T2 must hold the Q2 T
// factors; dev: sb_apply_few_scratch bytes of device scratch.  Syncs the
// stream (reads the barrier timeout flag).
bool sb_apply_few_ok(const SbPlan &pl, int n, int k);
size_t sb_apply_few_scratch(const SbPlan &pl, int n, int k);
hipError_t sb_apply_few(hipStream_t st, int n, double *Z, int k, const SbPlan &pl,
                        const SbBufs &b, void *dev, bool *timed_out);
// Z (n x k row-major) <- Q1 Z.
hipError_t sb_apply_q1(hipStream_t st, int n, double *Z, int k, const SbPlan &pl,
                       const SbBufs &b);

}  // namespace tg
