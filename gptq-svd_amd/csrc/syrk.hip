// Hessian accumulation H += X^T X (A1, gptq_utils.py:218-223 `H.addmm_(x.T, x)`
// with x cast to float64) for 16-bit activations (fp16 / bf16, what the
// harness hooks hand over), FP64 MFMA (v_mfma_f64_16x16x4_f64) on gfx950.
//
// Work: rows x n^2 / 2 FMAs on the lower 128 x 128 tiles (mirrored).  The
// inputs are exact in FP64, every product is formed and summed in FP64.
//
// Layout and schedule (two kernels, same decomposition):
//  * a workgroup (8 waves as 2 x 4, 64 x 32 per wave = 4 x 2 MFMA blocks;
//    two workgroups per CU) owns one 128 x 128 tile of H at a time and
//    streams the two 128-column strips of X it needs (tile row I, tile
//    column J) in slabs of rows, global loads 16 B per lane (8 columns of
//    one row) one slab ahead;
//  * default, `syrk64l_kernel`: each staged element is converted to FP64
//    once and the slab (16 rows) is kept FP64 in LDS, pieces permuted per row
//    for conflict-free writes and MFMA operand reads; 68.4 TF/s at n =
//    12,288, 65.4 at 4096 (`tools/syrk_time.py`);
//  * `syrk16_kernel` (TG_SYRK_LDS64=0): X stays 16-bit in LDS, column
//    major, 32-row sub-slabs whose 16-B chunks are XOR-swizzled; one 16-B
//    read holds a lane's operand for 8 MFMA steps and every wave converts
//    its operands in registers (each A value in 4 waves, each B in 2):
//    63.5 / 61.0 TF/s;
//  * a persistent grid (CUs x 2 workgroups) takes work units from an atomic
//    queue: whole tiles first, then the last round's tiles cut into NC = 16
//    chunks of K; a whole tile is added to H directly, a chunk leaves a
//    partial tile in the workspace and `syrk_fixup_kernel` adds a tile's
//    chunks to H in chunk order -- the decomposition is static, so H is
//    deterministic whichever workgroup ran which unit.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "../../include/truncgptq.h"
#include "common.h"

namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef double doublex2 __attribute__((ext_vector_type(2)));

constexpr int BT = 128;  // tile edge
constexpr int KC = 32;   // rows of X per sub-slab (one LDS image)
constexpr int NSUB = 2;  // sub-slabs per slab: one barrier per NSUB * KC rows
constexpr int NT = 512;  // threads per workgroup

template <bool BF16>
__device__ inline double h2d(unsigned bits16) {
  if (BF16) return double(__uint_as_float(bits16 << 16));
  return double(float(__builtin_bit_cast(_Float16, (unsigned short)bits16)));
}

// column c's 16-B chunk q (rows 8q..8q+7 of the slab) sits at chunk q ^ swz(c)
__device__ inline int swz(int c) { return (-(c >> 2)) & 3; }

struct SyrkArgs {
  const unsigned short *X;  // rows x n, 16-bit
  int64_t ldx;
  int64_t rows;
  int n;
  double *H;
  int64_t ldh;
  int T;          // lower tiles
  int NS;         // slabs (NSUB * KC rows) per tile
  int head;       // tiles 0 .. head - 1: one unit each (whole K), added to H directly
  int Tt;         // tiles head .. T - 1: NC units each (K in chunks of CK slabs)
  int NC, CK;
  int U;          // units = head + Tt * NC
  double *piece;  // Tt x NC x BT x BT partial tiles (chunk c of tail tile i at i * NC + c)
  unsigned *next; // unit queue head (zeroed before the launch)
  unsigned long long *stamps;  // TG_SYRK_STAMPS: per workgroup {start, end, xcc} (else null)
};

__device__ inline void tile_of(int b, int &I, int &J) {
  I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  J = b - I * (I + 1) / 2;
}

// Global -> registers: thread t stages strip t >> 8 (0 = tile row I's
// columns, 1 = tile column J's), rows 2rp, 2rp + 1 of the slab (rp =
// (t >> 4) & 15), columns cg * 8 .. cg * 8 + 7 (cg = t & 15).
struct Stage {
  u32x4 v[2];  // [row]
  bool ok[2];  // out-of-range rows / columns: a clamped load, zeroed at the store
               // (a select right after the load would wait for it there)
  __device__ inline void load(const SyrkArgs &a, int c0A, int c0B, int64_t k0) {
    const int t = threadIdx.x, cg = t & 15, rp = (t >> 4) & 15, sp = t >> 8;
    const int c = (sp == 0 ? c0A : c0B) + cg * 8;
    const bool cok = c < a.n;  // n % 8 == 0: a chunk is all in or all out
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t k = k0 + 2 * rp + r;
      ok[r] = cok && k < a.rows;
      const int64_t kc = ok[r] ? k : 0;
      const int cc = ok[r] ? c : 0;
      v[r] = *reinterpret_cast<const u32x4 *>(a.X + kc * a.ldx + cc);
    }
  }
  // registers -> LDS: column c, rows 2rp, 2rp+1 as one 4-byte word
  __device__ inline void store(unsigned short *SA, unsigned short *SB) const {
    const int t = threadIdx.x, cg = t & 15, rp = (t >> 4) & 15, sp = t >> 8;
    const int k = 2 * rp, q = k >> 3, kin = k & 7;
    unsigned short *S = sp == 0 ? SA : SB;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      const unsigned lo = ok[0] ? (v[0][j >> 1] >> ((j & 1) * 16)) & 0xffffu : 0u;
      const unsigned hi = ok[1] ? (v[1][j >> 1] >> ((j & 1) * 16)) & 0xffffu : 0u;
      *reinterpret_cast<unsigned *>(S + c * KC + ((q ^ swz(c)) << 3) + kin) = lo | (hi << 16);
    }
  }
};

// Wave w of the 8 owns rows wm * 64 .. + 63 (4 MFMA blocks) and columns
// wn * 32 .. + 31 (2 blocks) of the tile, wm = w >> 2, wn = w & 3.
constexpr int FI = 4, FJ = 2;

// A wave's operands of half a slab: for each of its 4 + 2 MFMA blocks, 4
// rows of its lane group (rows 8g + 4h .. + 3, one ds_read_b64 each).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
struct Frags {
  u32x2 a[FI], b[FJ];
  __device__ inline void read(const unsigned short *SA, const unsigned short *SB, int h) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 2, wn = w & 3, g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int c = wm * 64 + i * 16 + r;
      a[i] = *reinterpret_cast<const u32x2 *>(SA + c * KC + ((g ^ swz(c)) << 3) + 4 * h);
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int c = wn * 32 + j * 16 + r;
      b[j] = *reinterpret_cast<const u32x2 *>(SB + c * KC + ((g ^ swz(c)) << 3) + 4 * h);
    }
  }
};

template <bool BF16>
__device__ inline void half_slab_mfma(const Frags &f, doublex4 (&acc)[FI][FJ]) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    double av[FI], bv[FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i) av[i] = h2d<BF16>((f.a[i][kk >> 1] >> ((kk & 1) * 16)) & 0xffffu);
#pragma unroll
    for (int j = 0; j < FJ; ++j) bv[j] = h2d<BF16>((f.b[j][kk >> 1] >> ((kk & 1) * 16)) & 0xffffu);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
  }
}

// Two workgroups of eight waves per CU: four waves per SIMD, two of which
// keep the f64 MFMA pipe full (one wave alone issues an f64 MFMA only every
// ~128 cycles: tools/mfma64_peak.hip), while the others wait at their
// workgroup's barrier or on LDS.
template <bool BF16>
__global__ __launch_bounds__(NT, 4) void syrk16_kernel(SyrkArgs a) {
  // [stage][sub-slab][strip]
  __shared__ __attribute__((aligned(16))) unsigned short S[2][NSUB][2][BT * KC];
  __shared__ unsigned s_unit;
  const int g = blockIdx.x;
  if (a.stamps && threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    a.stamps[3 * g] = __builtin_amdgcn_s_memrealtime();
    a.stamps[3 * g + 2] = x;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wm = wv >> 2, wn = wv & 3;
  while (true) {
    __syncthreads();  // s_unit and the LDS stages of the previous unit are free
    if (threadIdx.x == 0) s_unit = atomicAdd(a.next, 1u);
    __syncthreads();
    const int u = int(s_unit);
    if (u >= a.U) break;
    int t, s0, s1, slot = -1;
    if (u < a.head) {
      t = u, s0 = 0, s1 = a.NS;
    } else {  // tail: chunk-major, so units running together share their rows of X
      const int v = u - a.head, c = v / a.Tt, i = v - c * a.Tt;
      t = a.head + i;
      s0 = c * a.CK;
      s1 = min(a.NS, s0 + a.CK);
      slot = i * a.NC + c;
    }
    int I, J;
    tile_of(t, I, J);
    const int tm = I * BT, tn = J * BT;
    doublex4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
    // slab s = NSUB sub-slabs of KC rows; the next slab's sub-slab b goes
    // from registers to the other stage right after this slab's sub-slab b
    // has been consumed, and its global loads for sub-slab b + 1 follow (one
    // sub-slab of registers in flight, a sub-slab of MFMAs to cover them)
    const int64_t R0 = int64_t(NSUB) * KC;
    Stage st;
#pragma unroll
    for (int b = 0; b < NSUB; ++b) {
      st.load(a, tm, tn, int64_t(s0) * R0 + b * KC);
      st.store(S[0][b][0], S[0][b][1]);
    }
    if (s0 + 1 < s1) st.load(a, tm, tn, int64_t(s0 + 1) * R0);
    __syncthreads();
    // slabs in pairs, so the stage of each is a compile-time index (LDS
    // addresses become immediates instead of registers)
    auto slab = [&]<int CUR>(std::integral_constant<int, CUR>, int s) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < NSUB; ++b) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          Frags f;
          f.read(S[CUR][b][0], S[CUR][b][1], h);
          half_slab_mfma<BF16>(f, acc);
        }
        if (s + 1 < s1) {
          st.store(S[CUR ^ 1][b][0], S[CUR ^ 1][b][1]);
          if (b + 1 < NSUB) st.load(a, tm, tn, int64_t(s + 1) * R0 + (b + 1) * KC);
          else if (s + 2 < s1) st.load(a, tm, tn, int64_t(s + 2) * R0);
        }
      }
      __syncthreads();
    };
    for (int s = s0; s < s1; s += 2) {
      slab(std::integral_constant<int, 0>{}, s);
      if (s + 1 < s1) slab(std::integral_constant<int, 1>{}, s + 1);
    }
    if (slot < 0) {  // H += acc on the tile, mirrored
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int gi = tm + wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int gj = tn + wn * 32 + j * 16 + (lane & 15);
            if (gi < a.n && gj < a.n) {
              double *p = a.H + int64_t(gi) * a.ldh + gj;
              const double v = *p + acc[i][j][rr];
              *p = v;
              if (I != J) a.H[int64_t(gj) * a.ldh + gi] = v;
            }
          }
    } else {  // partial tile of a tail tile's chunk
      double *P = a.piece + int64_t(slot) * (BT * BT);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int li = wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int lj = wn * 32 + j * 16 + (lane & 15);
            P[li * BT + lj] = acc[i][j][rr];
          }
    }
  }
  if (a.stamps) {
    __syncthreads();
    if (threadIdx.x == 0) a.stamps[3 * g + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// FP64-in-LDS variant (TG_SYRK_LDS64=1): every element of X is converted to
// FP64 once, by the thread that stages it, instead of once per wave that
// reads it (the 16-bit form converts each A operand in 4 waves and each B
// operand in 2: 768 conversions per row of a tile against 256).  A slab is
// 16 rows of both strips, row-major FP64 (2 x 16 x 128 x 8 B = 32 KB, two
// stages = 64 KB per workgroup, two workgroups per CU), its pieces permuted
// within each row (lpos) so that staging writes and MFMA operand reads are
// free of bank conflicts.  Same units, queue and fix-up as the
// 16-bit kernel; H agrees with it to FP64 rounding (every product is exact,
// only the grouping of rows into MFMA k-steps differs), deterministic.
constexpr int KL = 16;  // rows per slab

// Column c of slab row r: 16-B piece P = c / 2 of the row goes to piece
// P ^ ((P >> 4) & 3) ^ 8(r & 1).  The first term spreads a staging write
// (16 lanes, piece q of columns 8cg .. 8cg + 7 each) over all 64 banks; the
// second puts the odd row of a ds_read_b64 pass in the other bank half.
// Both permute pieces within aligned groups of 8, so a wave's 16 consecutive
// columns of a row still cover 32 distinct banks.
__device__ inline int lpos(int r, int c) {
  const int P = c >> 1;
  return r * BT + 2 * (P ^ ((P >> 4) & 3) ^ ((r & 1) << 3)) + (c & 1);
}

struct Stage64 {
  u32x4 v;  // 8 16-bit values: row (t >> 4) & 15, columns (t & 15) * 8 .. + 7 of strip t >> 8
  bool ok;  // rows past the end / columns past n: a clamped load, zeroed at the store
  __device__ inline void load(const SyrkArgs &a, int c0A, int c0B, int64_t k0) {
    const int t = threadIdx.x, cg = t & 15, r = (t >> 4) & 15, sp = t >> 8;
    const int c = (sp == 0 ? c0A : c0B) + cg * 8;
    const int64_t k = k0 + r;
    ok = c < a.n && k < a.rows;
    v = *reinterpret_cast<const u32x4 *>(a.X + (ok ? k : 0) * a.ldx + (ok ? c : 0));
  }
  template <bool BF16>
  __device__ inline void store(double *S) const {  // S: [strip][KL][BT]
    const int t = threadIdx.x, cg = t & 15, r = (t >> 4) & 15, sp = t >> 8;
    double *p = S + sp * (KL * BT);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned w = ok ? v[q] : 0u;
      doublex2 d{h2d<BF16>(w & 0xffffu), h2d<BF16>(w >> 16)};
      *reinterpret_cast<doublex2 *>(p + lpos(r, cg * 8 + 2 * q)) = d;
    }
  }
};

template <bool BF16>
__global__ __launch_bounds__(NT, 4) void syrk64l_kernel(SyrkArgs a) {
  __shared__ __attribute__((aligned(16))) double S[2][2 * KL * BT];  // [stage][strip][row][col]
  __shared__ unsigned s_unit;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wm = wv >> 2, wn = wv & 3, g = lane >> 4, l16 = lane & 15;
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) s_unit = atomicAdd(a.next, 1u);
    __syncthreads();
    const int u = int(s_unit);
    if (u >= a.U) break;
    int t, s0, s1, slot = -1;
    if (u < a.head) {
      t = u, s0 = 0, s1 = a.NS;
    } else {
      const int v = u - a.head, c = v / a.Tt, i = v - c * a.Tt;
      t = a.head + i;
      s0 = c * a.CK;
      s1 = min(a.NS, s0 + a.CK);
      slot = i * a.NC + c;
    }
    int I, J;
    tile_of(t, I, J);
    const int tm = I * BT, tn = J * BT;
    doublex4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
    Stage64 st;
    st.load(a, tm, tn, int64_t(s0) * KL);
    st.store<BF16>(S[0]);
    if (s0 + 1 < s1) st.load(a, tm, tn, int64_t(s0 + 1) * KL);
    __syncthreads();
    auto slab = [&]<int CUR>(std::integral_constant<int, CUR>, int s) __attribute__((always_inline)) {
      const double *SA = S[CUR], *SB = S[CUR] + KL * BT;
      // one k-step's operands at a time, a schedule barrier after its MFMAs:
      // the other three waves of the SIMD cover the read latency, and the
      // compiler cannot hoist the slab's reads (which spilled at the
      // 128-register cap of four waves per SIMD)
#pragma unroll
      for (int kk = 0; kk < KL / 4; ++kk) {
        const int r = 4 * kk + g;
        double av[FI], bv[FJ];
#pragma unroll
        for (int i = 0; i < FI; ++i) av[i] = SA[lpos(r, wm * 64 + i * 16 + l16)];
#pragma unroll
        for (int j = 0; j < FJ; ++j) bv[j] = SB[lpos(r, wn * 32 + j * 16 + l16)];
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (s + 1 < s1) {
        st.store<BF16>(S[CUR ^ 1]);
        if (s + 2 < s1) st.load(a, tm, tn, int64_t(s + 2) * KL);
      }
      __syncthreads();
    };
    for (int s = s0; s < s1; s += 2) {
      slab(std::integral_constant<int, 0>{}, s);
      if (s + 1 < s1) slab(std::integral_constant<int, 1>{}, s + 1);
    }
    if (slot < 0) {
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int gi = tm + wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int gj = tn + wn * 32 + j * 16 + (lane & 15);
            if (gi < a.n && gj < a.n) {
              double *p = a.H + int64_t(gi) * a.ldh + gj;
              const double v = *p + acc[i][j][rr];
              *p = v;
              if (I != J) a.H[int64_t(gj) * a.ldh + gi] = v;
            }
          }
    } else {
      double *P = a.piece + int64_t(slot) * (BT * BT);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int li = wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int lj = wn * 32 + j * 16 + (lane & 15);
            P[li * BT + lj] = acc[i][j][rr];
          }
    }
  }
}

// Tail tiles: H += their chunks' partial tiles in chunk order, mirrored.
__global__ __launch_bounds__(NT) void syrk_fixup_kernel(SyrkArgs a) {
  const int i = blockIdx.x, t = a.head + i;
  const int nc = min(a.NC, tg::cdiv(a.NS, a.CK));  // chunks with rows
  int I, J;
  tile_of(t, I, J);
  const int tm = I * BT, tn = J * BT;
  for (int e = threadIdx.x; e < BT * BT; e += NT) {
    const int li = e / BT, lj = e % BT;
    const int gi = tm + li, gj = tn + lj;
    if (gi >= a.n || gj >= a.n) continue;
    double v = a.H[int64_t(gi) * a.ldh + gj];
    for (int c = 0; c < nc; ++c) v += a.piece[(int64_t(i) * a.NC + c) * (BT * BT) + e];
    a.H[int64_t(gi) * a.ldh + gj] = v;
    if (I != J) a.H[int64_t(gj) * a.ldh + gi] = v;
  }
}

// Persistent grid: resident workgroups of the kernel that launches (both
// kernels run two per CU on MI355X: syrk64l_kernel's 64 KB of static LDS and
// syrk16_kernel's registers), cached per device and kernel.
int resident_groups(bool lds64) {
  static int cached[64][2] = {{0}};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 512;
  int &c = cached[dev][lds64 ? 1 : 0];
  if (c == 0) {
    int ncu = 0, occ = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu < 1)
      ncu = 256;
    const hipError_t e =
        lds64 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, syrk64l_kernel<false>, NT, 0)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, syrk16_kernel<false>, NT, 0);
    if (e != hipSuccess || occ < 1) occ = 1;
    c = ncu * std::min(occ, 2);
  }
  return c;
}
// workspace sizing: the larger of the two (TG_SYRK_LDS64 is read per call)
int resident_groups() { return std::max(resident_groups(true), resident_groups(false)); }

}  // namespace

namespace tg {

constexpr int NCMAX = 16;  // chunks per tail tile (G tail tiles); TG_SYRK_NC picks 1..NCMAX, default 16

// tail tiles cut into chunks: the last min(T, G) of the T lower tiles
static int syrk16_tail_tiles(int n) {
  const int nt = cdiv(n, BT);
  return std::min(nt * (nt + 1) / 2, resident_groups());
}
// Layout: partial tiles (Tt tail tiles x NCMAX chunks), the queue head, the
// TG_SYRK_STAMPS clocks (3 words per workgroup).
size_t syrk16_workspace_size(int n) {
  const size_t G = resident_groups();
  return sizeof(double) * (size_t(syrk16_tail_tiles(n)) * NCMAX * BT * BT + 64 + 3 * G);
}

bool syrk16_supported(const void *X, int n, int64_t ldx) {
  return n % 8 == 0 && ldx % 8 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

// Decomposition (static, so H does not depend on which workgroup ran what):
// the last min(T, G) tiles are cut into NCMAX chunks of K, every other tile
// is one unit; units are handed out by an atomic queue, so a workgroup that
// runs faster (the older of the two on a CU wins the issue arbitration: with
// equal static shares their times differed by up to 1.8x, TG_SYRK_STAMPS)
// simply takes more of them, and the last round is made of sixteenth tiles
// (interleaved medians, tools/syrk_nc_ab.py, n = 4096: quarters 62.4 TF/s,
// eighths 65.4-66.2, sixteenths 66.2-67.6; n = 12,288 68.2-68.3 alike).
// (Eighth tiles over only the last G / 2 tiles measured slower at n = 4096,
// 24.8 against 19.8 ms: the whole tiles then handed to the slower workgroups
// of the first round finish last.)
hipError_t syrk16(hipStream_t st, const void *X, bool bf16, int64_t rows, int n, int64_t ldx,
                  double *H, int64_t ldh, void *ws) {
  SyrkArgs a{};
  a.X = static_cast<const unsigned short *>(X);
  a.ldx = ldx;
  a.rows = rows;
  a.n = n;
  a.H = H;
  a.ldh = ldh;
  const int nt = cdiv(n, BT);
  a.T = nt * (nt + 1) / 2;
  // development switch (read per call): the FP64-in-LDS kernel
  const char *l64 = getenv("TG_SYRK_LDS64");
  const bool lds64 = !(l64 && l64[0] == '0');
  a.NS = cdiv(rows, lds64 ? KL : NSUB * KC);
  const int G = resident_groups(lds64);
  a.Tt = std::min(syrk16_tail_tiles(n), G);
  a.head = a.T - a.Tt;
  const char *ncs = getenv("TG_SYRK_NC");  // development switch (read per call)
  const int nc = ncs ? std::max(1, std::min(NCMAX, atoi(ncs))) : NCMAX;
  a.NC = std::min(nc, a.NS);
  a.CK = cdiv(a.NS, a.NC);
  a.U = a.head + a.Tt * a.NC;
  a.piece = static_cast<double *>(ws);
  double *tail = a.piece + int64_t(a.Tt) * NCMAX * BT * BT;
  a.next = reinterpret_cast<unsigned *>(tail);
  // development switch (read per call): per-workgroup start / end clocks and
  // XCD, for tools/syrk_time.py
  a.stamps = getenv("TG_SYRK_STAMPS") ? reinterpret_cast<unsigned long long *>(tail + 64) : nullptr;
  hipError_t e = hipMemsetAsync(a.next, 0, sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  const int grid = std::min(G, a.U);
  if (lds64 && bf16)
    hipLaunchKernelGGL(syrk64l_kernel<true>, dim3(grid), dim3(NT), 0, st, a);
  else if (lds64)
    hipLaunchKernelGGL(syrk64l_kernel<false>, dim3(grid), dim3(NT), 0, st, a);
  else if (bf16)
    hipLaunchKernelGGL(syrk16_kernel<true>, dim3(grid), dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL(syrk16_kernel<false>, dim3(grid), dim3(NT), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(syrk_fixup_kernel, dim3(a.Tt), dim3(NT), 0, st, a);
  return hipGetLastError();
}

}  // namespace tg

extern "C" size_t tg_syrk_workspace_size(int n) {
  return n > 0 ? tg::syrk16_workspace_size(n) : 0;
}

extern "C" int tg_syrk_accum_ws(void *stream, const void *X, int x_dtype, int64_t rows, int n,
                                int64_t ldx, double *H, int ldh, void *ws, size_t ws_bytes) {
  TG_ARG(X, 2, "null X");
  TG_ARG(x_dtype >= TG_F16 && x_dtype <= TG_F64, 3, "unsupported dtype");
  TG_ARG(rows >= 0, 4, "rows < 0");
  TG_ARG(n > 0, 5, "n <= 0");
  TG_ARG(ldx >= n, 6, "ldx < n");
  TG_ARG(H, 7, "null H");
  TG_ARG(ldh >= n, 8, "ldh < n");
  if (rows == 0) return 0;
  const bool b16 = x_dtype == TG_F16 || x_dtype == TG_BF16;
  if (!b16 || !tg::syrk16_supported(X, n, ldx) || rows > INT32_MAX)
    return tg_syrk_accum(stream, X, x_dtype, rows, n, ldx, H, ldh);
  TG_ARG(ws && ws_bytes >= tg::syrk16_workspace_size(n), 9, "workspace too small");
  TG_HIP(tg::syrk16((hipStream_t)stream, X, x_dtype == TG_BF16, rows, n, ldx, H, ldh, ws));
  return 0;
}

