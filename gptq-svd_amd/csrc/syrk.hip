// Hessian accumulation H += X^T X (A1, gptq_utils.py:218-223 `H.addmm_(x.T, x)`
// with x cast to float64) for 16-bit activations (fp16 / bf16, what the
// harness hooks hand over), FP64 MFMA (v_mfma_f64_16x16x4_f64) on gfx950.
//
// Work: rows x n^2 / 2 FMAs on the lower 128 x 128 tiles (mirrored).  The
// inputs are exact in FP64, every product is formed and summed in FP64.
//
// Layout and schedule:
//  * a workgroup (4 waves as 2 x 2, 64 x 64 per wave = 4 x 4 MFMA blocks)
//    owns one 128 x 128 tile of H at a time and streams the two 128-column
//    strips of X it needs (tile row I, tile column J) in slabs of 32 rows;
//  * X stays 16-bit in LDS: a strip slab is 128 columns x 32 rows, column
//    major, 64 B per column, its four 16-B chunks (8 consecutive rows each)
//    XOR-swizzled by the column's (c >> 2) & 3 so that the ds_read_b128
//    fragment reads of a wave hit 64 distinct banks; lane group g = lane >> 4
//    takes rows 8g..8g+7 of the slab, so one 16-B read holds the lane's
//    operand for 8 consecutive MFMA steps (converted to FP64 in registers);
//  * global loads are 16 B per lane (8 columns of one row), two slabs ahead,
//    written to LDS as row pairs (one ds_write_b32 per column);
//  * stream-K: the lower tiles' slabs form one list (tile-major), cut into
//    equal contiguous ranges, one per resident workgroup (grid = CUs x
//    occupancy), so every workgroup does the same work and the launch has no
//    tail round.  A tile finished inside one range is added to H directly;
//    a tile cut between ranges leaves partial tiles in the workspace, and
//    `syrk_fixup_kernel` adds them to H in range order (deterministic).
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cstdlib>

#include "../../include/truncgptq.h"
#include "common.h"

namespace {

typedef double doublex4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BT = 128;  // tile edge
constexpr int KC = 32;   // rows of X per slab
constexpr int NT = 256;  // threads per workgroup

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
  int NS;         // slabs per tile
  int64_t W;      // T * NS
  int G;          // workgroups (ranges)
  double *piece;  // G x 2 x BT x BT partial tiles
};

__device__ inline int64_t range_begin(const SyrkArgs &a, int g) {
  return a.W * g / a.G;
}

__device__ inline void tile_of(int b, int &I, int &J) {
  I = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= b) ++I;
  while (I * (I + 1) / 2 > b) --I;
  J = b - I * (I + 1) / 2;
}

// Global -> registers: this thread's two rows (2rp, 2rp + 1) of 8 columns
// (cg * 8 ..) of both strips.
struct Stage {
  u32x4 v[2][2];  // [strip][row]
  __device__ inline void load(const SyrkArgs &a, int c0A, int c0B, int64_t k0) {
    const int t = threadIdx.x, cg = t & 15, rp = t >> 4;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = (s == 0 ? c0A : c0B) + cg * 8;
      const bool cok = c < a.n;  // n % 8 == 0: a chunk is all in or all out
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int64_t k = k0 + 2 * rp + r;
        const bool ok = cok && k < a.rows;
        const int64_t kc = ok ? k : 0;
        const int cc = ok ? c : 0;
        u32x4 x = *reinterpret_cast<const u32x4 *>(a.X + kc * a.ldx + cc);
        v[s][r] = ok ? x : u32x4{0u, 0u, 0u, 0u};
      }
    }
  }
  // registers -> LDS: column c, rows 2rp, 2rp+1 as one 4-byte word
  __device__ inline void store(unsigned short *SA, unsigned short *SB) const {
    const int t = threadIdx.x, cg = t & 15, rp = t >> 4;
    const int k = 2 * rp, q = k >> 3, kin = k & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      unsigned short *S = s == 0 ? SA : SB;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = cg * 8 + j;
        const unsigned lo = (v[s][0][j >> 1] >> ((j & 1) * 16)) & 0xffffu;
        const unsigned hi = (v[s][1][j >> 1] >> ((j & 1) * 16)) & 0xffffu;
        *reinterpret_cast<unsigned *>(S + c * KC + ((q ^ swz(c)) << 3) + kin) = lo | (hi << 16);
      }
    }
  }
};

// A wave's operands of one slab: for each of its 4 + 4 MFMA blocks, the 8
// rows of its lane group (one ds_read_b128 each).
struct Frags {
  u32x4 a[4], b[4];
  __device__ inline void read(const unsigned short *SA, const unsigned short *SB) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1, g = lane >> 4, r = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = wm * 64 + i * 16 + r;
      a[i] = *reinterpret_cast<const u32x4 *>(SA + c * KC + ((g ^ swz(c)) << 3));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = wn * 64 + j * 16 + r;
      b[j] = *reinterpret_cast<const u32x4 *>(SB + c * KC + ((g ^ swz(c)) << 3));
    }
  }
};

template <bool BF16>
__device__ inline void slab_mfma(const Frags &f, doublex4 (&acc)[4][4]) {
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    double av[4], bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) av[i] = h2d<BF16>((f.a[i][kk >> 1] >> ((kk & 1) * 16)) & 0xffffu);
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = h2d<BF16>((f.b[j][kk >> 1] >> ((kk & 1) * 16)) & 0xffffu);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
  }
}

__device__ inline void lds_drain_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

template <bool BF16, int OCC>
__global__ __launch_bounds__(NT, OCC) void syrk16_kernel(SyrkArgs a) {
  // [stage][strip]; at the top of slab s the two stages hold slabs s and s + 1
  __shared__ __attribute__((aligned(16))) unsigned short S[2][2][BT * KC];
  const int g = blockIdx.x;
  const int64_t w0 = range_begin(a, g), w1 = range_begin(a, g + 1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int t_first = int(w0 / a.NS);
  int64_t w = w0;
  while (w < w1) {
    const int t = int(w / a.NS);
    const int s0 = int(w - int64_t(t) * a.NS);
    const int s1 = int(std::min<int64_t>(a.NS, s0 + (w1 - w)));
    w += s1 - s0;
    int I, J;
    tile_of(t, I, J);
    const int tm = I * BT, tn = J * BT;
    doublex4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
    // prologue: slabs s0, s0 + 1 into LDS, s0 + 2 into registers, frags of s0
    Stage st;
    st.load(a, tm, tn, int64_t(s0) * KC);
    st.store(S[0][0], S[0][1]);
    if (s0 + 1 < s1) {
      st.load(a, tm, tn, int64_t(s0 + 1) * KC);
      st.store(S[1][0], S[1][1]);
    }
    if (s0 + 2 < s1) st.load(a, tm, tn, int64_t(s0 + 2) * KC);
    __syncthreads();
    Frags f, fn;
    f.read(S[0][0], S[0][1]);
    lds_drain_barrier();  // every wave has its slab-s0 operands: stage 0 is free
    for (int s = s0; s < s1; ++s) {
      const int b = (s - s0) & 1;
      if (s + 1 < s1) fn.read(S[b ^ 1][0], S[b ^ 1][1]);  // slab s + 1, for the next step
      slab_mfma<BF16>(f, acc);
      if (s + 2 < s1) {
        st.store(S[b][0], S[b][1]);  // slab s + 2 over slab s (its operands are in f)
        if (s + 3 < s1) st.load(a, tm, tn, int64_t(s + 3) * KC);
      }
      lds_drain_barrier();
      f = fn;
    }
    const bool whole = s0 == 0 && s1 == a.NS;
    if (whole) {  // H += acc on the tile, mirrored
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int gi = tm + wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int gj = tn + wn * 64 + j * 16 + (lane & 15);
            if (gi < a.n && gj < a.n) {
              double *p = a.H + int64_t(gi) * a.ldh + gj;
              const double v = *p + acc[i][j][rr];
              *p = v;
              if (I != J) a.H[int64_t(gj) * a.ldh + gi] = v;
            }
          }
    } else {  // partial tile: slot 0 = the range's first tile, 1 = its last
      double *P = a.piece + (int64_t(g) * 2 + (t == t_first ? 0 : 1)) * (BT * BT);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int li = wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
            const int lj = wn * 64 + j * 16 + (lane & 15);
            P[li * BT + lj] = acc[i][j][rr];
          }
    }
  }
}

// Tiles cut between ranges: H += sum of the pieces in range order, mirrored.
__global__ __launch_bounds__(NT) void syrk_fixup_kernel(SyrkArgs a) {
  const int t = blockIdx.x;
  const int64_t t0 = int64_t(t) * a.NS, t1 = t0 + a.NS;
  // first range with w1 > t0
  int glo = int(t0 * a.G / a.W);
  while (glo > 0 && range_begin(a, glo) > t0) --glo;
  while (range_begin(a, glo + 1) <= t0) ++glo;
  if (range_begin(a, glo) <= t0 && range_begin(a, glo + 1) >= t1) return;  // whole in one range
  int I, J;
  tile_of(t, I, J);
  const int tm = I * BT, tn = J * BT;
  for (int e = threadIdx.x; e < BT * BT; e += NT) {
    const int li = e / BT, lj = e % BT;
    const int gi = tm + li, gj = tn + lj;
    double v = 0.0;
    const bool in = gi < a.n && gj < a.n;
    if (in) v = a.H[int64_t(gi) * a.ldh + gj];
    for (int gg = glo; gg < a.G && range_begin(a, gg) < t1; ++gg) {
      const int slot = (range_begin(a, gg) / a.NS == t) ? 0 : 1;
      v += a.piece[(int64_t(gg) * 2 + slot) * (BT * BT) + e];
    }
    if (in) {
      a.H[int64_t(gi) * a.ldh + gj] = v;
      if (I != J) a.H[int64_t(gj) * a.ldh + gi] = v;
    }
  }
}

// Workgroups per CU: 2 (two waves per SIMD from two workgroups, whose
// barriers fall at different times) or 1 (all 512 registers for one wave);
// TG_SYRK_OCC=1|2 picks one (development switch, read once).
int syrk_occ() {
  static const int occ = [] {
    const char *e = getenv("TG_SYRK_OCC");
    return (e && atoi(e) == 1) ? 1 : 2;
  }();
  return occ;
}

int resident_groups() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 512;
  if (cached[dev] == 0) {
    int ncu = 0, occ = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu < 1)
      ncu = 256;
    const hipError_t e = syrk_occ() == 1
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, syrk16_kernel<false, 1>, NT, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, syrk16_kernel<false, 2>, NT, 0);
    if (e != hipSuccess || occ < 1) occ = 1;
    cached[dev] = ncu * std::min(occ, syrk_occ());
  }
  return cached[dev];
}

}  // namespace

namespace tg {

size_t syrk16_workspace_size() {
  return sizeof(double) * size_t(resident_groups()) * 2 * BT * BT;
}

bool syrk16_supported(const void *X, int n, int64_t ldx) {
  return n % 8 == 0 && ldx % 8 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

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
  a.NS = cdiv(rows, KC);
  a.W = int64_t(a.T) * a.NS;
  a.G = int(std::min<int64_t>(resident_groups(), a.W));
  a.piece = static_cast<double *>(ws);
  if (syrk_occ() == 1) {
    if (bf16) hipLaunchKernelGGL((syrk16_kernel<true, 1>), dim3(a.G), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((syrk16_kernel<false, 1>), dim3(a.G), dim3(NT), 0, st, a);
  } else {
    if (bf16) hipLaunchKernelGGL((syrk16_kernel<true, 2>), dim3(a.G), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((syrk16_kernel<false, 2>), dim3(a.G), dim3(NT), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(syrk_fixup_kernel, dim3(a.T), dim3(NT), 0, st, a);
  return hipGetLastError();
}

}  // namespace tg

extern "C" size_t tg_syrk_workspace_size(int n) {
  (void)n;
  return tg::syrk16_workspace_size();
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
  TG_ARG(ws && ws_bytes >= tg::syrk16_workspace_size(), 9, "workspace too small");
  TG_HIP(tg::syrk16((hipStream_t)stream, X, x_dtype == TG_BF16, rows, n, ldx, H, ldh, ws));
  return 0;
}

