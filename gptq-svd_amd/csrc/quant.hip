// Quantize / error-propagate path of TruncGPTQ on MI355X (gfx950).
//
// Replaces, in /root/reference/src/TruncGPTQ/gptq_utils.py:
//   Quantizer.find_params            :249-266   -> group_params_kernel
//   gptq_fwrd prologue (permute)     :491-495   -> permute_kernel (S/Z gathered on the fly)
//   gptq_block_kernel (Triton)       :298-386   -> block_kernel
//   cross-block E @ (U/diag) update  :537-545   -> cross_gemm_kernel (FP32 MFMA 32x32x2)
//   tail RTN + unpermute             :547-557   -> finalize_kernel
//   (packing: new, README.md:133)                -> pack kernels
//
// Exactness contract (tests/test_gpu_quant.py): every elementwise op is the
// reference's IEEE f32 op in the reference's order.  FMA contraction is
// disabled for this file; the one place an FMA chain is *intended* is the
// cross-block GEMM, whose reduction order the reference leaves to the BLAS;
// here it is defined as the k-ordered fmaf chain from +0 (what MFMA computes
// and what oracle/quant_ref.c computes).
#pragma clang fp contract(off)

#include <type_traits>

#include "../../include/truncgptq.h"
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// ---------------------------------------------------------------------------
// A7: static-group scale / zero (gptq_utils.py:249-266), one wave per group.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void group_params_kernel(const float *__restrict__ W, int m,
                                                           int ldw, int g, int G, float maxq,
                                                           int sym, float *__restrict__ scale,
                                                           float *__restrict__ zero) {
  const int wave = int((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= m * G) return;
  const int r = wave / G, gi = wave % G;
  const float *p = W + size_t(r) * ldw + size_t(gi) * g;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = lane; i < g; i += 64) {
    float v = p[i];
    if (sym) {
      mx = fmaxf(mx, fabsf(v));
    } else {
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off));
    mx = fmaxf(mx, __shfl_xor(mx, off));
  }
  if (lane == 0) {
    float s, z;
    if (sym) {
      float a = mx < 1e-5f ? 1e-5f : mx;  // clamp(min=1e-5)          :259
      s = a / maxq;                       // true IEEE division (CPU torch) :260
      z = 0.0f;
    } else {
      float d = mx - mn;
      d = d < 1e-5f ? 1e-5f : d;          // (mx - mn).clamp(min=1e-5)      :265
      s = d / maxq;
      z = rintf(-mn / s);                 // torch.round = half-to-even     :266
      z = z < 0.0f ? 0.0f : (z > maxq ? maxq : z);
    }
    scale[size_t(r) * G + gi] = s;
    zero[size_t(r) * G + gi] = z;
  }
}

// ---------------------------------------------------------------------------
// Permutation helpers (gptq_utils.py:493, :556-557).
// ---------------------------------------------------------------------------
__global__ void invperm_kernel(const int64_t *__restrict__ perm, int n, int32_t *__restrict__ inv,
                               int32_t *__restrict__ perm32) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) {
    int p = int(perm[c]);
    inv[p] = c;
    perm32[c] = p;
  }
}

__global__ void permute_kernel(const float *__restrict__ W, int n, const int32_t *__restrict__ perm,
                               float *__restrict__ Wp) {
  const int r = blockIdx.y;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
    Wp[size_t(r) * n + c] = W[size_t(r) * n + perm[c]];
}

// ---------------------------------------------------------------------------
// Per-block prep: corr[c][j] = U[c, j] * (1/U[c, c])   (Triton :368-377)
//                 SM[c][j]   = U[c, i2 + j] / U[c, c]   (:539-541)
// ---------------------------------------------------------------------------
// Loop mode (use_triton=False, :516-534, :544): corr and SM are the raw rows
// U[c, :] and dg[c] = U[c, c] (the error is divided by it instead).
__global__ void prep_block_kernel(const float *__restrict__ Ublk, int ldu, int bw, int nc,
                                  float *__restrict__ corr, int ldcorr, float *__restrict__ SM,
                                  int ldsm, float *__restrict__ dg) {
  const int c = blockIdx.x;
  const float *urow = Ublk + size_t(c) * ldu;
  const float d = urow[c];
  if (dg) {
    if (threadIdx.x == 0) dg[c] = d;
    for (int j = threadIdx.x; j < bw; j += blockDim.x) corr[size_t(c) * ldcorr + j] = urow[j];
    if (SM)
      for (int j = threadIdx.x; j < nc; j += blockDim.x) SM[size_t(c) * ldsm + j] = urow[bw + j];
    return;
  }
  const float inv = 1.0f / d;
  for (int j = threadIdx.x; j < bw; j += blockDim.x) corr[size_t(c) * ldcorr + j] = urow[j] * inv;
  for (int j = threadIdx.x; j < nc; j += blockDim.x) SM[size_t(c) * ldsm + j] = urow[bw + j] / d;
}

// ---------------------------------------------------------------------------
// A9: the intra-block quantize + propagate loop.
//
// One workgroup owns RW rows and all `bw` columns of the block (rows are
// independent).  The block's W rows live in LDS.  Columns are processed in
// panels of P: wave 0 runs the sequential column chain for the panel with one
// lane per row (panel columns in registers, corr broadcast from LDS); then
// all waves apply the panel's P updates, in column order, to every later
// column of the block.  Per element this is exactly the reference sequence
// w_j <- w_j - e_c * corr[c][j] for c = 0, 1, ... (separately rounded mul
// and sub), so the result is bit-identical to the Triton kernel.
// ---------------------------------------------------------------------------
#ifndef TG_QUANT_RW
#define TG_QUANT_RW 16
#endif
constexpr int RW = TG_QUANT_RW;  // rows per workgroup
constexpr int P = 32;   // panel width

struct BlockArgs {
  const float *W;
  int ldw;  // block start (column i1), row stride
  float *Q;
  int ldq;
  uint8_t *codes;
  int ldc;
  float *E;
  int lde;
  const float *corr;
  int ldcorr;
  const float *dg;  // loop mode: U[c, c] per block column
  // explicit s/z (tg_process_block) ...
  const float *s;
  int lds;
  const float *z;
  int ldz;
  // ... or gathered from per-group params through the permutation
  const float *scale;
  const float *zero;
  const int32_t *perm;
  int G, g, col0;
  int m, bw;
  float minq, maxq;
  int code_off;
  int dbl;  // two diagonal corr buffers (block_smem(bw, true)): the grid has <= 1 workgroup per CU
};

template <bool GATHER>
__device__ inline void load_sz(const BlockArgs &a, int row, int c, float &s, float &z) {
  if (row >= a.m) {
    s = 1.0f;
    z = 0.0f;
    return;
  }
  if (GATHER) {
    const int gi = a.perm[a.col0 + c] / a.g;
    s = a.scale[size_t(row) * a.G + gi];
    z = a.zero[size_t(row) * a.G + gi];
  } else {
    s = a.s[size_t(row) * a.lds + c];
    z = a.z[size_t(row) * a.ldz + c];
  }
}

template <bool GATHER, bool LOOP>
__global__ __launch_bounds__(256) void block_kernel(BlockArgs a) {
  extern __shared__ float smem[];
  const int bwp = a.bw + 1;             // odd row stride: lane-per-row access is conflict-free
  float *Wb = smem;                      // [RW][bwp]
  float *el = Wb + RW * bwp;             // [2][RW][P+1] panel errors, parity by panel
  float *cpb = el + 2 * RW * (P + 1);    // [1 + dbl][P][P] corr diagonal panel block(s)
  float *cq = cpb + (a.dbl ? 2 : 1) * P * P;  // [P][P] corr[p0 + cc][p0 + P + j]: the next panel's columns
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * RW;

  for (int idx = tid; idx < RW * a.bw; idx += blockDim.x) {
    const int rr = idx / a.bw, c = idx % a.bw;
    const int row = r0 + rr;
    Wb[rr * bwp + c] = row < a.m ? a.W[size_t(row) * a.ldw + c] : 0.0f;
  }
  // corr[q0 + cc][c0 + j] (cc, j < P, zero outside the block) of 1024 entries:
  // this thread's share of them (threads t0, t0 + nt, ...) into registers
  constexpr int NS = (P * P + 191) / 192;
  auto corr_fetch = [&](int q0, int c0, int t0, int nt, float (&v)[NS]) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int idx = t0 + nt * u, cc = idx / P, j = idx % P;
      const bool ok = idx < P * P && q0 + cc < a.bw && c0 + j < a.bw;
      v[u] = ok ? a.corr[size_t(q0 + cc) * a.ldcorr + c0 + j] : 0.0f;
    }
  };
  auto corr_store = [&](float *dst, int t0, int nt, const float (&v)[NS]) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int idx = t0 + nt * u;
      if (idx < P * P) dst[idx] = v[u];
    }
  };
  {
    float v[NS];
    for (int t0 = tid; t0 < 192; t0 += blockDim.x) {  // (threads < 192)
      corr_fetch(0, 0, t0, 192, v);
      corr_store(cpb, t0, 192, v);
    }
  }
  // the chain's scales / zeros of a panel (lane rr < RW of wave 0)
  auto sz_fetch = [&](int p0, float (&sv)[P], float (&zv)[P]) {
    const int rr = tid, row = r0 + rr, pw = min(P, a.bw - p0);
#pragma unroll
    for (int t = 0; t < P; ++t) {
      if (t < pw) load_sz<GATHER>(a, row, p0 + t, sv[t], zv[t]);
      else { sv[t] = 1.0f; zv[t] = 0.0f; }
    }
  };
  float sv[P], zv[P];
  if (tid < RW) sz_fetch(0, sv, zv);
  __syncthreads();

  // Per panel p: wave 0 runs panel p's column chain (one lane per row);
  // waves 1-3 fetch the corr blocks the next steps need (the off-diagonal
  // block for the update of panel p+1's columns, into LDS before the barrier;
  // the next diagonal block for panel p+1's chain, into LDS after it, once
  // the chain is done with cp -- one buffer each keeps two workgroups per CU
  // at bw = 1024, the occupancy the 12,288-row layers need; with at most one
  // workgroup per CU anyway, dbl: two diagonal buffers by panel parity, the
  // next one stored before the barrier) and apply panel p-1's errors to the
  // columns after panel p, each thread's next column's corr loads in flight
  // while it updates the current one; then all threads apply panel p's errors
  // to panel p+1's columns from LDS.  Every element still receives the
  // panels' updates in panel order, cc ascending within a panel, each as the
  // separately rounded mul and sub: the result is the same bit for bit.
  for (int p0 = 0, it = 0; p0 < a.bw; p0 += P, ++it) {
    const int pw = min(P, a.bw - p0);
    float *elc = el + (it & 1) * RW * (P + 1);
    const float *elp = el + ((it + 1) & 1) * RW * (P + 1);
    const bool more = p0 + pw < a.bw;  // uniform
    const float *cp = cpb + (a.dbl ? (it & 1) * P * P : 0);
    float *cpn = cpb + (a.dbl ? ((it + 1) & 1) * P * P : 0);  // panel p+1's
    float vp[NS];  // waves 1-3: their share of panel p+1's diagonal corr block
    if (tid < RW) {  // sequential column chain: one lane per row
      const int rr = tid, row = r0 + rr;
      float wv[P];
#pragma unroll
      for (int t = 0; t < P; ++t) wv[t] = t < pw ? Wb[rr * bwp + p0 + t] : 0.0f;
#pragma unroll
      for (int cc = 0; cc < P; ++cc) {
        if (cc < pw) {
          const float x = wv[cc];
          float t = x / sv[cc];                               // :354
          t = t + zv[cc];
          float qi, err, qv;
          if (LOOP) {                                         // :524-529
            qi = clampf(rintf(t), a.minq, a.maxq);             // torch.round: half-to-even
            qv = (qi - zv[cc]) * sv[cc];
            err = (x - qv) / a.dg[p0 + cc];
          } else {
            t = t + 0.5f;
            qi = clampf(floorf(t), a.minq, a.maxq);            // :355
            qv = (qi - zv[cc]) * sv[cc];                       // :356
            err = x - qv;                                      // :358
          }
          if (row < a.m) {
            const int c = p0 + cc;
            a.Q[size_t(row) * a.ldq + c] = qv;
            a.E[size_t(row) * a.lde + c] = err;
            if (a.codes) a.codes[size_t(row) * a.ldc + c] = uint8_t(int(qi) + a.code_off);
          }
          elc[rr * (P + 1) + cc] = err;
#pragma unroll
          for (int j = cc + 1; j < P; ++j) {  // :377-386 inside the panel
            const float d = err * cp[cc * P + j];
            wv[j] = wv[j] - d;
          }
        }
      }
      if (more) sz_fetch(p0 + P, sv, zv);  // the next panel's, in flight through the barrier
    } else if (tid >= 64) {
      const int t0 = tid - 64;
      float vq[NS];
      if (more) {
        corr_fetch(p0, p0 + P, t0, 192, vq);      // off-diagonal block (p, p+1)
        corr_fetch(p0 + P, p0 + P, t0, 192, vp);  // diagonal block of panel p+1
      }
      if (p0 > 0) {
        // deferred trailing update of panel p-1: the columns after panel p
        const int q0 = p0 - P;
        int j = p0 + P + t0;
        float cv[P];
        if (j < a.bw) {
#pragma unroll
          for (int cc = 0; cc < P; ++cc) cv[cc] = a.corr[size_t(q0 + cc) * a.ldcorr + j];
        }
        for (; j < a.bw; j += 192) {
          float cn[P];
          const int jn = min(j + 192, a.bw - 1);  // clamped: the last prefetch is unused
#pragma unroll
          for (int cc = 0; cc < P; ++cc) cn[cc] = a.corr[size_t(q0 + cc) * a.ldcorr + jn];
#pragma unroll 2
          for (int rr = 0; rr < RW; ++rr) {
            float w = Wb[rr * bwp + j];
#pragma unroll
            for (int cc = 0; cc < P; ++cc) {
              const float d = elp[rr * (P + 1) + cc] * cv[cc];
              w = w - d;
            }
            Wb[rr * bwp + j] = w;
          }
#pragma unroll
          for (int cc = 0; cc < P; ++cc) cv[cc] = cn[cc];
        }
      }
      if (more) {
        corr_store(cq, t0, 192, vq);
        if (a.dbl) corr_store(cpn, t0, 192, vp);
      }
    }
    __syncthreads();
    if (more) {  // panel p+1's columns get panel p's errors (corr from LDS)
      if (tid >= 64 && !a.dbl) corr_store(cpn, tid - 64, 192, vp);  // the chain is done with cp
      const int q0 = p0 + P, qw = min(P, a.bw - q0);
      const int jj = tid & 31;
      if (jj < qw) {
        float cv[P];
#pragma unroll
        for (int cc = 0; cc < P; ++cc) cv[cc] = cq[cc * P + jj];
        for (int rr = tid >> 5; rr < RW; rr += 256 / 32) {
          float w = Wb[rr * bwp + q0 + jj];
#pragma unroll
          for (int cc = 0; cc < P; ++cc) {
            const float d = elc[rr * (P + 1) + cc] * cv[cc];
            w = w - d;
          }
          Wb[rr * bwp + q0 + jj] = w;
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// A10: cross-block update W[:, i2:] -= E @ SM with FP32 MFMA (32x32x2).
// acc starts at +0 and walks k in ascending order through one accumulator
// per output element, so each output is the k-ordered fmaf chain.
// Tile 128x128 per workgroup, 4 waves each 64x64 (2x2 MFMA tiles), K-tile 32.
// Staging: 16-B global loads with clamped addresses (out-of-range k -> 0 by
// select; out-of-range rows/columns only feed masked outputs), the next
// K-tile prefetched into registers while the current one is multiplied.
// LDS keeps even and odd k apart (A: [k & 1][row][k / 2], B: [k & 1][col][k / 2],
// runs of 20 floats: the 16-lane passes of a 16-B read hit distinct banks) so
// one 16-B LDS read gives a lane its operands for four consecutive MFMAs
// (lane half h = l >> 5 supplies k = kk + h).
// Requires lde % 4 == 0 and ldsm % 4 == 0 (host falls back otherwise).
// ---------------------------------------------------------------------------
constexpr int GM = 128, GN = 128, GK = 32;
constexpr int KH = GK / 2 + 4;  // floats per (k parity, row) run, padded

__global__ __launch_bounds__(256) void cross_gemm_kernel(const float *__restrict__ E, int lde,
                                                         const float *__restrict__ SM, int ldsm,
                                                         float *__restrict__ W, int ldw, int m,
                                                         int nc, int K) {
  __shared__ float As[2][GM][KH];
  __shared__ float Bs[2][GN][KH];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int tm = blockIdx.y * GM, tn = blockIdx.x * GN;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // A: thread -> rows (tid >> 3) + 32u, k quad (tid & 7);
  // B: k row (tid & 31), column quads (tid >> 5) + 8u
  const int aq = tid & 7, ar = tid >> 3, br = tid & 31, bq0 = tid >> 5;
  float4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gi = min(tm + ar + 32 * u, m - 1);
      const int gk = k0 + 4 * aq;  // < roundup32(K) <= lde
      float4 v = *reinterpret_cast<const float4 *>(E + size_t(gi) * lde + gk);
      v.x = gk < K ? v.x : 0.0f;
      v.y = gk + 1 < K ? v.y : 0.0f;
      v.z = gk + 2 < K ? v.z : 0.0f;
      v.w = gk + 3 < K ? v.w : 0.0f;
      ra[u] = v;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gk = k0 + br;
      const int gkc = min(gk, K - 1);
      const int gj = min(tn + 4 * (bq0 + 8 * u), ldsm - 4);
      float4 v = *reinterpret_cast<const float4 *>(SM + size_t(gkc) * ldsm + gj);
      if (gk >= K) v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      rb[u] = v;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = ar + 32 * u;  // k = 4 aq .. 4 aq + 3: even (4aq, 4aq+2), odd (4aq+1, 4aq+3)
      *reinterpret_cast<float2 *>(&As[0][row][2 * aq]) = make_float2(ra[u].x, ra[u].z);
      *reinterpret_cast<float2 *>(&As[1][row][2 * aq]) = make_float2(ra[u].y, ra[u].w);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c0 = 4 * (bq0 + 8 * u), kp = br & 1, kh = br >> 1;
      Bs[kp][c0 + 0][kh] = rb[u].x;
      Bs[kp][c0 + 1][kh] = rb[u].y;
      Bs[kp][c0 + 2][kh] = rb[u].z;
      Bs[kp][c0 + 3][kh] = rb[u].w;
    }
  };
  gload(0);
  for (int k0 = 0; k0 < K; k0 += GK) {
    lstore();
    __syncthreads();
    if (k0 + GK < K) gload(k0 + GK);  // in flight during the MFMAs below
#pragma unroll
    for (int c = 0; c < GK / 8; ++c) {  // four MFMA k-steps (kk = 8c .. 8c + 6) per 16-B read
      float4 av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        av[i] = *reinterpret_cast<const float4 *>(&As[h][wm * 64 + i * 32 + l32][4 * c]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bv[j] = *reinterpret_cast<const float4 *>(&Bs[h][wn * 64 + j * 32 + l32][4 * c]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][e], bv[j][e], acc[i][j], 0, 0,
                                                             0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int gi = tm + wm * 64 + i * 32 + row;
        const int gj = tn + wn * 64 + j * 32 + l32;
        if (gi < m && gj < nc) {
          float *p = W + size_t(gi) * ldw + gj;
          *p = *p - acc[i][j][r];  // W[:, i2:] -= Global_delta   (:545)
        }
      }
}

// Generic fallback (unaligned leading dimensions): scalar staging.
__global__ __launch_bounds__(256) void cross_gemm_scalar_kernel(const float *__restrict__ E,
                                                                int lde,
                                                                const float *__restrict__ SM,
                                                                int ldsm, float *__restrict__ W,
                                                                int ldw, int m, int nc, int K) {
  __shared__ float As[GM][GK + 1];
  __shared__ float Bs[GK][GN + 32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tm = blockIdx.y * GM, tn = blockIdx.x * GN;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += GK) {
    {
      const int row = tid >> 1, kb = (tid & 1) * 16;
      const int gi = min(tm + row, m - 1);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int gk = k0 + kb + t;
        const float v = E[size_t(gi) * lde + min(gk, K - 1)];
        As[row][kb + t] = gk < K ? v : 0.0f;
      }
    }
    {
      const int kr = tid >> 3, cb = (tid & 7) * 16;
      const int gk = k0 + kr, gkc = min(gk, K - 1);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int gj = min(tn + cb + t, nc - 1);
        const float v = SM[size_t(gkc) * ldsm + gj];
        Bs[kr][cb + t] = gk < K ? v : 0.0f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[wm * 64 + i * 32 + (lane & 31)][kk + (lane >> 5)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kk + (lane >> 5)][wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int gi = tm + wm * 64 + i * 32 + row;
        const int gj = tn + wn * 64 + j * 32 + (lane & 31);
        if (gi < m && gj < nc) {
          float *p = W + size_t(gi) * ldw + gj;
          *p = *p - acc[i][j][r];
        }
      }
}

// ---------------------------------------------------------------------------
// Tail RTN for truncated columns (:547-553) fused with the unpermute (:556-557).
// ---------------------------------------------------------------------------
__global__ void finalize_kernel(const float *__restrict__ Wp, const float *__restrict__ Qp,
                                const uint8_t *__restrict__ cp, const int32_t *__restrict__ inv,
                                const int32_t *__restrict__ perm, const float *__restrict__ scale,
                                const float *__restrict__ zero, int G, int g, int n, int k,
                                float minq, float maxq, int code_off, float *__restrict__ Wq,
                                uint8_t *__restrict__ codes) {
  const int r = blockIdx.y;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const int c = inv[j];
    const size_t o = size_t(r) * n + c;
    float qv;
    int code;
    if (c >= k) {
      const int gi = j / g;  // perm[c] == j
      const float s = scale[size_t(r) * G + gi], z = zero[size_t(r) * G + gi];
      float t = Wp[o] / s;
      t = t + z;
      const float qi = clampf(rintf(t), minq, maxq);  // torch.round: half-to-even
      qv = (qi - z) * s;
      code = int(qi) + code_off;
    } else {
      qv = Qp[o];
      code = cp[o];
    }
    Wq[size_t(r) * n + j] = qv;
    if (codes) codes[size_t(r) * n + j] = uint8_t(code);
  }
}

// ---------------------------------------------------------------------------
// A13: bit-stream packing (value i of a column at bits [i*b, i*b+b)).
// ---------------------------------------------------------------------------
__global__ void pack_codes_kernel(const uint8_t *__restrict__ codes, int m, int n, int b,
                                  int32_t *__restrict__ qw) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;  // output feature
  const int wi = blockIdx.y;                            // word along in_features
  if (r >= m) return;
  const int bit0 = wi * 32;
  const int i0 = bit0 / b, i1 = min(n - 1, (bit0 + 31) / b);
  uint64_t acc = 0;
  for (int i = i0; i <= i1; ++i) {
    const int64_t sh = int64_t(i) * b - bit0;
    const uint64_t v = codes[size_t(r) * n + i] & ((1u << b) - 1);
    if (sh >= 0) acc |= v << sh;
    else acc |= v >> (-sh);
  }
  qw[size_t(wi) * m + r] = int32_t(uint32_t(acc & 0xffffffffu));
}

__global__ void pack_zeros_kernel(const float *__restrict__ zero, int m, int G, int b, int off,
                                  int32_t *__restrict__ qz) {
  const int gi = blockIdx.y;
  const int wi = blockIdx.x * blockDim.x + threadIdx.x;
  const int nw = (m * b) / 32;
  if (wi >= nw) return;
  const int bit0 = wi * 32;
  const int i0 = bit0 / b, i1 = min(m - 1, (bit0 + 31) / b);
  uint64_t acc = 0;
  for (int i = i0; i <= i1; ++i) {
    const int64_t sh = int64_t(i) * b - bit0;
    const uint64_t v = uint64_t(int(rintf(zero[size_t(i) * G + gi])) + off) & ((1u << b) - 1);
    if (sh >= 0) acc |= v << sh;
    else acc |= v >> (-sh);
  }
  qz[size_t(gi) * nw + wi] = int32_t(uint32_t(acc & 0xffffffffu));
}

size_t block_smem(int bw, bool dbl = true) {
  return sizeof(float) * (size_t(RW) * (bw + 1) + 2 * RW * (P + 1) + (dbl ? 3 : 2) * P * P);
}
// two diagonal corr buffers when the grid puts at most one workgroup on a CU
bool block_dbl(int m) { return tg::cdiv(m, RW) <= tg::xcd_info().xcds * tg::xcd_info().cus_per_xcd; }

constexpr int MAX_BLOCK = 2048;

hipError_t ensure_block_smem() {
  static bool done = false;  // per-process; attribute is per function, device-independent
  if (done) return hipSuccess;
  const int bytes = int(block_smem(MAX_BLOCK));
  hipError_t e = hipSuccess;
  for (const void *f : {(const void *)block_kernel<true, false>,
                        (const void *)block_kernel<false, false>,
                        (const void *)block_kernel<true, true>}) {
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  }
  done = e == hipSuccess;
  return e;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" int tg_group_params(void *stream, const float *W, int m, int n, int ldw, int group,
                               int w_bits, int sym, float *scale, float *zero) {
  TG_ARG(W, 2, "null W");
  TG_ARG(m > 0, 3, "m <= 0");
  TG_ARG(n > 0, 4, "n <= 0");
  TG_ARG(ldw >= n, 5, "ldw < n");
  const int g = group > 0 ? group : n;
  TG_ARG(n % g == 0, 6, "n % group_size != 0 (gptq_utils.py:253)");
  TG_ARG(w_bits >= 2 && w_bits <= 8, 7, "w_bits must be in [2, 8]");
  TG_ARG(scale && zero, 9, "null output");
  const int G = n / g;
  const float maxq = sym ? float((1 << (w_bits - 1)) - 1) : float((1 << w_bits) - 1);
  const int64_t waves = int64_t(m) * G;
  hipLaunchKernelGGL(group_params_kernel, dim3(tg::cdiv(waves * 64, 256)), dim3(256), 0,
                     (hipStream_t)stream, W, m, ldw, g, G, maxq, sym, scale, zero);
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_process_block(void *stream, const float *w, int ldw, const float *s, int lds,
                                const float *z, int ldz, const float *R, int ldr, int m, int B,
                                int minq, int maxq, float *q, int ldq, float *e, int lde,
                                void *ws, size_t ws_bytes) {
  TG_ARG(w && s && z && R, 2, "null input");
  TG_ARG(m > 0, 10, "m <= 0");
  TG_ARG(B > 0 && B <= MAX_BLOCK, 11, "block width must be in [1, 2048]");
  TG_ARG(q && e, 14, "null output");
  hipStream_t st = (hipStream_t)stream;
  tg::Arena ar(ws, ws_bytes);
  float *corr = ar.take<float>(size_t(B) * B);
  TG_WS(ar);
  TG_HIP(ensure_block_smem());
  hipLaunchKernelGGL(prep_block_kernel, dim3(B), dim3(256), 0, st, R, ldr, B, 0, corr, B,
                     (float *)nullptr, 0, (float *)nullptr);
  TG_LAUNCHED();
  BlockArgs a{};
  a.W = w; a.ldw = ldw; a.Q = q; a.ldq = ldq; a.codes = nullptr; a.ldc = 0; a.E = e; a.lde = lde;
  a.corr = corr; a.ldcorr = B; a.s = s; a.lds = lds; a.z = z; a.ldz = ldz;
  a.m = m; a.bw = B; a.minq = float(minq); a.maxq = float(maxq); a.code_off = 0;
  a.dbl = block_dbl(m);
  hipLaunchKernelGGL((block_kernel<false, false>), dim3(tg::cdiv(m, RW)), dim3(256), block_smem(B, a.dbl),
                     st, a);
  TG_LAUNCHED();
  return 0;
}

extern "C" size_t tg_process_block_workspace_size(int B) { return sizeof(float) * size_t(B) * B + 512; }

namespace {
struct QuantWs {
  float *Wp, *Qp, *E, *corr, *SM, *dg;
  uint8_t *cp;
  int32_t *inv, *perm32;
};
template <class A>
void quant_layout(A &ar, int m, int n, int block, QuantWs *p) {
  const int bp = (block + 31) & ~31;
  auto t = [&](auto *&dst, size_t cnt) {
    using T = std::remove_reference_t<decltype(*dst)>;
    if constexpr (std::is_same_v<A, tg::Arena>) dst = ar.template take<T>(cnt);
    else ar.template take<T>(cnt);
  };
  QuantWs d{};
  QuantWs &q = p ? *p : d;
  t(q.Wp, size_t(m) * n);
  t(q.Qp, size_t(m) * n);
  t(q.E, size_t(m) * bp);
  t(q.corr, size_t(bp) * bp);
  t(q.SM, size_t(bp) * n);
  t(q.dg, size_t(bp));
  t(q.cp, size_t(m) * n);
  t(q.inv, size_t(n));
  t(q.perm32, size_t(n));
}
}  // namespace

extern "C" size_t tg_quantize_workspace_size(int m, int n, int block) {
  tg::Sizer s;
  quant_layout(s, m, n, block, nullptr);
  return s.off + 256;
}

static int gptq_quantize_impl(bool loop, void *stream, const float *W, int m, int n,
                              const float *U, int k, int ldu, const int64_t *perm,
                              const float *scale, const float *zero, int group, int w_bits,
                              int sym, int block, float *Wq, uint8_t *codes, void *ws,
                              size_t ws_bytes) {
  TG_ARG(W, 2, "null W");
  TG_ARG(m > 0, 3, "m <= 0");
  TG_ARG(n > 0, 4, "n <= 0");
  TG_ARG(U, 5, "null U");
  TG_ARG(k >= 1 && k <= n, 6, "rank k must be in [1, n]");
  TG_ARG(ldu >= n, 7, "ldu < n");
  TG_ARG(perm, 8, "null perm");
  TG_ARG(scale && zero, 9, "null scale/zero");
  const int g = group > 0 ? group : n;
  TG_ARG(n % g == 0, 11, "n % group_size != 0");
  TG_ARG(w_bits >= 2 && w_bits <= 8, 12, "w_bits must be in [2, 8]");
  TG_ARG(block >= 1 && block <= MAX_BLOCK, 14, "block_size must be in [1, 2048]");
  TG_ARG(Wq, 15, "null output");
  hipStream_t st = (hipStream_t)stream;
  TG_HIP(ensure_block_smem());
  tg::Arena ar(ws, ws_bytes);
  QuantWs q{};
  quant_layout(ar, m, n, block, &q);
  TG_WS(ar);
  const int G = n / g;
  const float minq = sym ? -float((1 << (w_bits - 1)) - 1) : 0.0f;
  const float maxq = sym ? float((1 << (w_bits - 1)) - 1) : float((1 << w_bits) - 1);
  const int code_off = sym ? (1 << (w_bits - 1)) : 0;
  const int bp = (block + 31) & ~31;

  hipLaunchKernelGGL(invperm_kernel, dim3(tg::cdiv(n, 256)), dim3(256), 0, st, perm, n, q.inv,
                     q.perm32);
  TG_LAUNCHED();
  hipLaunchKernelGGL(permute_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, m),
                     dim3(256), 0, st, W, n, q.perm32, q.Wp);
  TG_LAUNCHED();

  for (int i1 = 0; i1 < k; i1 += block) {
    const int i2 = min(i1 + block, k);
    const int bw = i2 - i1;
    const int nc = n - i2;
    hipLaunchKernelGGL(prep_block_kernel, dim3(bw), dim3(256), 0, st, U + size_t(i1) * ldu + i1,
                       ldu, bw, nc, q.corr, bp, q.SM, n, loop ? q.dg : (float *)nullptr);
    TG_LAUNCHED();
    BlockArgs a{};
    a.W = q.Wp + i1; a.ldw = n; a.Q = q.Qp + i1; a.ldq = n; a.codes = q.cp + i1; a.ldc = n;
    a.E = q.E; a.lde = bp; a.corr = q.corr; a.ldcorr = bp; a.dg = q.dg;
    a.scale = scale; a.zero = zero; a.perm = q.perm32; a.G = G; a.g = g; a.col0 = i1;
    a.m = m; a.bw = bw; a.minq = minq; a.maxq = maxq; a.code_off = code_off;
    a.dbl = block_dbl(m);
    auto qtok = tg::prof_begin(st, tg::PROF_QBLOCK, 4.0 * 4.0 * double(m) * bw,
                               double(m) * bw * (bw - 1));
    if (loop)
      hipLaunchKernelGGL((block_kernel<true, true>), dim3(tg::cdiv(m, RW)), dim3(256),
                         block_smem(bw, a.dbl), st, a);
    else
      hipLaunchKernelGGL((block_kernel<true, false>), dim3(tg::cdiv(m, RW)), dim3(256),
                         block_smem(bw, a.dbl), st, a);
    tg::prof_end(st, qtok);
    TG_LAUNCHED();
    if (nc > 0) {
      auto gtok = tg::prof_begin(st, tg::PROF_CROSS_GEMM,
                                 4.0 * (double(m) * bw + double(bw) * nc + 2.0 * double(m) * nc),
                                 2.0 * double(m) * bw * nc);
      if (bp % 4 == 0 && n % 4 == 0 && n >= 4)
        hipLaunchKernelGGL(cross_gemm_kernel, dim3(tg::cdiv(nc, GN), tg::cdiv(m, GM)), dim3(256),
                           0, st, q.E, bp, q.SM, n, q.Wp + i2, n, m, nc, bw);
      else
        hipLaunchKernelGGL(cross_gemm_scalar_kernel, dim3(tg::cdiv(nc, GN), tg::cdiv(m, GM)),
                           dim3(256), 0, st, q.E, bp, q.SM, n, q.Wp + i2, n, m, nc, bw);
      tg::prof_end(st, gtok);
      TG_LAUNCHED();
    }
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(tg::cdiv(n, 256) < 16 ? tg::cdiv(n, 256) : 16, m),
                     dim3(256), 0, st, q.Wp, q.Qp, q.cp, q.inv, q.perm32, scale, zero, G, g, n, k,
                     minq, maxq, code_off, Wq, codes);
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_gptq_quantize(void *stream, const float *W, int m, int n, const float *U, int k,
                                int ldu, const int64_t *perm, const float *scale,
                                const float *zero, int group, int w_bits, int sym, int block,
                                float *Wq, uint8_t *codes, void *ws, size_t ws_bytes) {
  return gptq_quantize_impl(false, stream, W, m, n, U, k, ldu, perm, scale, zero, group, w_bits,
                            sym, block, Wq, codes, ws, ws_bytes);
}

extern "C" int tg_gptq_quantize_loop(void *stream, const float *W, int m, int n, const float *U,
                                     int k, int ldu, const int64_t *perm, const float *scale,
                                     const float *zero, int group, int w_bits, int sym, int block,
                                     float *Wq, uint8_t *codes, void *ws, size_t ws_bytes) {
  return gptq_quantize_impl(true, stream, W, m, n, U, k, ldu, perm, scale, zero, group, w_bits,
                            sym, block, Wq, codes, ws, ws_bytes);
}

extern "C" int tg_pack_codes(void *stream, const uint8_t *codes, int m, int n, int w_bits,
                             int32_t *qweight) {
  TG_ARG(codes, 2, "null codes");
  TG_ARG(m > 0, 3, "m <= 0");
  TG_ARG(n > 0, 4, "n <= 0");
  TG_ARG(w_bits >= 2 && w_bits <= 8, 5, "w_bits must be in [2, 8]");
  TG_ARG((int64_t(n) * w_bits) % 32 == 0, 4, "n * w_bits must be a multiple of 32");
  TG_ARG(qweight, 6, "null output");
  const int nw = int((int64_t(n) * w_bits) / 32);
  hipLaunchKernelGGL(pack_codes_kernel, dim3(tg::cdiv(m, 256), nw), dim3(256), 0,
                     (hipStream_t)stream, codes, m, n, w_bits, qweight);
  TG_LAUNCHED();
  return 0;
}

extern "C" int tg_pack_zeros(void *stream, const float *zero, int m, int G, int w_bits, int sym,
                             int32_t *qzeros) {
  TG_ARG(zero, 2, "null zero");
  TG_ARG(m > 0, 3, "m <= 0");
  TG_ARG(G > 0, 4, "G <= 0");
  TG_ARG(w_bits >= 2 && w_bits <= 8, 5, "w_bits must be in [2, 8]");
  TG_ARG((int64_t(m) * w_bits) % 32 == 0, 3, "m * w_bits must be a multiple of 32");
  TG_ARG(qzeros, 7, "null output");
  const int nw = int((int64_t(m) * w_bits) / 32);
  const int off = sym ? (1 << (w_bits - 1)) : 0;
  hipLaunchKernelGGL(pack_zeros_kernel, dim3(tg::cdiv(nw, 256), G), dim3(256), 0,
                     (hipStream_t)stream, zero, m, G, w_bits, off, qzeros);
  TG_LAUNCHED();
  return 0;
}
