// A6: the relative prediction error logged per sublayer
// (/root/reference/src/TruncGPTQ/gptq_utils.py:275-291, called from
// gptq_fwrd :560-561):
//
//   R = R_x.float();  W_o = W[:, perm];  W_q = Wq[:, perm]
//   err = ||(W_o - W_q) R^T||_F / ||W_o R^T||_F
//
// Both products share the B operand R^T, so one FP32 MFMA pass (32x32x2,
// the reference's FP32 GEMM with TF32 off, gptq_utils.py:474-475) forms the
// two 128x128 output tiles of a workgroup side by side and reduces their
// squares on the spot; nothing of the m x k products reaches HBM.  Per
// workgroup the two sums of squares are accumulated in FP64 and written as
// partials; one small kernel adds the partials in workgroup order
// (deterministic).  The gathers W[:, perm] and (W - Wq)[:, perm] are one
// streaming pass that writes both permuted operands (the GEMM then reads
// K-contiguous rows), R_x is converted to FP32 on the fly in the B loads.
#include <type_traits>

#include "../../include/truncgptq.h"
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int TM = 128, TN = 128, TK = 32;
constexpr int KP = TK / 2 + 4;  // floats per (k parity, row) run, padded (bank spread)

// Wp = W[:, perm], Dp = (W - Wq)[:, perm]   (gptq_utils.py:286-289)
__global__ void metric_gather_kernel(const float *__restrict__ W, const float *__restrict__ Wq,
                                     int n, int ldw, const int64_t *__restrict__ perm,
                                     float *__restrict__ Wp, float *__restrict__ Dp) {
  const int r = blockIdx.y;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const int64_t p = perm[c];
    const float w = W[size_t(r) * ldw + p], q = Wq[size_t(r) * ldw + p];
    Wp[size_t(r) * n + c] = w;
    Dp[size_t(r) * n + c] = w - q;
  }
}

__device__ inline double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// One 128 (rows of W) x 128 (rows of R_x) output tile of both products.
// Waves 2 x 2, each 64 x 64 = 2 x 2 MFMA blocks per product.
template <bool VEC>
__global__ __launch_bounds__(256) void metric_gemm_kernel(const float *__restrict__ Wp,
                                                          const float *__restrict__ Dp, int m,
                                                          int n, const double *__restrict__ Rx,
                                                          int ldr, int k,
                                                          double *__restrict__ part) {
  __shared__ float Aw[2][TM][KP];
  __shared__ float Ad[2][TM][KP];
  __shared__ float Bs[2][TN][KP];
  __shared__ double red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int tm = blockIdx.y * TM, tn = blockIdx.x * TN;
  floatx16 aw[2][2], ad[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) aw[i][j][r] = ad[i][j][r] = 0.0f;
  // staging: thread -> rows (tid >> 3) + 32 u, k quad (tid & 7)
  const int q4 = tid & 7, rr = tid >> 3;
  float4 rw[4], rd[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gr = min(tm + rr + 32 * u, m - 1);
      const int gi = min(tn + rr + 32 * u, k - 1);
      const int gk = k0 + 4 * q4;
      if (VEC) {  // n % 4 == 0: the four k of a quad are all in range or all out
        const int gkc = min(gk, n - 4);
        float4 w = *reinterpret_cast<const float4 *>(Wp + size_t(gr) * n + gkc);
        float4 d = *reinterpret_cast<const float4 *>(Dp + size_t(gr) * n + gkc);
        const double2 r0 = *reinterpret_cast<const double2 *>(Rx + size_t(gi) * ldr + gkc);
        const double2 r1 = *reinterpret_cast<const double2 *>(Rx + size_t(gi) * ldr + gkc + 2);
        float4 b = make_float4(float(r0.x), float(r0.y), float(r1.x), float(r1.y));  // :285
        if (gk >= n) w = d = b = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        rw[u] = w;
        rd[u] = d;
        rb[u] = b;
      } else {
        float t[3][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int gkc = min(gk + e, n - 1);
          const bool ok = gk + e < n;
          t[0][e] = ok ? Wp[size_t(gr) * n + gkc] : 0.0f;
          t[1][e] = ok ? Dp[size_t(gr) * n + gkc] : 0.0f;
          t[2][e] = ok ? float(Rx[size_t(gi) * ldr + gkc]) : 0.0f;  // R_x.to(float32)  :285
        }
        rw[u] = make_float4(t[0][0], t[0][1], t[0][2], t[0][3]);
        rd[u] = make_float4(t[1][0], t[1][1], t[1][2], t[1][3]);
        rb[u] = make_float4(t[2][0], t[2][1], t[2][2], t[2][3]);
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = rr + 32 * u;  // k = 4 q4 .. 4 q4 + 3: even (4q4, 4q4+2), odd (4q4+1, 4q4+3)
      *reinterpret_cast<float2 *>(&Aw[0][row][2 * q4]) = make_float2(rw[u].x, rw[u].z);
      *reinterpret_cast<float2 *>(&Aw[1][row][2 * q4]) = make_float2(rw[u].y, rw[u].w);
      *reinterpret_cast<float2 *>(&Ad[0][row][2 * q4]) = make_float2(rd[u].x, rd[u].z);
      *reinterpret_cast<float2 *>(&Ad[1][row][2 * q4]) = make_float2(rd[u].y, rd[u].w);
      *reinterpret_cast<float2 *>(&Bs[0][row][2 * q4]) = make_float2(rb[u].x, rb[u].z);
      *reinterpret_cast<float2 *>(&Bs[1][row][2 * q4]) = make_float2(rb[u].y, rb[u].w);
    }
  };
  gload(0);
  for (int k0 = 0; k0 < n; k0 += TK) {
    lstore();
    __syncthreads();
    if (k0 + TK < n) gload(k0 + TK);  // in flight during the MFMAs below
#pragma unroll
    for (int c = 0; c < TK / 8; ++c) {  // four MFMA k-steps per 16-B LDS read
      float4 xw[2], xd[2], xb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        xw[i] = *reinterpret_cast<const float4 *>(&Aw[h][wm * 64 + i * 32 + l32][4 * c]);
        xd[i] = *reinterpret_cast<const float4 *>(&Ad[h][wm * 64 + i * 32 + l32][4 * c]);
        xb[i] = *reinterpret_cast<const float4 *>(&Bs[h][wn * 64 + i * 32 + l32][4 * c]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            aw[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xw[i][e], xb[j][e], aw[i][j], 0, 0, 0);
            ad[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xd[i][e], xb[j][e], ad[i][j], 0, 0, 0);
          }
    }
    __syncthreads();
  }
  // squares of the valid outputs, FP64
  double sw = 0.0, sd = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gr = tm + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int gi = tn + wn * 64 + j * 32 + l32;
        const bool ok = gr < m && gi < k;
        const double vw = ok ? double(aw[i][j][r]) : 0.0, vd = ok ? double(ad[i][j][r]) : 0.0;
        sw += vw * vw;
        sd += vd * vd;
      }
  sw = wave_sum(sw);
  sd = wave_sum(sd);
  if (lane == 0) {
    red[0][wid] = sw;
    red[1][wid] = sd;
  }
  __syncthreads();
  if (tid == 0) {
    const int64_t b = int64_t(blockIdx.y) * gridDim.x + blockIdx.x;
    part[2 * b] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * b + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// out[0] = ||W_o R^T||_F^2, out[1] = ||(W_o - W_q) R^T||_F^2: partials added
// in a fixed order (lane-strided, then a fixed butterfly).
__global__ __launch_bounds__(64) void metric_sum_kernel(const double *__restrict__ part,
                                                        int64_t nb, double *__restrict__ out) {
  const int lane = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int64_t i = lane; i < nb; i += 64) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    out[0] = a;
    out[1] = b;
  }
}

template <class A>
void metric_layout(A &ar, int m, int n, int k, float **Wp, float **Dp, double **part) {
  const int64_t nb = int64_t(tg::cdiv(m, TM)) * tg::cdiv(k, TN);
  if constexpr (std::is_same_v<A, tg::Arena>) {
    *Wp = ar.template take<float>(size_t(m) * n);
    *Dp = ar.template take<float>(size_t(m) * n);
    *part = ar.template take<double>(size_t(2 * nb));
  } else {
    ar.template take<float>(size_t(m) * n);
    ar.template take<float>(size_t(m) * n);
    ar.template take<double>(size_t(2 * nb));
  }
}

}  // namespace

extern "C" size_t tg_pred_error_workspace_size(int m, int n, int k) {
  if (m < 1 || n < 1 || k < 1) return 0;
  tg::Sizer s;
  metric_layout(s, m, n, k, nullptr, nullptr, nullptr);
  return s.off + 256;
}

extern "C" int tg_pred_error(void *stream, const float *W, const float *Wq, int m, int n, int ldw,
                             const double *Rx, int k, int ldr, const int64_t *perm, double *out,
                             void *ws, size_t ws_bytes) {
  TG_ARG(W && Wq, 2, "null W / Wq");
  TG_ARG(m >= 1, 4, "m < 1");
  TG_ARG(n >= 1, 5, "n < 1");
  TG_ARG(ldw >= n, 6, "ldw < n");
  TG_ARG(Rx, 7, "null R_x");
  TG_ARG(k >= 1, 8, "k < 1");
  TG_ARG(ldr >= n, 9, "ldr < n");
  TG_ARG(perm, 10, "null perm");
  TG_ARG(out, 11, "null out");
  hipStream_t st = static_cast<hipStream_t>(stream);
  tg::Arena ar(ws, ws_bytes);
  float *Wp = nullptr, *Dp = nullptr;
  double *part = nullptr;
  metric_layout(ar, m, n, k, &Wp, &Dp, &part);
  TG_WS(ar);
  hipLaunchKernelGGL(metric_gather_kernel, dim3(std::min(16, tg::cdiv(n, 256)), m), dim3(256), 0,
                     st, W, Wq, n, ldw, perm, Wp, Dp);
  TG_LAUNCHED();
  const dim3 grid(tg::cdiv(k, TN), tg::cdiv(m, TM));
  // 16-B rows need n % 4 == 0 and 16-B aligned R_x rows (ldr even, R_x aligned)
  if (n % 4 == 0 && ldr % 2 == 0 && (reinterpret_cast<uintptr_t>(Rx) & 15) == 0)
    hipLaunchKernelGGL(metric_gemm_kernel<true>, grid, dim3(256), 0, st, Wp, Dp, m, n, Rx, ldr, k,
                       part);
  else
    hipLaunchKernelGGL(metric_gemm_kernel<false>, grid, dim3(256), 0, st, Wp, Dp, m, n, Rx, ldr,
                       k, part);
  TG_LAUNCHED();
  hipLaunchKernelGGL(metric_sum_kernel, dim3(1), dim3(64), 0, st, part,
                     int64_t(grid.x) * grid.y, out);
  TG_LAUNCHED();
  return 0;
}
