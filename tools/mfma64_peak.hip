// FP64 MFMA ceiling on this device and what co-issued work costs it:
// back-to-back v_mfma_f64_16x16x4_f64 on register operands (NACC independent
// accumulators per wave, no global memory traffic), WPS waves per SIMD,
// every CU busy, optionally with NV f16 -> f64 operand conversions per MFMA
// (the 16-bit SYRK's pattern) or NL ds_read_b64 per 8 MFMAs.  Prints TF/s and
// the in-kernel shader clock (s_memtime / s_memrealtime x 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma64_peak.hip -o tools/mfma64_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double doublex4 __attribute__((ext_vector_type(4)));

template <int WPS, int NACC, int NV, int NL>
__global__ __launch_bounds__(256 * WPS) void peak(double *out, long long *clk, int iters,
                                                  unsigned seed) {
  __shared__ double lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1.0 + i * 1e-6;
  __syncthreads();
  doublex4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = doublex4{0.0, 0.0, 0.0, 0.0};
  unsigned bits = seed ^ (threadIdx.x * 2654435761u);
  double a = 0.5 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      double av = a, bv = b;
      if (NV > 0) {  // operand from 16-bit bits: extract + cvt f16->f32->f64
        const unsigned h = (bits >> ((i & 1) * 16)) & 0xffffu;
        av = double(float(__builtin_bit_cast(_Float16, (unsigned short)h)));
        if (NV > 1) {
          const unsigned h2 = (bits >> (((i + 1) & 1) * 16)) & 0xffffu;
          bv = double(float(__builtin_bit_cast(_Float16, (unsigned short)h2)));
        }
      }
      if (NL > 0 && (i & 7) == 0) {
#pragma unroll
        for (int l = 0; l < NL; ++l) bits += __double_as_longlong(lds[(threadIdx.x + l * 64 + i) & 4095]);
      }
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i], 0, 0, 0);
    }
    bits = bits * 1664525u + 1013904223u;
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + bits;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int WPS, int NACC, int NV, int NL>
void run(int ncu, const char *what) {
  const int blocks = ncu, threads = 256 * WPS, iters = 64000 / NACC;
  double *out;
  long long *clk;
  (void)hipMalloc(&out, sizeof(double) * blocks * threads);
  (void)hipMalloc(&clk, sizeof(long long) * 2 * blocks);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  long long h[2] = {0, 1};
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((peak<WPS, NACC, NV, NL>), dim3(blocks), dim3(threads), 0, 0, out, clk,
                       iters, 12345u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    }
  }
  const double flops = 2.0 * 16 * 16 * 4 * double(NACC) * iters * (double(blocks) * threads / 64);
  printf("%-44s waves/SIMD %d acc %2d: %6.1f TF/s  clock %.2f GHz\n", what, WPS, NACC,
         flops / (best * 1e-3) / 1e12, double(h[0]) / double(h[1]) * 0.1);
  (void)hipFree(out);
  (void)hipFree(clk);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs: %d\n", ncu);
  run<1, 16, 0, 0>(ncu, "mfma only");
  run<2, 16, 0, 0>(ncu, "mfma only");
  run<2, 8, 0, 0>(ncu, "mfma only");
  run<4, 8, 0, 0>(ncu, "mfma only");
  run<3, 8, 0, 0>(ncu, "mfma only");
  run<2, 8, 1, 0>(ncu, "+1 f16->f64 operand per mfma");
  run<2, 8, 2, 0>(ncu, "+2 f16->f64 operands per mfma");
  run<4, 8, 2, 0>(ncu, "+2 f16->f64 operands per mfma");
  run<2, 8, 0, 6>(ncu, "+6 ds_read_b64 per 8 mfma");
  run<4, 8, 0, 6>(ncu, "+6 ds_read_b64 per 8 mfma");
  run<4, 8, 2, 6>(ncu, "+2 cvt/mfma +6 ds_read_b64 per 8");
  return 0;
}
