#include <hip/hip_runtime.h>
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


__shared__ double Lt[32][33];
__shared__ double rinv[32];
__shared__ double Xs[256][34];
__global__ __launch_bounds__(256) void tk(double* out, int n) {
  for (int e = threadIdx.x; e < 1024; e += 256) Lt[e>>5][e&31] = out[e];
  if (threadIdx.x < 32) rinv[threadIdx.x] = out[threadIdx.x];
  for (int l = 0; l < 32; ++l) Xs[threadIdx.x][l] = out[threadIdx.x * 32 + l];
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < n; ++it) {
    double x[32];
    for (int l = 0; l < 32; ++l) x[l] = Xs[threadIdx.x][l];
    asm volatile("" ::: "memory");
    trsm_row(x, Lt, rinv);
    for (int l = 0; l < 32; ++l) Xs[threadIdx.x][l] = x[l];
  }
  uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  out[threadIdx.x] = Xs[threadIdx.x][5];
  if (threadIdx.x == 0) out[300] = double(t1 - t0);
}
int main() {
  double* d; hipMalloc(&d, 65536 * 8);
  hipMemset(d, 0, 65536*8);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(tk, dim3(1), dim3(256), 0, 0, d, 100); }
  double h[301]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("trsm_row: %.3f us per call (256 threads, 1 WG)\n", h[300] / 100.0 / 100.0);
  hipLaunchKernelGGL(tk, dim3(1), dim3(64), 0, 0, d, 100);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("trsm_row: %.3f us per call (64 threads)\n", h[300] / 100.0 / 100.0);
  return 0;
}
