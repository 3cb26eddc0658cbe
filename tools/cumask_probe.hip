// CU-mask layout probe: for streams masked to 16 CU bits, report where
// workgroups run (XCC id, SE id, CU id from the hardware id registers): bit k
// selects a CU of XCD k % 8.  Then copy bandwidth on masked streams.
// Build: hipcc --offload-arch=gfx950 -O3 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ void where(unsigned *out) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x + 0] = xcc & 0xf;
    out[3 * blockIdx.x + 1] = (hw >> 13) & 0x7;  // SE_ID
    out[3 * blockIdx.x + 2] = (hw >> 8) & 0xf;   // CU_ID
  }
}

__global__ void copyk(const double4 *__restrict__ a, double4 *__restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    b[i] = a[i];
}

static float time_copy(hipStream_t s, const double4 *a, double4 *b, size_t n, int grid) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(copyk, dim3(grid), dim3(256), 0, s, a, b, n);
  (void)hipEventRecord(e0, s);
  for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(copyk, dim3(grid), dim3(256), 0, s, a, b, n);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, dev);
  printf("CUs %d\n", p.multiProcessorCount);
  unsigned *d;
  (void)hipMalloc(&d, 3 * 64 * sizeof(unsigned));
  const int nw = (p.multiProcessorCount + 31) / 32;
  // (single-bit masks leave XCDs without CUs: workgroups dispatched there may
  // never run, so every mask below keeps CUs on all eight XCDs)
  // 16 bits 0..15 (first word): where do 64 workgroups land?
  for (int first : {0, 8}) {
    std::vector<uint32_t> m(nw, 0u);
    for (int k = first; k < first + 16; ++k) m[k / 32] |= 1u << (k % 32);
    hipStream_t s;
    (void)hipExtStreamCreateWithCUMask(&s, nw, m.data());
    hipLaunchKernelGGL(where, dim3(16), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    unsigned h[48];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("bits %d..%d:", first, first + 15);
    for (int b = 0; b < 16; ++b) printf(" %u/%u/%u", h[3 * b], h[3 * b + 1], h[3 * b + 2]);
    printf("\n");
    (void)hipStreamDestroy(s);
  }
  // bandwidth of a copy kernel: default stream vs CU-masked streams
  {
    const size_t n = size_t(64) << 20;  // 64 Mi double4 = 2 GiB each way
    double4 *a, *b;
    (void)hipMalloc(&a, n * sizeof(double4));
    (void)hipMalloc(&b, n * sizeof(double4));
    (void)hipMemset(a, 0, n * sizeof(double4));
    hipStream_t s0;
    (void)hipStreamCreate(&s0);
    for (size_t ns : {size_t(1) << 19, size_t(1) << 21}) {  // short kernels: 1 element per thread
      const int grid = int(ns / 256);
      printf("short grid %5d default: %.4f ms\n", grid, time_copy(s0, a, b, ns, grid));
      for (int skip : {0, 16}) {
        std::vector<uint32_t> m(nw, 0u);
        for (int k = skip; k < p.multiProcessorCount; ++k) m[k / 32] |= 1u << (k % 32);
        hipStream_t s;
        (void)hipExtStreamCreateWithCUMask(&s, nw, m.data());
        printf("short grid %5d mask without bits [0,%d): %.4f ms\n", grid, skip, time_copy(s, a, b, ns, grid));
        (void)hipStreamDestroy(s);
      }
    }
    for (int grid : {1024, 4096, 16384}) {
      printf("grid %5d default: %.3f ms\n", grid, time_copy(s0, a, b, n, grid));
      for (int skip : {0, 16, 64}) {
        std::vector<uint32_t> m(nw, 0u);
        for (int k = skip; k < p.multiProcessorCount; ++k) m[k / 32] |= 1u << (k % 32);
        hipStream_t s;
        (void)hipExtStreamCreateWithCUMask(&s, nw, m.data());
        printf("grid %5d mask without bits [0,%d): %.3f ms\n", grid, skip, time_copy(s, a, b, n, grid));
        (void)hipStreamDestroy(s);
      }
    }
  }
  return 0;
}
