// Device geometry the persistent kernels size their grids from.
#include <mutex>

#include "common.h"

namespace {

// every workgroup records its XCD: the largest id + 1 is the XCD count
__global__ void xcc_probe_kernel(unsigned *out) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  if (threadIdx.x == 0) atomicMax(out, x + 1);
}

}  // namespace

namespace tg {

XcdInfo xcd_info() {
  constexpr int MAXDEV = 64;
  static std::mutex mu;
  static XcdInfo cache[MAXDEV];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return XcdInfo{8, 32};
  std::lock_guard<std::mutex> lock(mu);
  if (cache[dev].xcds > 0) return cache[dev];
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu < 1)
    ncu = 256;
  int xcds = 8;
  unsigned *d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned)) == hipSuccess) {
    unsigned h = 0;
    if (hipMemset(d, 0, sizeof(unsigned)) == hipSuccess) {
      // a few workgroups per CU: every XCD receives some under any dispatch order
      hipLaunchKernelGGL(xcc_probe_kernel, dim3(4 * ncu), dim3(64), 0, 0, d);
      if (hipGetLastError() == hipSuccess &&
          hipMemcpy(&h, d, sizeof(unsigned), hipMemcpyDeviceToHost) == hipSuccess && h >= 1 &&
          h <= 16)
        xcds = int(h);
    }
    (void)hipFree(d);
  }
  cache[dev] = XcdInfo{xcds, std::max(1, ncu / xcds)};
  return cache[dev];
}

}  // namespace tg
