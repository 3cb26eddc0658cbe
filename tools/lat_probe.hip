// Latency probe: dependent FP64 op chains on one lane, timed with s_memtime
// (wall clock 100 MHz) and clock64 (shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
constexpr int N = 4096;
__global__ void probe(double *out, long long *t, double a, double b) {
  if (threadIdx.x != 0) return;
  double x = a;
  long long c0, c1;
  // 0: fma chain
  c0 = clock64();
  for (int i = 0; i < N; ++i) x = fma(x, b, a);
  c1 = clock64(); t[0] = c1 - c0; out[0] = x;
  // 1: rcp chain
  c0 = clock64();
  for (int i = 0; i < N; ++i) x = __builtin_amdgcn_rcp(x + a);
  c1 = clock64(); t[1] = c1 - c0; out[1] = x;
  // 2: compare + select chain
  c0 = clock64();
  for (int i = 0; i < N; ++i) x = fabs(x) >= b ? x * a : x + b;
  c1 = clock64(); t[2] = c1 - c0; out[2] = x;
  // 3: LDS write/read round trip chain
  __shared__ double s[64];
  c0 = clock64();
  for (int i = 0; i < N; ++i) { s[i & 63] = x; __builtin_amdgcn_s_waitcnt(0); x = s[(i + 0) & 63] + a; }
  c1 = clock64(); t[3] = c1 - c0; out[3] = x;
  // 4: mul chain
  c0 = clock64();
  for (int i = 0; i < N; ++i) x = x * b;
  c1 = clock64(); t[4] = c1 - c0; out[4] = x;
}
int main() {
  double *o; long long *t;
  hipMalloc(&o, 64 * 8); hipMalloc(&t, 64 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    probe<<<1, 64>>>(o, t, 0.5, 0.999);
    hipDeviceSynchronize();
  }
  long long h[8];
  hipMemcpy(h, t, 5 * 8, hipMemcpyDeviceToHost);
  const char *nm[] = {"fma", "rcp+add", "cmp+sel(+mul/add)", "lds w+r+add", "mul"};
  for (int i = 0; i < 5; ++i) printf("%-20s %.1f cycles/iter\n", nm[i], double(h[i]) / N);
  return 0;
}
