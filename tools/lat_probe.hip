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
  // 0: fma chain (also on the 100 MHz wall clock, to calibrate clock64)
  long long w0 = wall_clock64();
  c0 = clock64();
  for (int i = 0; i < 64 * N; ++i) x = fma(x, b, a);
  c1 = clock64(); t[0] = (c1 - c0) / 64; out[0] = x;
  t[7] = wall_clock64() - w0; t[8] = c1 - c0;
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
  // 5/6: the inverse-iteration dgttrf step (branch-free selects), without / with LDS stores
  __shared__ double st[4][256];
  for (int pass = 0; pass < 2; ++pass) {
    double cur_d = x, cur_u = a, xi = b;
    const double tol = 1e-300;
    c0 = clock64();
    for (int i = 0; i < N; ++i) {
      const double sub = 0.3 + (i & 7) * 0.1, nd = 1.1 - (i & 3) * 0.2, nu = 0.4, xnext = 1.0;
      const bool sw = !(fabs(cur_d) >= fabs(sub));
      const double cl = fabs(cur_d) < tol ? (cur_d < 0.0 ? -tol : tol) : cur_d;
      const double den = sw ? sub : cl, num = sw ? cur_d : sub;
      double r = __builtin_amdgcn_rcp(den);
      r = fma(fma(-den, r, 1.0), r, r);
      r = fma(fma(-den, r, 1.0), r, r);
      double q = num * r;
      const double f = fma(fma(-den, q, num), r, q);
      const double A = sw ? xi : xnext, B = sw ? xnext : xi;
      const double C = sw ? cur_u : nd, D = sw ? nd : cur_u;
      if (pass) {
        st[0][i & 255] = r; st[1][i & 255] = D; st[2][i & 255] = sw ? nu : 0.0; st[3][i & 255] = B;
      }
      xi = A - f * B;
      cur_d = C - f * D;
      cur_u = sw ? -f * nu : nu;
    }
    c1 = clock64(); t[5 + pass] = c1 - c0; out[5 + pass] = cur_d + xi + cur_u + st[1][3];
  }
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
  long long h[16];
  hipMemcpy(h, t, 9 * 8, hipMemcpyDeviceToHost);
  const char *nm[] = {"fma", "rcp+add", "cmp+sel(+mul/add)", "lds w+r+add", "mul", "dgttrf step", "dgttrf step+lds"};
  for (int i = 0; i < 7; ++i) printf("%-20s %.1f cycles/iter\n", nm[i], double(h[i]) / N);
  printf("fma chain: %lld wall ticks (10 ns) for %lld clock64 -> %.2f GHz\n", h[7], h[8], double(h[8]) / (h[7] * 10.0));
  return 0;
}
