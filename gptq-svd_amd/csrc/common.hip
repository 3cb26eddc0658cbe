// Error reporting and small utility entry points of the C ABI.
#include <cstdarg>
#include <cstdio>

#include "../../include/truncgptq.h"
#include "common.h"

namespace tg {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tg

extern "C" const char *tg_last_error(void) { return tg::g_err; }
extern "C" int tg_version(void) { return 1; }

__global__ void scale_f64_kernel(const double *__restrict__ in, int64_t count, double s,
                                 double *__restrict__ out) {
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (; i < count; i += stride) out[i] = in[i] * s;
}

// HessianAccumulator.get_hessian: H / n_samples (gptq_utils.py:225-228).
// torch computes tensor / python-int as a true division; H * (1/N) differs in
// the last bit, so divide.
__global__ void div_f64_kernel(const double *__restrict__ in, int64_t count, double d,
                               double *__restrict__ out) {
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (; i < count; i += stride) out[i] = in[i] / d;
}

extern "C" int tg_scale_f64(void *stream, const double *H, int64_t count, double inv_n,
                            double *out) {
  TG_ARG(H != nullptr, 2, "null");
  TG_ARG(count >= 0, 3, "negative count");
  TG_ARG(out != nullptr, 5, "null");
  if (count == 0) return 0;
  int blocks = int(count / 256 + 1 < 4096 ? count / 256 + 1 : 4096);
  // inv_n < 0 encodes "divide by -inv_n" (exact get_hessian semantics).
  if (inv_n < 0)
    hipLaunchKernelGGL(div_f64_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, H, count,
                       -inv_n, out);
  else
    hipLaunchKernelGGL(scale_f64_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, H,
                       count, inv_n, out);
  TG_LAUNCHED();
  return 0;
}
