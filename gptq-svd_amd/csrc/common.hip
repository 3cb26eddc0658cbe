// Error reporting and small utility entry points of the C ABI.
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <vector>

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

namespace tg {
struct ProfClass {
  std::vector<hipEvent_t> ev;  // pairs
  std::vector<double> bytes, flops;
  int64_t launches = 0;
  int used = 0;
};
static std::mutex g_prof_mu;
static int g_prof_on = 0, g_prof_every = 1;
static ProfClass g_prof[PROF_N];

ProfTok prof_begin(hipStream_t st, int id, double bytes, double flops) {
  ProfTok t;
  if (!g_prof_on || id < 0 || id >= PROF_N) return t;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfClass &c = g_prof[id];
  const int64_t n = c.launches++;
  if (n % g_prof_every) return t;
  if (c.used * 2 + 2 > int(c.ev.size())) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return t;
    c.ev.push_back(a);
    c.ev.push_back(b);
    c.bytes.push_back(0);
    c.flops.push_back(0);
  }
  t.id = id;
  t.slot = c.used++;
  c.bytes[t.slot] = bytes;
  c.flops[t.slot] = flops;
  (void)hipEventRecord(c.ev[2 * t.slot], st);
  return t;
}

void prof_end(hipStream_t st, ProfTok tok) {
  if (tok.id < 0) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  (void)hipEventRecord(g_prof[tok.id].ev[2 * tok.slot + 1], st);
}
}  // namespace tg

extern "C" const char *tg_last_error(void) { return tg::g_err; }

// Profiling control: on != 0 enables sampling of every `every`-th launch per class.
extern "C" int tg_profile_enable(int on, int every) {
  std::lock_guard<std::mutex> lk(tg::g_prof_mu);
  tg::g_prof_on = on;
  tg::g_prof_every = every > 0 ? every : 1;
  return 0;
}

extern "C" int tg_profile_reset(void) {
  std::lock_guard<std::mutex> lk(tg::g_prof_mu);
  for (auto &c : tg::g_prof) {
    c.used = 0;
    c.launches = 0;
  }
  return 0;
}

// Sums over the sampled launches of class `id`: kernel ms, launches sampled,
// algorithmic bytes and flops; `total_launches` counts every launch of the class.
extern "C" int tg_profile_query(int id, double *ms, int64_t *sampled, double *bytes, double *flops,
                                int64_t *total_launches) {
  if (id < 0 || id >= tg::PROF_N) return -1;
  std::lock_guard<std::mutex> lk(tg::g_prof_mu);
  tg::ProfClass &c = tg::g_prof[id];
  double t = 0, b = 0, f = 0;
  for (int s = 0; s < c.used; ++s) {
    (void)hipEventSynchronize(c.ev[2 * s + 1]);
    float e = 0;
    (void)hipEventElapsedTime(&e, c.ev[2 * s], c.ev[2 * s + 1]);
    t += e;
    b += c.bytes[s];
    f += c.flops[s];
  }
  *ms = t;
  *sampled = c.used;
  *bytes = b;
  *flops = f;
  *total_launches = c.launches;
  return 0;
}
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
