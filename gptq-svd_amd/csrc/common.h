// Shared helpers for the MI355X (gfx950) TruncGPTQ kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace tg {

void set_error(const char *fmt, ...);

// Carve aligned sub-buffers out of a caller workspace.
struct Arena {
  char *base;
  size_t cap, off = 0;
  Arena(void *p, size_t n) : base(static_cast<char *>(p)), cap(n) {}
  template <class T>
  T *take(size_t count) {
    off = (off + 255) & ~size_t(255);
    T *p = reinterpret_cast<T *>(base + off);
    off += count * sizeof(T);
    return p;
  }
  // absolute alignment (the buffer's address, not its offset): A - 1 bytes
  // of slack per call in the Sizer's count
  template <class T>
  T *take_aligned(size_t count, size_t A) {
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    off = ((b + off + A - 1) & ~uintptr_t(A - 1)) - b;
    T *p = reinterpret_cast<T *>(base + off);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

// Same layout arithmetic without a base pointer (for *_workspace_size()).
struct Sizer {
  size_t off = 0;
  template <class T>
  void take(size_t count) {
    off = (off + 255) & ~size_t(255);
    off += count * sizeof(T);
  }
  template <class T>
  void take_aligned(size_t count, size_t A) {
    off += A - 1 + count * sizeof(T);
  }
};

__host__ __device__ inline int cdiv(int64_t a, int64_t b) { return int((a + b - 1) / b); }

// Geometry of the current device (device.hip): XCD count (largest
// HW_REG_XCC_ID seen by a probe launch, + 1) and CUs per XCD; measured once
// per device and cached.
struct XcdInfo {
  int xcds = 0, cus_per_xcd = 0;
};
XcdInfo xcd_info();

// Sampled HIP-event timing of tagged kernel classes (tg_profile_* in the C ABI).
// A launch site calls prof_begin/prof_end around the launch on its stream; when
// profiling is on, every `every`-th launch of the class is bracketed by events
// and its algorithmic bytes / flops are recorded for roofline reporting.
enum ProfId { PROF_TRI_SYMV = 0, PROF_CROSS_GEMM = 1, PROF_QBLOCK = 2, PROF_SYR2K = 3,
              PROF_PIVSTEP = 4, PROF_BISECT = 5, PROF_INVIT = 6, PROF_BACKTR = 7,
              PROF_BULGE = 8, PROF_TSQR = 9, PROF_SBUPD = 10, PROF_Q1 = 11, PROF_Q2 = 12,
              PROF_N = 13 };
struct ProfTok {
  int id = -1;
  int slot = -1;
};
ProfTok prof_begin(hipStream_t st, int id, double bytes, double flops);
void prof_end(hipStream_t st, ProfTok tok);

// 16-bit Hessian SYRK (syrk.hip)
size_t syrk16_workspace_size(int n);
bool syrk16_supported(const void *X, int n, int64_t ldx);
hipError_t syrk16(hipStream_t st, const void *X, bool bf16, int64_t rows, int n, int64_t ldx,
                  double *H, int64_t ldh, void *ws);

}  // namespace tg

#define TG_ARG(cond, idx, msg)                                   \
  do {                                                           \
    if (!(cond)) {                                               \
      tg::set_error("%s: argument %d: %s", __func__, idx, msg); \
      return -(idx);                                             \
    }                                                            \
  } while (0)

#define TG_HIP(call)                                                                 \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) {                                                          \
      tg::set_error("%s: %s failed: %s", __func__, #call, hipGetErrorString(e_));    \
      return int(e_);                                                                \
    }                                                                                \
  } while (0)

#define TG_LAUNCHED() TG_HIP(hipGetLastError())

#define TG_WS(arena)                                                        \
  do {                                                                      \
    if (!(arena).ok()) {                                                    \
      tg::set_error("%s: workspace too small (%zu > %zu bytes)", __func__, \
                    (arena).off, (arena).cap);                              \
      return -99;                                                           \
    }                                                                       \
  } while (0)
