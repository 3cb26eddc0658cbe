// In-launch deterministic cross-workgroup reduction (last-arriver pattern).
//
// Each workgroup publishes `cnt` partial values; the workgroup whose ticket is
// last sums all partials in workgroup order (fixed order => bit-reproducible)
// and writes out[0..cnt).  Publication follows the agent-scope release /
// acquire recipe of the MI355X guide (cdna_hip_programming.md §5 "In-launch
// split-K reduction"): stores -> vmcnt(0) -> barrier -> lane-0 release fence
// -> vmcnt(0) -> relaxed agent ticket; the last arriver acquires before it
// reads.  The ticket counter must be zero before the first launch (the
// caller memsets it) and is reset by the last arriver.
#pragma once
#include <hip/hip_runtime.h>

namespace tg {

__device__ inline bool publish_partials(const double *vals, int cnt, double *part, int stride,
                                        unsigned *counter) {
  __shared__ int s_last;
  const int tid = threadIdx.x;
  for (int j = tid; j < cnt; j += blockDim.x) part[size_t(blockIdx.x) * stride + j] = vals[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return s_last != 0;
}

// Sum the published partials (call only in the last workgroup).
__device__ inline void sum_partials(const double *part, int stride, int cnt, double *out,
                                    unsigned *counter) {
  const int tid = threadIdx.x;
  for (int j = tid; j < cnt; j += blockDim.x) {
    double s = 0.0;
    for (int g = 0; g < int(gridDim.x); ++g) s += part[size_t(g) * stride + j];
    out[j] = s;
  }
  if (tid == 0) *counter = 0u;
}

// Block-wide sum of one double per thread into LDS slot (all threads get it).
__device__ inline double block_sum(double v, double *scratch /* >= 4 doubles */) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < int(blockDim.x >> 6); ++w) s += scratch[w];
  return s;
}

}  // namespace tg
