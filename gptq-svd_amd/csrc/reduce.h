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

// Partials are stored transposed: part[j * gridDim.x + blockIdx.x].
// Hand-off form (MI355X guide, "Valid forms", table row 1): every partial is
// stored write-through (agent-scope relaxed atomic store = global_store sc1),
// every storing wave drains vmcnt, a workgroup barrier, then ONE lane adds to
// the ticket; the last adder's workgroup reads every partial with sc1 loads
// (sum_partials).  No release/acquire fences (measured 2 us cheaper per
// reduction on MI355X, tools/redbench.hip).
__device__ inline bool publish_partials(const double *vals, int cnt, double *part,
                                        unsigned *counter) {
  __shared__ int s_last;
  const int tid = threadIdx.x;
  const int G = int(gridDim.x);
  for (int j = tid; j < cnt; j += blockDim.x)
    __hip_atomic_store(&part[size_t(j) * G + blockIdx.x], vals[j], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  return s_last != 0;
}

__device__ inline double load_partial(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum the published partials (call only in the last workgroup).  Wave w owns
// values j = w + nw*u (u < 5); its lanes cover partials g = lane + 64*s
// (s < 4) -- all loads of one batch are issued before any is used.  Each value
// is summed in a fixed order (per-lane in s, then a fixed butterfly), so the
// result is bit-reproducible.
__device__ inline void sum_partials(const double *part, int cnt, double *out, unsigned *counter) {
  constexpr int MJ = 5, MG = 4;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = int(blockDim.x >> 6);
  const int G = int(gridDim.x);
  for (int jb = 0; jb < cnt; jb += nw * MJ) {
    double acc[MJ];
#pragma unroll
    for (int u = 0; u < MJ; ++u) acc[u] = 0.0;
    for (int gb = 0; gb < G; gb += 64 * MG) {
      double v[MJ][MG];
#pragma unroll
      for (int u = 0; u < MJ; ++u)
#pragma unroll
        for (int s = 0; s < MG; ++s) {
          const int j = jb + wid + nw * u, g = gb + lane + 64 * s;
          v[u][s] = (j < cnt && g < G) ? load_partial(&part[size_t(j) * G + g]) : 0.0;
        }
#pragma unroll
      for (int u = 0; u < MJ; ++u)
#pragma unroll
        for (int s = 0; s < MG; ++s) acc[u] += v[u][s];
    }
#pragma unroll
    for (int u = 0; u < MJ; ++u) {
      double a = acc[u];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
      const int j = jb + wid + nw * u;
      if (lane == 0 && j < cnt) out[j] = a;
    }
  }
  if (threadIdx.x == 0) *counter = 0u;
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
