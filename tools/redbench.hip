// Microbenchmark: cost of an in-launch cross-workgroup reduction of CNT doubles
// per workgroup (the tridiagonalisation's per-column reduction), three ways:
//  A: plain stores + release fence + ticket + acquire + plain loads (guide recipe)
//  B: sc1 (write-through) stores + ticket, reducer reads with sc1 loads (no fences)
//  C: plain stores only (reduction left to the next launch)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int CNT = 65;
__device__ inline void reduce_all(const double* part, int G, double* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int j = wid; j < CNT; j += nw) {
    double v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) { int g = lane + 64 * s; v[s] = g < G ? part[j * G + g] : 0.0; }
    double a = 0; for (int s = 0; s < 8; ++s) a += v[s];
    for (int off = 32; off; off >>= 1) a += __shfl_xor(a, off);
    if (lane == 0) out[j] = a;
  }
}
__device__ inline void reduce_all_sc1(const double* part, int G, double* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int j = wid; j < CNT; j += nw) {
    double v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) { int g = lane + 64 * s;
      v[s] = g < G ? __hip_atomic_load(&part[j * G + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0; }
    double a = 0; for (int s = 0; s < 8; ++s) a += v[s];
    for (int off = 32; off; off >>= 1) a += __shfl_xor(a, off);
    if (lane == 0) out[j] = a;
  }
}
template <int MODE>
__global__ __launch_bounds__(1024) void kern(double* part, unsigned* cnt, double* out, int iter) {
  __shared__ int last;
  const int G = gridDim.x, tid = threadIdx.x;
  if (tid < CNT) {
    double v = double(blockIdx.x + 1) * (tid + 1) + iter;
    if (MODE == 1) __hip_atomic_store(&part[tid * G + blockIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else part[tid * G + blockIdx.x] = v;
  }
  if (MODE == 2) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (MODE == 0) { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1;
    if (last && MODE == 0) { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
  }
  __syncthreads();
  if (last) {
    if (MODE == 0) reduce_all(part, G, out); else reduce_all_sc1(part, G, out);
    if (tid == 0) *cnt = 0;
  }
}
__global__ void reducer(const double* part, int G, double* out) { reduce_all(part, G, out); }
int main() {
  for (int G : {64, 256, 512}) for (int T : {256, 1024}) {
    double *part, *out; unsigned* cnt;
    hipMalloc(&part, sizeof(double) * CNT * G); hipMalloc(&out, sizeof(double) * CNT); hipMalloc(&cnt, 64);
    hipMemset(cnt, 0, 64);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int N = 400;
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        for (int it = 0; it < N; ++it) {
          if (mode == 0) kern<0><<<G, T>>>(part, cnt, out, it);
          else if (mode == 1) kern<1><<<G, T>>>(part, cnt, out, it);
          else { kern<2><<<G, T>>>(part, cnt, out, it); reducer<<<1, 1024>>>(part, G, out); }
        }
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        std::vector<double> h(CNT); hipMemcpy(h.data(), out, sizeof(double) * CNT, hipMemcpyDeviceToHost);
        double exp0 = 0; for (int g = 0; g < G; ++g) exp0 += double(g + 1) * 1 + (N - 1);
        if (rep == 1) printf("G=%4d T=%4d mode=%d  %.2f us/launch-step  check %s\n", G, T, mode, ms * 1e3 / N, h[0] == exp0 ? "ok" : "BAD");
      }
    }
  }
  return 0;
}
