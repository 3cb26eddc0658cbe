// Instruction-fetch probe: one wave runs K KB of straight-line code once
// (cold instruction cache) vs a 4 KB block looped (hot).  Prints cycles per
// 64-B line, to tell whether fully unrolled single-pass kernels are fetch bound.
// Build: hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o /tmp/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define STR2(x) #x
#define STR(x) STR2(x)

template <int KB>
__global__ void straight(unsigned long long *out) {
  const unsigned long long t0 = __builtin_readcyclecounter();
  asm volatile(".rept " STR(256) "*%c0\n s_nop 0\n .endr" ::"i"(KB));
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int KB>
__global__ void straight_valu(unsigned long long *out) {  // 8-B VOP3, 4 cycles each
  const unsigned long long t0 = __builtin_readcyclecounter();
  asm volatile(".rept " STR(128) "*%c0\n v_add_f32_e64 v1, v2, v3\n .endr" ::"i"(KB) : "v1");
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int KB>
__global__ void straight_salu(unsigned long long *out) {  // 4-B SOP1
  const unsigned long long t0 = __builtin_readcyclecounter();
  asm volatile(".rept " STR(256) "*%c0\n s_mov_b32 s0, 0\n .endr" ::"i"(KB) : "s0");
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int KB>
__global__ void hot_salu(unsigned long long *out) {
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < KB / 4; ++i) asm volatile(".rept 1024\n s_mov_b32 s0, 0\n .endr" ::: "s0");
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

__global__ void hot(unsigned long long *out, int reps) {
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < reps; ++i) asm volatile(".rept 1024\n s_nop 0\n .endr");
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <typename F>
static void run(const char *name, F launch, int kb, int blocks, unsigned long long *d) {
  unsigned long long h[256];
  for (int it = 0; it < 3; ++it) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    for (int i = 0; i < blocks; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("%-14s %4d KB blocks %3d it %d: %8llu cyc (%.1f cyc/line)  event %.1f us\n", name, kb,
           blocks, it, mx, double(mx) / (kb * 16.0), ms * 1e3);
  }
}

int main() {
  unsigned long long *d;
  hipMalloc(&d, 256 * sizeof(unsigned long long));
  for (int blocks : {1}) {
    run("hot_salu", [&] { hot_salu<64><<<blocks, 64>>>(d); }, 64, blocks, d);
    run("straight_salu", [&] { straight_salu<64><<<blocks, 64>>>(d); }, 64, blocks, d);
    run("straight_salu", [&] { straight_salu<128><<<blocks, 64>>>(d); }, 128, blocks, d);
  }
  for (int blocks : {1}) {
    run("hot 4KBx32", [&] { hot<<<blocks, 64>>>(d, 32); }, 128, blocks, d);
    run("straight", [&] { straight<16><<<blocks, 64>>>(d); }, 16, blocks, d);
    run("straight", [&] { straight<64><<<blocks, 64>>>(d); }, 64, blocks, d);
    run("straight", [&] { straight<128><<<blocks, 64>>>(d); }, 128, blocks, d);
    run("straight_valu", [&] { straight_valu<64><<<blocks, 64>>>(d); }, 64, blocks, d);
  }
  return 0;
}
