// Bounded spin-waits of the persistent kernels (bulge chasing, panel QR, the
// few-vector back-transform, the pivot steps).
//
// Every persistent launch owns one STALL word in device memory (zeroed by the
// host before the launch, read back after it).  A waiter that runs past its
// timeout sets the word; every other wait of the launch also polls the word
// and gives up as soon as it is set, so a stalled launch drains after ONE
// timeout instead of one timeout per remaining wait (the caller reports the
// stall and poisons its outputs).  A wait that gives up returns false.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace tg {

typedef __attribute__((address_space(1))) unsigned spin_u32;

// Relaxed agent-scope (sc1, L1-bypassing) load / store of a control word.
__device__ __forceinline__ unsigned ctl_load(const unsigned *p) {
  return __hip_atomic_load((spin_u32 *)const_cast<unsigned *>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ctl_store(unsigned *p, unsigned v) {
  __hip_atomic_store((spin_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Give-up path of a bounded wait: mark the launch's stall word.  An atomic OR
// (not a store), so tools/check_handoff_isa.py can tell it from the
// hand-off signals, which must follow a drain of the signalling wave's stores.
__device__ __forceinline__ void stall_set(unsigned *p) {
  (void)__hip_atomic_fetch_or((spin_u32 *)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Words no wave of the launch waits on -- a ticket counter reset by its last
// user for the next launch, a path record the host reads afterwards -- are
// written by an atomic exchange, so the hand-off check can tell them from
// signals too.
__device__ __forceinline__ void ctl_reset(unsigned *p) {
  (void)__hip_atomic_exchange((spin_u32 *)p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ctl_record(unsigned *p, unsigned v) {
  (void)__hip_atomic_exchange((spin_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until *word >= target.  Called by EVERY lane of a wave (the lanes
// load the same word in one request and the value is made scalar), so the
// loop and its exits are wave-uniform scalar branches: no exec-masked loop
// with divergent exits inside the callers' barrier loops.  `timeout` is in
// ticks of the 100 MHz s_memrealtime clock.  The last value seen goes to
// *seen when non-null.
__device__ inline bool spin_geq(const unsigned *word, unsigned target, unsigned *stall,
                                unsigned long long timeout, unsigned *seen = nullptr) {
  unsigned v = __builtin_amdgcn_readfirstlane(ctl_load(word));
  bool ok = true;
  if (v < target) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0;; ++it) {
      __builtin_amdgcn_s_sleep(1);
      v = __builtin_amdgcn_readfirstlane(ctl_load(word));
      if (v >= target) break;
      if ((it & 31u) == 31u) {  // short waits never pay for these reads
        if (__builtin_amdgcn_readfirstlane(ctl_load(stall)) != 0u) {
          ok = false;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
          stall_set(stall);
          ok = false;
          break;
        }
      }
    }
  }
  if (seen) *seen = v;
  // acquire edge for the compiler: no load of the caller moves above the poll
  // (no instruction: the hand-offs behind these waits are read with sc1 loads
  // from the one L2 they were stored to, or behind a workgroup barrier the
  // polling wave joins -- see each caller and tools/check_handoff_isa.py)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok;
}

// One arrival on a counter, called by a whole wave: lane 0 adds 1 (a plain
// lane-0 `if` around the one atomic: with a per-lane 1 / 0 value the atomic
// optimizer would scan the wave lane by lane).  No return value: the add is
// fire-and-forget and the caller's poll of the same word starts at once.
// Keep such lane-0 blocks away from loop headers and latches: a pair of them
// there let the CFG structurizer run lane 0 through a loop nest of its own
// (bulge.hip); the waits themselves are whole-wave loops (spin_geq).
__device__ __forceinline__ void wave_arrive(unsigned *cnt) {
  if (__lane_id() == 0)
    (void)__hip_atomic_fetch_add((spin_u32 *)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Host: spin timeout of the persistent kernels, in 100 MHz ticks.  Every wait
// in them is one pipeline step or one grid barrier (microseconds), so the
// default of 2 s only ever fires on a real stall; TG_SPIN_TIMEOUT_MS
// overrides it, the per-kernel variables (TG_BULGE_TIMEOUT_TICKS, ...) too.
inline unsigned long long spin_timeout_ticks(const char *kernel_env) {
  if (kernel_env) {
    const char *t = getenv(kernel_env);
    if (t) return strtoull(t, nullptr, 10);
  }
  const char *ms = getenv("TG_SPIN_TIMEOUT_MS");
  return ms ? strtoull(ms, nullptr, 10) * 100000ull : 200000000ull;
}

}  // namespace tg
