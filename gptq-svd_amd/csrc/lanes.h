// Cross-lane helpers for 64-wide wavefronts (gfx950), without the LDS
// crossbar: v_permlane{32,16}_swap and DPP row mirrors / quad permutes.
#pragma once
#include <hip/hip_runtime.h>

namespace tg {
namespace lanes {

template <int CTRL>
__device__ inline double xdpp(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
constexpr int DPP_MIRROR = 0x140, DPP_HALF_MIRROR = 0x141, DPP_XOR3 = 0x1B, DPP_XOR1 = 0xB1;

// x of lane l (l uniform) in every lane, through two v_readlane_b32.
__device__ inline double rl(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}

// v_permlane{32,16}_swap(a, b) exchanges the upper half of `a` with the lower
// half of `b`; the two results are lane-aligned, so their sum is the pairwise
// sum of `a` in the lower half and of `b` in the upper half (no selects).
__device__ inline double rs_swap32(double a, double b) {
  const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
__device__ inline double rs_swap16(double a, double b) {
  const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}

// Column whose wave sum a lane holds after reduce_scatter32 (lanes l and
// l ^ 1 hold the same column).
__device__ inline int rs_col(int lane) {
  return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 +
         ((lane >> 2) & 1) * 2 + ((lane >> 1) & 1);
}

// Wave reduce-scatter of 32 per-lane values: lane ends with the wave sum of
// p[rs_col(lane)].  p is clobbered.
__device__ inline double reduce_scatter32(double (&p)[32], int lane) {
#pragma unroll
  for (int k = 0; k < 16; ++k) p[k] = rs_swap32(p[k], p[k + 16]);
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = rs_swap16(p[k], p[k + 8]);
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double recv = xdpp<DPP_MIRROR>(up ? p[k] : p[k + 4]);
      p[k] = (up ? p[k + 4] : p[k]) + recv;
    }
  }
  {
    const bool up = (lane & 4) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double recv = xdpp<DPP_HALF_MIRROR>(up ? p[k] : p[k + 2]);
      p[k] = (up ? p[k + 2] : p[k]) + recv;
    }
  }
  {
    const bool up = (lane & 2) != 0;
    const double recv = xdpp<DPP_XOR3>(up ? p[0] : p[1]);
    p[0] = (up ? p[1] : p[0]) + recv;
  }
  return p[0] + xdpp<DPP_XOR1>(p[0]);
}

}  // namespace lanes
}  // namespace tg
