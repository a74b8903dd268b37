// online_f32.hpp -- the f32 arithmetic of the online update SGDUpdater.nextFactors
// (core/FactorUpdater.scala:37-45: e = r - u.i; u' = u + lr e i; i' = i + lr e u), shared by the
// one-launch sweep (k_online_f32, kernels_online_sweep.hip) and the level-by-level replay
// (k_level / k_level_out, kernels_det.hip) so that the two stay bitwise equal.  Included inside
// namespace mfhip { namespace { ... } }.  k <= 256 (KPL <= 4 floats per lane); wider rows keep the
// sequential fold of seq_fold.hpp.
//
// The f64 path keeps the reference's exact order (a left fold, F2jBLAS.ddot).  The f32 path is the
// fast mode judged on its distance to the f64 oracle (tests/test_gpu_configs.py: 1e-4 relative
// per row), so its dot product is a fixed tree: each lane folds its own KPL products with fused
// multiply-adds, then the 64 lane partials are summed by a butterfly (two half swaps, four DPP
// row steps) -- ~10 dependent VALU operations instead of a 128-add chain.  The updates are fused
// multiply-adds.  The order is fixed, so the results are deterministic and equal in every kernel
// that includes this header.
#pragma once

// KPL = ceil(k / 64) elements per lane.  Lane l's elements of a row of k floats: FULL (k == 64 KPL,
// KPL = 1, 2 or 4) l*KPL + c, contiguous, so a row moves with one 4/8/16-B access per lane;
// otherwise l + 64 c (elements >= k are zero)
template <int KPL, bool FULL>
__device__ __forceinline__ int f32_elem(int lane, int c) {
  return FULL ? lane * KPL + c : lane + 64 * c;
}

template <int CTRL>
__device__ __forceinline__ float f32_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// The 64-lane sum of x, the same in every lane: lanes 0-31 + 32-63 (v_permlane32_swap), rows 0 +
// 1 and 2 + 3 (v_permlane16_swap), then within a row of 16: quad perm [1,0,3,2], [2,3,0,1], row
// half mirror, row mirror.
__device__ __forceinline__ float f32_wave_sum(float x) {
#pragma clang fp contract(off)
  const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float a = __uint_as_float(h[0]) + __uint_as_float(h[1]);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  s = s + f32_dpp<0xB1>(s);
  s = s + f32_dpp<0x4E>(s);
  s = s + f32_dpp<0x141>(s);
  s = s + f32_dpp<0x140>(s);
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s)));
}

template <int KPL>
__device__ __forceinline__ float f32_lane_dot(const float (&p)[KPL], const float (&q)[KPL]) {
#pragma clang fp contract(off)
  float part = p[0] * q[0];
#pragma unroll
  for (int c = 1; c < KPL; ++c) part = __builtin_fmaf(p[c], q[c], part);
  return part;
}

// le = lr * e, e = r - u.i (uniform); u' and i' in place of p and q
template <int KPL>
__device__ __forceinline__ void f32_sgd_next(float (&p)[KPL], float (&q)[KPL], float le) {
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const float pn = __builtin_fmaf(le, q[c], p[c]);
    q[c] = __builtin_fmaf(le, p[c], q[c]);
    p[c] = pn;
  }
}

__device__ __forceinline__ float f32_err(double r, float dot, float eta) {
#pragma clang fp contract(off)
  return eta * (static_cast<float>(r) - dot);
}
