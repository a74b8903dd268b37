// kernels_lean.hip -- fast-mode DSGD sweep, one wave per cell with a deep row prefetch (f32).
//
// Schedule: build_fast_plan's rotation (plan.cpp); sub-step t runs every cell (item group g,
// user group (g+t) mod G) of the superstep's rating blocks at once, one wave per cell, longest
// cells first (build_lean_plan).  Cells of a sub-step share no row: no atomics, no locks.
//
// Why this shape (measured): a cell is a dependent chain -- consecutive records
// of one item reuse the item row -- so a superstep lasts as long as its hottest item's chain
// (29k updates per NFLX superstep).  Each step's user row comes from HBM at ~1.2 us loaded
// latency, so the step time is max(issue time, latency / prefetch distance).  With k split
// over the 64 lanes a row costs KPL = k/64 VGPRs, which is what makes a D = 24 row ring fit
// in registers (a 16-lane split would need 4x as many).
//
// Per step j of a cell (records are uniform across the wave):
//  * record scalars come from a 64-record chunk held one record per lane (v_readlane);
//  * the user row of record j+D is loaded into ring slot j mod D -- unless the record continues
//    the previous user (forwarded in registers) -- and the item row of record j+D only when it
//    starts an item run; both are raw-buffer loads with the row's byte offset as the scalar
//    offset, skipped by a uniform branch;
//  * w = eta*(r - p.q) (DPP wave reduction), p' = (1 - eta*ru) p + w q, q' = (1 - eta*ri) q + w p
//    (DSGDforMF.scala:405-410); p' is stored, q' only at the end of its item run.
// Loads for record j+D are issued after the stores of record j, and the host keeps a row either
// adjacent (forwarded) or >= D records apart inside a cell (plan window), so every prefetched
// row is current.  vmcnt counts at most 63 operations: two per step (user load and store)
// bound D at ~30.
// B_f32(k) = 16k + 20 algorithmic bytes per update.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ float rlf(float v, int l) { return __uint_as_float(rl(__float_as_uint(v), l)); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 64 lanes, uniform result: four row butterflies, two row broadcasts into lane 63.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return rlf(v, 63);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xFFFFF000ull ? 0xFFFFF000u : static_cast<uint32_t>(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

template <int KPL>
struct Row {
  f2 v[KPL == 1 ? 1 : KPL / 2];
};

// Lane l holds floats [l*KPL, (l+1)*KPL) of a row; `off` (scalar) is the row's byte offset.
template <int KPL>
__device__ __forceinline__ Row<KPL> ld(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off) {
  Row<KPL> r;
  if constexpr (KPL == 1) {
    r.v[0] = f2{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, off, 0)), 0.f};
  } else if constexpr (KPL == 2) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, off, 0);
    r.v[0] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
  } else {
#pragma unroll
    for (int c = 0; c < KPL / 4; ++c) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u * c, off, 0);
      r.v[2 * c] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
      r.v[2 * c + 1] = f2{__uint_as_float(x[2]), __uint_as_float(x[3])};
    }
  }
  return r;
}

template <int KPL>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off, const Row<KPL>& r) {
  if constexpr (KPL == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[0].x), rs, voff, off, 0);
  } else if constexpr (KPL == 2) {
    using u2 = uint32_t __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(r.v[0].x), __float_as_uint(r.v[0].y)}, rs, voff, off, 0);
  } else {
#pragma unroll
    for (int c = 0; c < KPL / 4; ++c)
      __builtin_amdgcn_raw_buffer_store_b128(u4v{__float_as_uint(r.v[2 * c].x), __float_as_uint(r.v[2 * c].y),
                                                 __float_as_uint(r.v[2 * c + 1].x), __float_as_uint(r.v[2 * c + 1].y)},
                                             rs, voff + 16u * c, off, 0);
  }
}

// 64 consecutive records of the cell, record y in lane y (indices clamped to the cell).
struct Chunk {
  uint32_t ul, il, us, is;  // load / store byte offsets (kOffOOB: none)
  float er, a, b;           // eta*r, 1 - eta*ri, 1 - eta*ru
};

__device__ __forceinline__ void chunk_load(const u4v* __restrict__ R, int c, int len, int lane, float eta, Chunk& ch) {
  const int64_t x = min(c * 64 + lane, len - 1);
  const u4v A = R[2 * x], B = R[2 * x + 1];
  ch.ul = A[0];
  ch.il = A[1];
  ch.us = A[2];
  ch.is = A[3];
  ch.er = eta * __uint_as_float(B[0]);
  ch.b = fmaf(-eta, __uint_as_float(B[1]), 1.f);
  ch.a = fmaf(-eta, __uint_as_float(B[2]), 1.f);
}

template <int KPL, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_sweep_lean(
    const WaveDesc* __restrict__ waves, const u4v* __restrict__ recs, float* __restrict__ U, float* __restrict__ I,
    uint64_t u_bytes, uint64_t i_bytes, float eta, uint64_t* __restrict__ trace) {
  constexpr int NV = KPL == 1 ? 1 : KPL / 2;
  const int lane = threadIdx.x;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  const WaveDesc d = waves[blockIdx.x];
  const int len = d.steps;
  const u4v* R = recs + 2 * d.base;
  const uint32_t voff = static_cast<uint32_t>(lane) * KPL * 4u;
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);

  Chunk A, B;
  chunk_load(R, 0, len, lane, eta, A);
  chunk_load(R, 1, len, lane, eta, B);
  Row<KPL> P[D], Q[D];
  // prefetch of record y into slot y % D (skipped loads leave the slot stale; unused then)
#define MF_PREFETCH(slot, CH, YY)                                  \
  do {                                                            \
    const uint32_t uo_ = rl(CH.ul, (YY)), io_ = rl(CH.il, (YY));    \
    if (uo_ != kOffOOB) P[slot] = ld<KPL>(urs, voff, uo_);        \
    if (io_ != kOffOOB) Q[slot] = ld<KPL>(irs, voff, io_);        \
  } while (0)
#pragma unroll
  for (int s = 0; s < D; ++s) MF_PREFETCH(s, A, s);

  Row<KPL> q, pl;
#pragma unroll
  for (int e = 0; e < NV; ++e) q.v[e] = pl.v[e] = f2{0.f, 0.f};

#define MF_STEP(slot, CH, YY)                                                              \
  do {                                                                                    \
    const uint32_t ul_ = rl(CH.ul, (YY)), il_ = rl(CH.il, (YY));                            \
    const uint32_t us_ = rl(CH.us, (YY)), is_ = rl(CH.is, (YY));                            \
    const float er_ = rlf(CH.er, (YY)), a_ = rlf(CH.a, (YY)), b_ = rlf(CH.b, (YY));          \
    Row<KPL> p_;                                                                          \
    if (ul_ == kOffOOB) p_ = pl; else p_ = P[slot];                                       \
    if (il_ != kOffOOB) q = Q[slot];                                                      \
    f2 acc_ = p_.v[0] * q.v[0];                                                           \
    _Pragma("unroll") for (int e = 1; e < NV; ++e) acc_ = p_.v[e] * q.v[e] + acc_;        \
    const float w_ = fmaf(-eta, wave_sum(KPL == 1 ? acc_.x : acc_.x + acc_.y), er_);      \
    _Pragma("unroll") for (int e = 0; e < NV; ++e) {                                      \
      const f2 pe_ = p_.v[e];                                                             \
      pl.v[e] = b_ * pe_ + w_ * q.v[e];                                                   \
      q.v[e] = a_ * q.v[e] + w_ * pe_;                                                    \
    }                                                                                     \
    st<KPL>(urs, voff, us_, pl);                                                          \
    if (is_ != kOffOOB) st<KPL>(irs, voff, is_, q);                                       \
  } while (0)

  for (int c = 0;; c += 2) {
    // A holds records [64c, 64c+64), B the next 64
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      if (c * 64 + s >= len) goto done;
      MF_STEP(s % D, A, s);
      if (s + D < 64) MF_PREFETCH(s % D, A, s + D);
      else MF_PREFETCH(s % D, B, s + D - 64);
    }
    chunk_load(R, c + 2, len, lane, eta, A);
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      if ((c + 1) * 64 + s >= len) goto done;
      MF_STEP((64 + s) % D, B, s);
      if (s + D < 64) MF_PREFETCH((64 + s) % D, B, s + D);
      else MF_PREFETCH((64 + s) % D, A, s + D - 64);
    }
    chunk_load(R, c + 3, len, lane, eta, B);
  }
done:
#undef MF_PREFETCH
#undef MF_STEP
  if (trace && lane == 0) {
    trace[2 * blockIdx.x] = t_start;
    trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int KPL, int D>
void dispatch(hipStream_t st, const WaveDesc* waves, int nwaves, const StreamRec* recs, float* U, float* I,
              uint64_t ub, uint64_t ib, float eta, uint64_t* trace) {
  hipLaunchKernelGGL((k_sweep_lean<KPL, D>), dim3(static_cast<unsigned>(nwaves)), dim3(64), 0, st, waves,
                     reinterpret_cast<const u4v*>(recs), U, I, ub, ib, eta, trace);
}

}  // namespace

bool lean_kernel_supports(int k) { return k == 64 || k == 128 || k == 256; }
int lean_ring_depth(int k) { return k == 256 ? kLeanRingK256 : kLeanRing; }

void launch_sweep_lean(hipStream_t st, const WaveDesc* waves, int nwaves, const StreamRec* recs, float* U, float* I,
                       uint64_t u_bytes, uint64_t i_bytes, int k, float eta, uint64_t* trace) {
  if (nwaves <= 0) return;
  switch (k) {
    case 64: dispatch<1, kLeanRing>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace); break;
    case 128: dispatch<2, kLeanRing>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace); break;
    case 256: dispatch<4, kLeanRingK256>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace); break;
    default: break;
  }
}

}  // namespace mfhip
