// kernels_fast.hip -- fast-mode DSGD sweep (f32), one rotation sub-step per launch.
//
// Schedule (plan.cpp build_fast_plan): a rating block is split into G item groups x G user
// groups; in sub-step t, wave g of a block sweeps cell (item group g, user group (g+t) mod G).
// No two waves of a launch share a user or item row (conflict-free batching), so plain loads
// and stores are race-free and kernel boundaries order the sub-steps.
//
// Inside a cell the ratings form one contiguous run per item: the item row lives in VGPRs
// for the whole run (hot items never leave registers), user rows are gathered D ratings
// ahead into a register ring and written back after their update.  A user that reappears
// within the ring window gets the fresh row forwarded register-to-register, so the wave's
// result equals the sequential sweep of its cell.
//
// Per update (k=128): dot (KPL FMAs + DPP row reduction + 4 readlanes), two axpy rows,
// one 512-B user-row gather and one 512-B scatter; B_f32(k) = 16k + 20 algorithmic bytes.
// HBM-bound: roofline = 8 TB/s / B_f32(k) updates/s.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

constexpr uint32_t kNone = 0xffffffffu;

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ float rlf(uint32_t v, int l) { return __uint_as_float(rl(v, l)); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 64 lanes, returned uniformly.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror: every lane holds its 16-lane row sum
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (a + b) + (c + d);
}

// Row access: lane holds elements [lane*KPL, lane*KPL + KPL).  FULL: k == 64*KPL (vector I/O).
template <int KPL, bool FULL>
__device__ __forceinline__ void load_row(const float* __restrict__ row, int lane, int k, float (&v)[KPL]) {
  if constexpr (FULL) {
    if constexpr (KPL == 1) {
      v[0] = row[lane];
    } else if constexpr (KPL == 2) {
      const float2 x = reinterpret_cast<const float2*>(row)[lane];
      v[0] = x.x; v[1] = x.y;
    } else {
#pragma unroll
      for (int c = 0; c < KPL; c += 4) {
        const float4 x = reinterpret_cast<const float4*>(row)[lane * (KPL / 4) + c / 4];
        v[c] = x.x; v[c + 1] = x.y; v[c + 2] = x.z; v[c + 3] = x.w;
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane * KPL + c;
      v[c] = f < k ? row[f] : 0.f;
    }
  }
}

template <int KPL, bool FULL>
__device__ __forceinline__ void store_row(float* __restrict__ row, int lane, int k, const float (&v)[KPL]) {
  if constexpr (FULL) {
    if constexpr (KPL == 1) {
      row[lane] = v[0];
    } else if constexpr (KPL == 2) {
      reinterpret_cast<float2*>(row)[lane] = make_float2(v[0], v[1]);
    } else {
#pragma unroll
      for (int c = 0; c < KPL; c += 4)
        reinterpret_cast<float4*>(row)[lane * (KPL / 4) + c / 4] = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane * KPL + c;
      if (f < k) row[f] = v[c];
    }
  }
}

template <int KPL, bool FULL>
__global__ __launch_bounds__(256) void k_fast_substep(const FastBlk* __restrict__ blks, int nblk, int G,
                                                      int t, const uint4* __restrict__ recs,
                                                      const int32_t* __restrict__ cell_off,
                                                      float* __restrict__ U, float* __restrict__ I,
                                                      const float* __restrict__ regI, int k, float eta) {
  constexpr int D = 4;  // user-row prefetch depth (register ring)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // blockIdx % nblk picks the rating block: with 8 blocks a block's waves share one XCD's L2.
  const int slot = static_cast<int>(blockIdx.x % static_cast<unsigned>(nblk));
  const int g = static_cast<int>(blockIdx.x / static_cast<unsigned>(nblk)) * 4 + wave;
  if (g >= G) return;
  const FastBlk d = blks[slot];
  if (d.rec_base < 0) return;
  const int32_t* off = cell_off + d.cell_base + static_cast<int64_t>(t) * G + g;
  const int64_t beg = d.rec_base + off[0];
  const int64_t end = d.rec_base + off[1];
  if (beg >= end) return;

  // Two 64-record chunks of the cell's record stream in VGPRs (lane l holds record cbase+l).
  int64_t cbase = beg;
  uint4 cur = make_uint4(kNone, kNone, 0u, 0u), nxt = cur;
  if (cbase + lane < end) cur = recs[cbase + lane];
  if (cbase + 64 + lane < end) nxt = recs[cbase + 64 + lane];

  // Prefetch ring (slot s holds the record to be processed at position ≡ s mod D).
  uint32_t ru[D], ri[D];
  float rr[D], rreg[D], rregi[D];
  bool rnew[D];
  float rp[D][KPL], rq[D][KPL];
  uint32_t last_item = kNone;

  float q[KPL];
  float regi = 0.f;
  uint32_t cur_item = kNone;

  auto fetch = [&](int64_t jj, uint32_t& u_o, uint32_t& i_o, float& r_o, float& reg_o, bool& new_o,
                   float& regi_o, float (&p_o)[KPL], float (&q_o)[KPL], uint32_t just_u,
                   const float (&just_p)[KPL]) {
    if (jj >= end) { u_o = kNone; i_o = kNone; new_o = false; return; }
    if (jj - cbase >= 128) {  // slide the record window by one chunk
      cur = nxt;
      cbase += 64;
      nxt = make_uint4(kNone, kNone, 0u, 0u);
      if (cbase + 64 + lane < end) nxt = recs[cbase + 64 + lane];
    }
    const int o = static_cast<int>(jj - cbase);
    const uint4 x = o < 64 ? cur : nxt;
    const int l = o & 63;
    u_o = rl(x.x, l);
    i_o = rl(x.y, l);
    r_o = rlf(x.z, l);
    reg_o = rlf(x.w, l);
    if (u_o == just_u) {
#pragma unroll
      for (int c = 0; c < KPL; ++c) p_o[c] = just_p[c];
    } else {
      load_row<KPL, FULL>(U + static_cast<size_t>(u_o) * k, lane, k, p_o);
    }
    new_o = i_o != last_item;
    if (new_o) {
      load_row<KPL, FULL>(I + static_cast<size_t>(i_o) * k, lane, k, q_o);
      regi_o = regI[i_o];
      last_item = i_o;
    }
  };

  {
    float dummy[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) dummy[c] = 0.f;
#pragma unroll
    for (int s = 0; s < D; ++s)
      fetch(beg + s, ru[s], ri[s], rr[s], rreg[s], rnew[s], rregi[s], rp[s], rq[s], kNone, dummy);
  }

  for (int64_t j0 = beg; j0 < end; j0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      const int64_t jj = j0 + s;
      if (jj < end) {
        if (rnew[s]) {  // a new item run starts: retire the old item row, adopt the prefetched one
          if (cur_item != kNone) store_row<KPL, FULL>(I + static_cast<size_t>(cur_item) * k, lane, k, q);
#pragma unroll
          for (int c = 0; c < KPL; ++c) q[c] = rq[s][c];
          regi = rregi[s];
          cur_item = ri[s];
        }
        float part = 0.f;
#pragma unroll
        for (int c = 0; c < KPL; ++c) part = fmaf(rp[s][c], q[c], part);
        const float e = rr[s] - wave_sum(part);
        float pn[KPL];
#pragma unroll
        for (int c = 0; c < KPL; ++c) {
          const float p = rp[s][c], qq = q[c];
          pn[c] = p - eta * (rreg[s] * p - e * qq);
          q[c] = qq - eta * (regi * qq - e * p);
        }
        const uint32_t u_now = ru[s];
        store_row<KPL, FULL>(U + static_cast<size_t>(u_now) * k, lane, k, pn);
        // forward the fresh user row to pending ring slots of the same user
#pragma unroll
        for (int s2 = 0; s2 < D; ++s2) {
          if (s2 != s && ru[s2] == u_now) {
#pragma unroll
            for (int c = 0; c < KPL; ++c) rp[s2][c] = pn[c];
          }
        }
        fetch(jj + D, ru[s], ri[s], rr[s], rreg[s], rnew[s], rregi[s], rp[s], rq[s], u_now, pn);
      }
    }
  }
  if (cur_item != kNone) store_row<KPL, FULL>(I + static_cast<size_t>(cur_item) * k, lane, k, q);
}

template <int KPL>
void fast_dispatch(hipStream_t st, dim3 grid, const FastBlk* blks, int nblk, int G, int t,
                   const FastRec* recs, const int32_t* off, float* U, float* I, const float* regI,
                   int k, float eta) {
  const uint4* r = reinterpret_cast<const uint4*>(recs);
  if (k == 64 * KPL)
    hipLaunchKernelGGL((k_fast_substep<KPL, true>), grid, dim3(256), 0, st, blks, nblk, G, t, r, off, U, I, regI, k, eta);
  else
    hipLaunchKernelGGL((k_fast_substep<KPL, false>), grid, dim3(256), 0, st, blks, nblk, G, t, r, off, U, I, regI, k, eta);
}

}  // namespace

void launch_fast_substep(hipStream_t st, const FastBlk* blks, int nblk, int G, int t,
                         const FastRec* recs, const int32_t* cell_off, float* U, float* I,
                         const float* regI, int k, float eta) {
  const dim3 grid(static_cast<unsigned>(nblk * ((G + 3) / 4)));
  if (k <= 64) fast_dispatch<1>(st, grid, blks, nblk, G, t, recs, cell_off, U, I, regI, k, eta);
  else if (k <= 128) fast_dispatch<2>(st, grid, blks, nblk, G, t, recs, cell_off, U, I, regI, k, eta);
  else if (k <= 256) fast_dispatch<4>(st, grid, blks, nblk, G, t, recs, cell_off, U, I, regI, k, eta);
  else fast_dispatch<8>(st, grid, blks, nblk, G, t, recs, cell_off, U, I, regI, k, eta);
}

}  // namespace mfhip
