// kernels_fast.hip -- fast-mode DSGD sweep (f32).
//
// Schedule (plan.cpp build_fast_plan): a rating block is split into G item groups x G user
// groups; in rotation sub-step t, wave g of a block sweeps cell (item group g, user group
// (g+t) mod G).  Cells of one sub-step share no user or item row (conflict-free batching).
//
// Two drivers of the same schedule (identical results, bit for bit):
//  * k_fast_superstep (default): ONE persistent launch per superstep.  Wave g sweeps its G
//    cells in order; before cell t it waits until wave g+1 has finished cell t-1 -- the only
//    earlier user of user group (g+t) mod G in this superstep -- so the rotation runs as a
//    systolic pipeline instead of G grid-wide barriers, and a wave holding a hot item never
//    waits for the slowest cell of every sub-step.  Hand-off (MI355X_MICROARCH.md, Valid
//    forms, row 1): every user-row byte is stored and loaded with sc1 (write-through, L1
//    bypass), the wave drains with s_waitcnt vmcnt(0), then one lane stores the progress word
//    with an agent-scope relaxed atomic; the consumer polls that word with sc1 loads.  Each
//    workgroup is one wave.  Spins are bounded by s_memrealtime; a timeout sets err[0].
//  * k_fast_substep: one launch per sub-step (kernel boundaries order the sub-steps).
//
// Inside a cell the ratings form one contiguous run per item: the item row lives in VGPRs
// for the whole run (hot items never leave registers), user rows are gathered D ratings ahead
// into a register ring and written back after their update.  The host orders each cell so a
// user never repeats within the ring window (plan.cpp), so a wave's result equals the
// sequential sweep of its cell.
//
// Per update (k=128): dot (KPL FMAs + DPP row reduction + 4 readlanes), two axpy rows, one
// 512-B user-row gather and one 512-B scatter.  B_f32(k) = 16k + 20 algorithmic bytes.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kPad = kPadBit;

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ float rlf(uint32_t v, int l) { return __uint_as_float(rl(v, l)); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// ---- row I/O ------------------------------------------------------------------------------
// A lane holds elements [lane*KPL, lane*KPL + KPL) of a row.  FULL: k == 64*KPL (vector I/O);
// otherwise loads read a clamped in-row address and the k-tail is masked at use.  Rows are
// read and written through buffer descriptors; AUX = 16 sets sc1 (write-through stores,
// L1-bypassing loads) for rows handed between waves inside one launch.
template <int KPL>
struct Row {
  float v[KPL];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

// `off` is the row's byte offset in the slab (scalar, passed as soffset); the per-lane part of
// the address is a constant VGPR.
template <int KPL, bool FULL, int AUX>
__device__ __forceinline__ Row<KPL> load_row(__amdgpu_buffer_rsrc_t rs, uint32_t off, int lane, int k) {
  Row<KPL> r;
  if constexpr (FULL) {
    const uint32_t vo = static_cast<uint32_t>(lane) * KPL * 4u;
    if constexpr (KPL == 1) {
      r.v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, off, AUX));
    } else if constexpr (KPL == 2) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, off, AUX);
      r.v[0] = __uint_as_float(x[0]); r.v[1] = __uint_as_float(x[1]);
    } else {
#pragma unroll
      for (int c = 0; c < KPL; c += 4) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + c * 4u, off, AUX);
        r.v[c] = __uint_as_float(x[0]); r.v[c + 1] = __uint_as_float(x[1]);
        r.v[c + 2] = __uint_as_float(x[2]); r.v[c + 3] = __uint_as_float(x[3]);
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = min(lane * KPL + c, k - 1);  // clamped: the tail is masked at use
      r.v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<uint32_t>(f) * 4u, off, AUX));
    }
  }
  return r;
}

template <int KPL, bool FULL>
__device__ __forceinline__ void mask_row(Row<KPL>& r, int lane, int k) {
  if constexpr (!FULL) {
#pragma unroll
    for (int c = 0; c < KPL; ++c) r.v[c] = (lane * KPL + c < k) ? r.v[c] : 0.f;
  }
}

template <int KPL, bool FULL, int AUX>
__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t rs, uint32_t off, int lane, int k, const Row<KPL>& r) {
  if constexpr (FULL) {
    const uint32_t vo = static_cast<uint32_t>(lane) * KPL * 4u;
    if constexpr (KPL == 1) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[0]), rs, vo, off, AUX);
    } else if constexpr (KPL == 2) {
      using u2 = uint32_t __attribute__((ext_vector_type(2)));
      u2 x = {__float_as_uint(r.v[0]), __float_as_uint(r.v[1])};
      __builtin_amdgcn_raw_buffer_store_b64(x, rs, vo, off, AUX);
    } else {
      using u4 = uint32_t __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int c = 0; c < KPL; c += 4) {
        u4 x = {__float_as_uint(r.v[c]), __float_as_uint(r.v[c + 1]), __float_as_uint(r.v[c + 2]),
                __float_as_uint(r.v[c + 3])};
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, vo + c * 4u, off, AUX);
        // two wait states before the data VGPRs may be rewritten (gfx950 store-data hazard, pair_device.hpp)
        asm volatile("s_nop 1" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane * KPL + c;
      if (f < k) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[c]), rs, static_cast<uint32_t>(f) * 4u, off, AUX);
    }
  }
}

// Bounded wait until *flag >= want (sc1 polls).  Returns false on timeout (sets *err).
__device__ __forceinline__ bool wait_flag(const int32_t* flag, int32_t want, int32_t* err) {
  if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (true) {
    __builtin_amdgcn_s_sleep(8);  // ~0.25 us back-off between polls
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s: a wave never arrived
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// ---- record staging ----------------------------------------------------------------------
// A chunk is CH consecutive records of a cell, one per lane (lanes >= CH repeat them): the
// scalars of record y of the chunk are read with v_readlane at a compile-time lane.  a, b, er
// are the per-record update coefficients 1 - eta*ri, 1 - eta*ru and eta*r, computed once per
// chunk as vector ops.
constexpr int CH = 32;
struct Chunk {
  uint32_t u, i;     // row byte offsets
  float r, ru, ri;
  float a, b, er;
};

__device__ __forceinline__ void chunk_load(const uint32_t* __restrict__ recw, int64_t beg, int len, int c, int lane,
                                           Chunk& ch) {
  const int64_t x = beg + min(c * CH + (lane & (CH - 1)), len - 1);  // clamped: loads are unconditional
  const uint4 w = *reinterpret_cast<const uint4*>(recw + 8 * x);
  ch.u = w.x;
  ch.i = w.y;
  ch.r = __uint_as_float(w.z);
  ch.ru = __uint_as_float(w.w);
  ch.ri = __uint_as_float(recw[8 * x + 4]);
}
__device__ __forceinline__ void chunk_prep(Chunk& ch, float eta) {
  ch.a = fmaf(-eta, ch.ri, 1.f);
  ch.b = fmaf(-eta, ch.ru, 1.f);
  ch.er = eta * ch.r;
}

// Sum over the 64 lanes, returned uniformly.  Four DPP butterflies leave every lane with its
// 16-lane row sum; two row broadcasts fold the rows into lane 63.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return rlf(__float_as_uint(v), 63);
}

// Sequential sweep of one cell: `len` records starting at record `beg`.  Per step the wave
// issues the same memory operations unconditionally -- gathers of the user row and the item
// row of record j+D into a register ring, stores of the updated user and item rows of record
// j -- so the compiler's vmcnt waits stay counted (no control-flow join forces a drain).  The
// item row stays in VGPRs for its whole run and is written back every step; it is taken from
// the ring only when a new run starts (otherwise the ring reads a never-written dummy row, so
// no load trails a store to the row the run keeps updating).  The host keeps a user from
// recurring within kHazardWindow records of a cell (padding records are exact no-ops), so the
// prefetched user row is always current.  Update, per record (DSGDforMF.scala:405-410):
//   w = eta*(r - p.q);  p' = (1 - eta*ru) p + w q;  q' = (1 - eta*ri) q + w p.
template <int KPL, bool FULL, int D, int UAUX>
__device__ __forceinline__ void sweep_cell(int64_t beg, int len, const uint32_t* __restrict__ recw,
                                           __amdgpu_buffer_rsrc_t urs, __amdgpu_buffer_rsrc_t irs, int k,
                                           float eta, int lane, uint32_t dummy_u_off, uint32_t dummy_i_off) {
  static_assert(D <= kHazardWindow && D <= CH && CH % D == 0, "ring depth");
  uint32_t su[D], si[D];
  Row<KPL> rp[D], rq[D];
  Chunk A, B;
  chunk_load(recw, beg, len, 0, lane, A);
  chunk_load(recw, beg, len, 1, lane, B);
  chunk_prep(A, eta);
  uint32_t last_u = kNone, last_i = kNone;

  // A row that continues the previous record's run is forwarded in registers; its ring slot
  // reads a never-written dummy row instead (no load ever trails a store to a live row).
#define MF_FETCH(slot, X, y) MF_FETCH_AT(slot, rl(X.u, (y)), rl(X.i, (y)))
  // The offsets are read (v_readlane) at the top of a step and the loads issued after its
  // stores: named early, the readlanes no longer sit right before the buffer ops that take
  // them as soffset (an s_nop hazard wait each).
#define MF_FETCH_AT(slot, U_, I_)                                                             \
  do {                                                                                      \
    const uint32_t uo_ = (U_);                                                              \
    const uint32_t io_ = (I_);                                                              \
    su[slot] = uo_;                                                                         \
    si[slot] = io_;                                                                         \
    rp[slot] = load_row<KPL, FULL, UAUX>(urs, uo_ != last_u ? uo_ : dummy_u_off, lane, k);  \
    rq[slot] = load_row<KPL, FULL, 0>(irs, io_ != last_i ? io_ : dummy_i_off, lane, k);     \
    last_u = uo_;                                                                           \
    last_i = io_;                                                                           \
  } while (0)

#define MF_STEP(slot, X, y)                                                                 \
  do {                                                                                      \
    const uint32_t uo_ = su[slot], io_ = si[slot];                                          \
    const bool nr_ = io_ != cur_i, nu_ = uo_ != cur_u;                                      \
    cur_i = io_;                                                                            \
    cur_u = uo_;                                                                            \
    Row<KPL> p_ = rp[slot];                                                                 \
    mask_row<KPL, FULL>(p_, lane, k);                                                       \
    _Pragma("unroll") for (int e = 0; e < KPL; ++e) p_.v[e] = nu_ ? p_.v[e] : pl.v[e];      \
    Row<KPL> ql_ = rq[slot];                                                                \
    mask_row<KPL, FULL>(ql_, lane, k);                                                      \
    _Pragma("unroll") for (int e = 0; e < KPL; ++e) q.v[e] = nr_ ? ql_.v[e] : q.v[e];       \
    float part_ = 0.f;                                                                      \
    _Pragma("unroll") for (int e = 0; e < KPL; ++e) part_ = fmaf(p_.v[e], q.v[e], part_);   \
    const float w_ = fmaf(-eta, wave_sum(part_), rlf(__float_as_uint(X.er), (y)));          \
    const float a_ = rlf(__float_as_uint(X.a), (y)), b_ = rlf(__float_as_uint(X.b), (y));   \
    Row<KPL> pn_;                                                                           \
    _Pragma("unroll") for (int e = 0; e < KPL; ++e) {                                       \
      pn_.v[e] = fmaf(w_, q.v[e], b_ * p_.v[e]);                                            \
      q.v[e] = fmaf(w_, p_.v[e], a_ * q.v[e]);                                              \
    }                                                                                       \
    store_row<KPL, FULL, UAUX>(urs, uo_, lane, k, pn_);                                     \
    store_row<KPL, FULL, 0>(irs, io_, lane, k, q);                                          \
    pl = pn_;                                                                               \
  } while (0)

#pragma unroll
  for (int s = 0; s < D; ++s) MF_FETCH(s, A, s);

  Row<KPL> q, pl;  // the item row of the current run, the last updated user row
#pragma unroll
  for (int c = 0; c < KPL; ++c) q.v[c] = pl.v[c] = 0.f;
  uint32_t cur_i = kNone, cur_u = kNone;
  for (int base = 0;; base += 2 * CH) {
    // A holds records [base, base+CH) (prepared), B holds [base+CH, base+2CH)
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (base + s >= len) goto done;
      const uint32_t fu_ = s + D < CH ? rl(A.u, s + D) : rl(B.u, s + D - CH);
      const uint32_t fi_ = s + D < CH ? rl(A.i, s + D) : rl(B.i, s + D - CH);
      MF_STEP(s % D, A, s);
      MF_FETCH_AT(s % D, fu_, fi_);
    }
    chunk_prep(B, eta);
    chunk_load(recw, beg, len, base / CH + 2, lane, A);
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (base + CH + s >= len) goto done;
      const uint32_t fu_ = s + D < CH ? rl(B.u, s + D) : rl(A.u, s + D - CH);
      const uint32_t fi_ = s + D < CH ? rl(B.i, s + D) : rl(A.i, s + D - CH);
      MF_STEP(s % D, B, s);
      MF_FETCH_AT(s % D, fu_, fi_);
    }
    chunk_prep(A, eta);
    chunk_load(recw, beg, len, base / CH + 3, lane, B);
  }
done:
#undef MF_FETCH
#undef MF_FETCH_AT
#undef MF_STEP
  return;
}

// ---- one launch per sub-step ---------------------------------------------------------------
// amdgpu_waves_per_eu(1, 4): the register budget of 4 waves/SIMD lets the scheduler keep the
// ring loads D records ahead instead of sinking them toward their use to save VGPRs.
template <int KPL, bool FULL, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_fast_substep(
    const FastBlk* __restrict__ blks, int nblk, int G, int t, const uint32_t* __restrict__ recw,
    const int32_t* __restrict__ cell_off, float* __restrict__ U, float* __restrict__ I, int k, float eta,
    uint64_t u_bytes, uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int prio_len) {
  const int lane = threadIdx.x;
  // blockIdx % nblk picks the rating block: with 8 blocks a block's waves share one XCD's L2.
  const int slot = static_cast<int>(blockIdx.x % static_cast<unsigned>(nblk));
  const int g = static_cast<int>(blockIdx.x / static_cast<unsigned>(nblk));
  if (g >= G) return;
  const FastBlk d = blks[slot];
  if (d.rec_base < 0) return;
  const int32_t* off = cell_off + d.cell_base + static_cast<int64_t>(t) * G + g;
  const int64_t beg = d.rec_base + off[0];
  const int len = off[1] - off[0];
  if (len <= 0) return;
  // the longest cells set the sub-step's length: give their waves issue priority on the SIMD
  if (len >= prio_len) __builtin_amdgcn_s_setprio(3);
  sweep_cell<KPL, FULL, D, 0>(beg, len, recw, make_rsrc(U, u_bytes), make_rsrc(I, i_bytes), k, eta, lane,
                              dummy_u_off, dummy_i_off);
}

// ---- one persistent launch per superstep (systolic rotation) --------------------------------
template <int KPL, bool FULL, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_fast_superstep(
    const FastBlk* __restrict__ blks, int nblk, int G, const uint32_t* __restrict__ recw,
    const int32_t* __restrict__ cell_off, float* __restrict__ U, float* __restrict__ I, int k, float eta,
    uint64_t u_bytes, uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int32_t* __restrict__ progress,
    int32_t* __restrict__ err) {
  const int lane = threadIdx.x;
  const int slot = static_cast<int>(blockIdx.x % static_cast<unsigned>(nblk));
  const int g = static_cast<int>(blockIdx.x / static_cast<unsigned>(nblk));
  if (g >= G) return;
  const FastBlk d = blks[slot];
  if (d.rec_base < 0) return;  // empty rating block: nobody waits on it
  // one 128-B line per progress word: pollers of different waves never share a line
  int32_t* prog = progress + static_cast<int64_t>(slot) * G * kProgStride;
  const int32_t* off = cell_off + d.cell_base;
  const int32_t* next_prog = prog + static_cast<int64_t>(g + 1 == G ? 0 : g + 1) * kProgStride;
  const __amdgpu_buffer_rsrc_t urs = make_rsrc(U, u_bytes), irs = make_rsrc(I, i_bytes);
  for (int t = 0; t < G; ++t) {
    const int64_t cb = static_cast<int64_t>(t) * G + g;
    const int64_t beg = d.rec_base + off[cb];
    const int len = off[cb + 1] - off[cb];
    // user group (g+t) mod G was last swept by wave g+1 in sub-step t-1
    if (t > 0 && G > 1 && !wait_flag(next_prog, t, err)) return;
    if (len > 0) sweep_cell<KPL, FULL, D, 16>(beg, len, recw, urs, irs, k, eta, lane, dummy_u_off, dummy_i_off);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every user-row store of this wave has landed
    if (lane == 0) __hip_atomic_store(prog + static_cast<int64_t>(g) * kProgStride, t + 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int KPL, int D>
void fast_dispatch(hipStream_t st, dim3 grid, const FastBlk* blks, int nblk, int G, int t,
                   const FastRec* recs, const int32_t* off, float* U, float* I, int k, float eta, uint64_t ub,
                   uint64_t ib, uint32_t du, uint32_t di, int prio_len) {
  const uint32_t* r = reinterpret_cast<const uint32_t*>(recs);
  if (k == 64 * KPL)
    hipLaunchKernelGGL((k_fast_substep<KPL, true, D>), grid, dim3(64), 0, st, blks, nblk, G, t, r, off, U, I, k, eta, ub, ib, du, di, prio_len);
  else
    hipLaunchKernelGGL((k_fast_substep<KPL, false, D>), grid, dim3(64), 0, st, blks, nblk, G, t, r, off, U, I, k, eta, ub, ib, du, di, prio_len);
}

template <int KPL, int D>
void persistent_dispatch(hipStream_t st, const FastBlk* blks, int nblk, int G, const FastRec* recs,
                         const int32_t* off, float* U, float* I, int k, float eta, uint64_t ub, uint64_t ib,
                         uint32_t du, uint32_t di, int32_t* progress, int32_t* err) {
  const uint32_t* r = reinterpret_cast<const uint32_t*>(recs);
  const dim3 grid(static_cast<unsigned>(nblk * G)), block(64);
  if (k == 64 * KPL)
    hipLaunchKernelGGL((k_fast_superstep<KPL, true, D>), grid, block, 0, st, blks, nblk, G, r, off, U, I, k, eta, ub,
                       ib, du, di, progress, err);
  else
    hipLaunchKernelGGL((k_fast_superstep<KPL, false, D>), grid, block, 0, st, blks, nblk, G, r, off, U, I, k, eta, ub,
                       ib, du, di, progress, err);
}

}  // namespace

void launch_fast_substep(hipStream_t st, const FastBlk* blks, int nblk, int G, int t, const FastRec* recs,
                         const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                         uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int prio_len) {
  const dim3 grid(static_cast<unsigned>(nblk * G));
#define MF_ARGS st, grid, blks, nblk, G, t, recs, cell_off, U, I, k, eta, u_bytes, i_bytes, dummy_u_off, dummy_i_off, prio_len
  if (k <= 64) fast_dispatch<1, 8>(MF_ARGS);
  else if (k <= 128) fast_dispatch<2, 8>(MF_ARGS);
  else if (k <= 256) fast_dispatch<4, 8>(MF_ARGS);
  else fast_dispatch<8, 4>(MF_ARGS);
#undef MF_ARGS
}

void launch_fast_superstep(hipStream_t st, const FastBlk* blks, int nblk, int G, const FastRec* recs,
                           const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                           uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int32_t* progress,
                           int32_t* err) {
#define MF_ARGS st, blks, nblk, G, recs, cell_off, U, I, k, eta, u_bytes, i_bytes, dummy_u_off, dummy_i_off, progress, err
  if (k <= 64) persistent_dispatch<1, 8>(MF_ARGS);
  else if (k <= 128) persistent_dispatch<2, 8>(MF_ARGS);
  else if (k <= 256) persistent_dispatch<4, 8>(MF_ARGS);
  else persistent_dispatch<8, 4>(MF_ARGS);
#undef MF_ARGS
}

}  // namespace mfhip
