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

template <int KPL, bool FULL, int AUX>
__device__ __forceinline__ Row<KPL> load_row(__amdgpu_buffer_rsrc_t rs, uint32_t row, int lane, int k) {
  Row<KPL> r;
  const uint32_t base = row * static_cast<uint32_t>(k) * 4u;
  if constexpr (FULL) {
    const uint32_t off = base + static_cast<uint32_t>(lane) * KPL * 4u;
    if constexpr (KPL == 1) {
      r.v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, AUX));
    } else if constexpr (KPL == 2) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, AUX);
      r.v[0] = __uint_as_float(x[0]); r.v[1] = __uint_as_float(x[1]);
    } else {
#pragma unroll
      for (int c = 0; c < KPL; c += 4) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off + c * 4u, 0, AUX);
        r.v[c] = __uint_as_float(x[0]); r.v[c + 1] = __uint_as_float(x[1]);
        r.v[c + 2] = __uint_as_float(x[2]); r.v[c + 3] = __uint_as_float(x[3]);
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = min(lane * KPL + c, k - 1);  // clamped: the tail is masked at use
      r.v[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base + static_cast<uint32_t>(f) * 4u, 0, AUX));
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
__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t rs, uint32_t row, int lane, int k, const Row<KPL>& r) {
  const uint32_t base = row * static_cast<uint32_t>(k) * 4u;
  if constexpr (FULL) {
    const uint32_t off = base + static_cast<uint32_t>(lane) * KPL * 4u;
    if constexpr (KPL == 1) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[0]), rs, off, 0, AUX);
    } else if constexpr (KPL == 2) {
      using u2 = uint32_t __attribute__((ext_vector_type(2)));
      u2 x = {__float_as_uint(r.v[0]), __float_as_uint(r.v[1])};
      __builtin_amdgcn_raw_buffer_store_b64(x, rs, off, 0, AUX);
    } else {
      using u4 = uint32_t __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int c = 0; c < KPL; c += 4) {
        u4 x = {__float_as_uint(r.v[c]), __float_as_uint(r.v[c + 1]), __float_as_uint(r.v[c + 2]),
                __float_as_uint(r.v[c + 3])};
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off + c * 4u, 0, AUX);
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane * KPL + c;
      if (f < k) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[c]), rs, base + static_cast<uint32_t>(f) * 4u, 0, AUX);
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

// A record is 32 B = two uint4: {user row, item row | kPad, rating, lambda/omega_u} and
// {lambda/omega_i, 0, 0, 0}.  The first two 64-record chunks of a cell go through VGPRs.
__device__ __forceinline__ void stage_load(const uint4* __restrict__ recs, int64_t b, int64_t len, int lane,
                                           uint4 (&st)[4]) {
  const int64_t x0 = b + min<int64_t>(lane, len - 1), x1 = b + min<int64_t>(64 + lane, len - 1);
  st[0] = recs[2 * x0];
  st[1] = recs[2 * x0 + 1];
  st[2] = recs[2 * x1];
  st[3] = recs[2 * x1 + 1];
}
__device__ __forceinline__ void stage_store(uint4* lds, int lane, const uint4 (&st)[4]) {
  lds[2 * lane] = st[0];
  lds[2 * lane + 1] = st[1];
  lds[2 * (64 + lane)] = st[2];
  lds[2 * (64 + lane) + 1] = st[3];
}

// Sequential sweep of one cell: `len` records starting at recs[beg].  On entry the LDS
// double buffer (128 records) holds the cell's first two 64-record chunks; chunk c+2 streams in
// through VGPRs while chunk c is swept.  Every step issues the same memory operations
// unconditionally -- prefetch of the user row and the item row of record j+D, store of the
// updated user row and item row of record j -- so the compiler's vmcnt waits
// stay counted (no control-flow join ever forces a full drain).  The item row is kept in VGPRs
// across its run and written back every step (L2-resident); a record whose item differs from
// the previous one adopts the prefetched row.  Host-side the cell order guarantees that a user
// never repeats within kHazardWindow records (plan.cpp), and kPad records are no-ops (select,
// NaN-safe), so the prefetched user row is always the current one.
template <int KPL, bool FULL, int D, int UAUX>
__device__ __forceinline__ void sweep_cell(int64_t beg, int64_t len, const uint4* __restrict__ recs,
                                           uint4* lds, __amdgpu_buffer_rsrc_t urs, __amdgpu_buffer_rsrc_t irs,
                                           int k, float eta, int lane, uint32_t dummy_i,
                                           uint32_t dummy_u_store) {
  static_assert(D <= kHazardWindow && 64 % D == 0, "ring depth");
  uint32_t su[D], si[D];
  float sr[D], sru[D];
  bool spad[D];
  Row<KPL> rp[D], rq[D];
  float rri[D];  // lambda / omega_i of the record (uniform)

  // record of the next prefetch, read from LDS one step ahead of its use
  uint4 nrec;
  uint32_t nri;
#define MF_FETCH(s, idx)                                                                  \
  do {                                                                                    \
    const uint4 rec_ = nrec;                                                              \
    const uint32_t rri_ = nri;                                                            \
    nrec = lds[2 * (((idx) + 1) & 127)];                                                  \
    nri = lds[2 * (((idx) + 1) & 127) + 1].x;                                             \
    su[s] = __builtin_amdgcn_readfirstlane(rec_.x);                                       \
    const uint32_t iw_ = __builtin_amdgcn_readfirstlane(rec_.y);                          \
    si[s] = iw_ & ~kPad;                                                                  \
    spad[s] = (iw_ & kPad) != 0;                                                          \
    sr[s] = __uint_as_float(__builtin_amdgcn_readfirstlane(rec_.z));                      \
    sru[s] = __uint_as_float(__builtin_amdgcn_readfirstlane(rec_.w));                     \
    rri[s] = __uint_as_float(__builtin_amdgcn_readfirstlane(rri_));                       \
    rp[s] = load_row<KPL, FULL, UAUX>(urs, su[s], lane, k);                               \
    /* the item row is only needed when a new run starts; otherwise read the never-written \
       dummy row so no load ever trails a store to the row the run keeps updating */       \
    rq[s] = load_row<KPL, FULL, 0>(irs, si[s] != last_fetched ? si[s] : dummy_i, lane, k); \
    last_fetched = si[s];                                                                 \
  } while (0)

  uint32_t last_fetched = kNone;
  nrec = lds[0];
  nri = lds[1].x;
#pragma unroll
  for (int s = 0; s < D; ++s) MF_FETCH(s, s);

  Row<KPL> q;
#pragma unroll
  for (int c = 0; c < KPL; ++c) q.v[c] = 0.f;
  float regi = 0.f;
  uint32_t cur_i = kNone;
  int64_t idx = 0;
  for (int64_t c = 0;; ++c) {
    // chunk c+2 is staged now (clamped, unconditional) and written to LDS after chunk c; the
    // chunk's 64 steps are fully unrolled so the compiler counts vmcnt exactly across them.
    const bool more = (c + 2) * 64 < len;
    const int64_t sx = beg + min((c + 2) * 64 + lane, len - 1);
    const uint4 stage0 = recs[2 * sx], stage1 = recs[2 * sx + 1];
#pragma unroll
    for (int jb = 0; jb < 64; jb += D) {
#pragma unroll
      for (int s = 0; s < D; ++s) {
        if (idx >= len) goto done;
        const bool nr = si[s] != cur_i;
        cur_i = si[s];
        Row<KPL> p = rp[s];
        mask_row<KPL, FULL>(p, lane, k);
        Row<KPL> qi = rq[s];
        mask_row<KPL, FULL>(qi, lane, k);
#pragma unroll
        for (int e = 0; e < KPL; ++e) q.v[e] = nr ? qi.v[e] : q.v[e];
        regi = nr ? rri[s] : regi;
        float part = 0.f;
#pragma unroll
        for (int e = 0; e < KPL; ++e) part = fmaf(p.v[e], q.v[e], part);
        const float err = sr[s] - wave_sum(part);
        const bool pad = spad[s];
        Row<KPL> pn;
#pragma unroll
        for (int e = 0; e < KPL; ++e) {
          const float pv = p.v[e], qv = q.v[e];
          const float np = pv - eta * (sru[s] * pv - err * qv);
          const float nq = qv - eta * (regi * qv - err * pv);
          pn.v[e] = pad ? pv : np;
          q.v[e] = pad ? qv : nq;
        }
        // padding stores go to a second dummy row that is never loaded (no store->load trail)
        store_row<KPL, FULL, UAUX>(urs, pad ? dummy_u_store : su[s], lane, k, pn);
        store_row<KPL, FULL, 0>(irs, cur_i, lane, k, q);
        MF_FETCH(s, idx + D);
        ++idx;
      }
    }
    if (more) {
      lds[2 * ((c & 1) * 64 + lane)] = stage0;
      lds[2 * ((c & 1) * 64 + lane) + 1] = stage1;
    }
  }
done:
#undef MF_FETCH
  return;
}

// ---- one launch per sub-step ---------------------------------------------------------------
// amdgpu_waves_per_eu(1, 4): the register budget of 4 waves/SIMD lets the scheduler keep the
// ring loads D records ahead instead of sinking them toward their use to save VGPRs.
template <int KPL, bool FULL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_fast_substep(const FastBlk* __restrict__ blks, int nblk, int G,
                                                     int t, const uint4* __restrict__ recs,
                                                     const int32_t* __restrict__ cell_off,
                                                     float* __restrict__ U, float* __restrict__ I,
                                                     int k, float eta, uint64_t u_bytes, uint64_t i_bytes,
                                                     uint32_t dummy_i, uint32_t dummy_u_store, int prio_len) {
  __shared__ uint4 lds[256];
  const int lane = threadIdx.x;
  // blockIdx % nblk picks the rating block: with 8 blocks a block's waves share one XCD's L2.
  const int slot = static_cast<int>(blockIdx.x % static_cast<unsigned>(nblk));
  const int g = static_cast<int>(blockIdx.x / static_cast<unsigned>(nblk));
  if (g >= G) return;
  const FastBlk d = blks[slot];
  if (d.rec_base < 0) return;
  const int32_t* off = cell_off + d.cell_base + static_cast<int64_t>(t) * G + g;
  const int64_t beg = d.rec_base + off[0], len = off[1] - off[0];
  if (len <= 0) return;
  // the longest cells set the sub-step's length: give their waves issue priority on the SIMD
  if (len >= prio_len) __builtin_amdgcn_s_setprio(3);
  uint4 st[4];
  stage_load(recs, beg, len, lane, st);
  stage_store(lds, lane, st);
  sweep_cell<KPL, FULL, 8, 0>(beg, len, recs, lds, make_rsrc(U, u_bytes), make_rsrc(I, i_bytes), k, eta, lane,
                              dummy_i, dummy_u_store);
}

// ---- one persistent launch per superstep (systolic rotation) --------------------------------
template <int KPL, bool FULL, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_fast_superstep(const FastBlk* __restrict__ blks, int nblk, int G,
                                                       const uint4* __restrict__ recs,
                                                       const int32_t* __restrict__ cell_off,
                                                       float* __restrict__ U, float* __restrict__ I,
                                                       int k, float eta, uint64_t u_bytes, uint64_t i_bytes,
                                                       uint32_t dummy_i, uint32_t dummy_u_store,
                                                       int32_t* __restrict__ progress, int32_t* __restrict__ err) {
  __shared__ uint4 lds[256];
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
  // the first two record chunks of the next cell are staged in VGPRs one cell ahead
  uint4 st[4];
  {
    const int64_t l0 = off[g + 1] - off[g];
    if (l0 > 0) stage_load(recs, d.rec_base + off[g], l0, lane, st);
  }
  for (int t = 0; t < G; ++t) {
    const int64_t cb = static_cast<int64_t>(t) * G + g;
    const int64_t beg = d.rec_base + off[cb], len = off[cb + 1] - off[cb];
    if (len > 0) stage_store(lds, lane, st);
    if (t + 1 < G) {
      const int64_t nb = static_cast<int64_t>(t + 1) * G + g;
      const int64_t l1 = off[nb + 1] - off[nb];
      if (l1 > 0) stage_load(recs, d.rec_base + off[nb], l1, lane, st);
    }
    // user group (g+t) mod G was last swept by wave g+1 in sub-step t-1
    if (t > 0 && G > 1 && !wait_flag(next_prog, t, err)) return;
    if (len > 0) sweep_cell<KPL, FULL, D, 16>(beg, len, recs, lds, urs, irs, k, eta, lane, dummy_i, dummy_u_store);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every user-row store of this wave has landed
    if (lane == 0) __hip_atomic_store(prog + static_cast<int64_t>(g) * kProgStride, t + 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int KPL>
void fast_dispatch(hipStream_t st, dim3 grid, const FastBlk* blks, int nblk, int G, int t,
                   const FastRec* recs, const int32_t* off, float* U, float* I, int k, float eta, uint64_t ub,
                   uint64_t ib, uint32_t di, uint32_t du, int prio_len) {
  const uint4* r = reinterpret_cast<const uint4*>(recs);
  if (k == 64 * KPL)
    hipLaunchKernelGGL((k_fast_substep<KPL, true>), grid, dim3(64), 0, st, blks, nblk, G, t, r, off, U, I, k, eta, ub, ib, di, du, prio_len);
  else
    hipLaunchKernelGGL((k_fast_substep<KPL, false>), grid, dim3(64), 0, st, blks, nblk, G, t, r, off, U, I, k, eta, ub, ib, di, du, prio_len);
}

template <int KPL, int D>
void persistent_dispatch(hipStream_t st, const FastBlk* blks, int nblk, int G, const FastRec* recs,
                         const int32_t* off, float* U, float* I, int k, float eta, uint64_t ub, uint64_t ib,
                         uint32_t di, uint32_t du, int32_t* progress, int32_t* err) {
  const uint4* r = reinterpret_cast<const uint4*>(recs);
  const dim3 grid(static_cast<unsigned>(nblk * G)), block(64);
  if (k == 64 * KPL)
    hipLaunchKernelGGL((k_fast_superstep<KPL, true, D>), grid, block, 0, st, blks, nblk, G, r, off, U, I, k, eta, ub,
                       ib, di, du, progress, err);
  else
    hipLaunchKernelGGL((k_fast_superstep<KPL, false, D>), grid, block, 0, st, blks, nblk, G, r, off, U, I, k, eta, ub,
                       ib, di, du, progress, err);
}

}  // namespace

void launch_fast_substep(hipStream_t st, const FastBlk* blks, int nblk, int G, int t, const FastRec* recs,
                         const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                         uint64_t i_bytes, uint32_t dummy_i, uint32_t dummy_u_store, int prio_len) {
  const dim3 grid(static_cast<unsigned>(nblk * G));
#define MF_ARGS st, grid, blks, nblk, G, t, recs, cell_off, U, I, k, eta, u_bytes, i_bytes, dummy_i, dummy_u_store, prio_len
  if (k <= 64) fast_dispatch<1>(MF_ARGS);
  else if (k <= 128) fast_dispatch<2>(MF_ARGS);
  else if (k <= 256) fast_dispatch<4>(MF_ARGS);
  else fast_dispatch<8>(MF_ARGS);
#undef MF_ARGS
}

void launch_fast_superstep(hipStream_t st, const FastBlk* blks, int nblk, int G, const FastRec* recs,
                           const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                           uint64_t i_bytes, uint32_t dummy_i, uint32_t dummy_u_store, int32_t* progress,
                           int32_t* err) {
#define MF_ARGS st, blks, nblk, G, recs, cell_off, U, I, k, eta, u_bytes, i_bytes, dummy_i, dummy_u_store, progress, err
  if (k <= 64) persistent_dispatch<1, 8>(MF_ARGS);
  else if (k <= 128) persistent_dispatch<2, 8>(MF_ARGS);
  else if (k <= 256) persistent_dispatch<4, 8>(MF_ARGS);
  else persistent_dispatch<8, 4>(MF_ARGS);
#undef MF_ARGS
}

}  // namespace mfhip
