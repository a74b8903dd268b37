// kernels_pair.hip -- fast-mode DSGD sweep, two updates of one item per step (f32).
//
// Schedule: build_fast_plan's rotation (plan.cpp); sub-step t runs every cell (item group g,
// user group (g+t) mod G) of the superstep's rating blocks at once, one wave per cell, longest
// first (build_pair_plan).  Cells of a sub-step share no row: no atomics, no locks.
//
// A cell is a dependent chain through its item rows, and the hottest item's chain (29k
// updates per NFLX superstep) sets the superstep's length.  One sequential SGD update costs a
// 64-lane reduction on that chain.  Here a step applies two consecutive updates A, B of the
// same item q (distinct users pA, pB) with ONE reduction round, using
//   eA = rA - pA.q
//   q1 = aA q + wA pA                               (wA = eta*eA, aA = 1 - eta*ri)
//   eB = rB - pB.q1 = rB - (aA pB.q + wA pB.pA)
// so the three dot products pA.q, pB.q, pB.pA are reduced together and only scalar work
// separates them; the rows are then updated exactly as two sequential steps would:
//   pA' = bA pA + wA q,  pB' = bB pB + wB q1,  q2 = aB q1 + wB pB   (DSGDforMF.scala:405-410).
// A "split" pair (B on another item qB: A's run ends, B's starts) is the same step with the
// coupling switched off: eB = rB - pB.qB, pB' = bB pB + wB qB, qB' = aB qB + wB pB.  The
// result equals the sequential order up to f32 rounding.
//
// Memory: every step issues the same eight vector-memory operations (user rows of A and B,
// item rows of A and B, and their stores) with raw-buffer scalar offsets; a row that must not
// be touched gets an offset past the slab (kOffOOB: the load returns zeros, the store is
// dropped), which is also how forwarded rows and no-op records are expressed.  Rows of pair
// j+D are loaded after the stores of pair j; the host keeps every row adjacent (forwarded in
// registers) or at least 2D records apart inside a cell (plan window), so a prefetched row is
// always current.  8 operations x D pairs stay under vmcnt's 63 (D = plan.hpp pair_ring: 4 or 6).  A cell that is a single
// item run (hot items) takes a leaner loop with no item traffic at all.
// B_f32(k) = 16k + 20 algorithmic bytes per update.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <utility>

#include "kernels.hpp"

namespace mfhip {
namespace {

#include "pair_device.hpp"

// experiment: explicit agent-scope acquire / release around a launch (L2 invalidate / write-back)
#ifdef MFHIP_EXP_FENCES
#define MF_LAUNCH_ACQUIRE() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent")
#define MF_LAUNCH_RELEASE() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent")
#else
#define MF_LAUNCH_ACQUIRE() ((void)0)
#define MF_LAUNCH_RELEASE() ((void)0)
#endif

#ifdef MFHIP_EXP_ITEM_SC1
constexpr int kItemPolicy = kSC1;
#else
constexpr int kItemPolicy = 0;
#endif

// A cell that is one item run (build_pair_plan): the item row stays in registers from the first
// pair to the last, so a pair moves no item row, only user rows (4 VMEM operations).  B's user row
// is stored where it was loaded from (its offset rides an SGPR ring).  FWD = false: so is A's (no
// user repeats at the next record: kWaveSingleRun); FWD = true (kWaveSingleRunFwd): A's row may be
// the previous pair's result (a user rating the item twice in a row), forwarded in registers.
// IP = cache policy of the item-row accesses (kItemPolicy)
template <int KPL, int UP, bool FWD, int IP = kItemPolicy>
__device__ __forceinline__ void single_run_cell(Chunk C0, __amdgpu_buffer_rsrc_t RR,
                                                __amdgpu_buffer_rsrc_t urs, __amdgpu_buffer_rsrc_t irs, float eta,
                                                uint32_t vlane, uint32_t voff, int npairs, uint64_t& wait_clk) {
  (void)wait_clk;
  constexpr int NV = Row<KPL>::NV;
  constexpr int CH = pair_chunk(KPL);
  constexpr int DS = pair_ring(KPL);
  const uint32_t item_off = rl(C0.ia, 0);
  Row<KPL> q = ld<KPL, IP>(irs, voff, item_off);
  Row<KPL> RA[DS], RB[DS], plA, plB;
#pragma unroll
  for (int e = 0; e < NV; ++e) plA.v[e] = plB.v[e] = f2{0.f, 0.f};
#pragma unroll
  for (int s = 0; s < DS; ++s) {
    RA[s] = ld<KPL, UP>(urs, voff, rl(C0.ua, s));
    RB[s] = ld<KPL, UP>(urs, voff, rl(C0.ub, s));
  }
  if constexpr (KPL >= 4) drain_vmem();  // prefill_wait (pair_device.hpp)
  const float neta = vgpr_of(-eta);
  ChunkRaw N{};  // the next chunk (sweep_chunks loads it when the current one starts)
  auto pair = [&](auto S) __attribute__((always_inline)) {
    constexpr int s = decltype(S)::value;
    const int slot = s % DS;
#if defined(MFHIP_EXPERIMENTS) && defined(MFHIP_WAITPROBE)
    {  // experiment build: shader cycles spent waiting for this pair's prefetched user rows
      const uint64_t a = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_waitcnt((4 * (DS - 1)) & 15 | (((4 * (DS - 1)) >> 4) << 14) | 0x0F70 & ~0xF);
      wait_clk += __builtin_amdgcn_s_memtime() - a;
    }
#endif
    // the ring's next offsets (pair s + DS), named up front
    const uint32_t noa = s + DS < CH ? rl(C0.ua, s + DS) : rl(N.w0[0], s + DS - CH);
    const uint32_t nob = s + DS < CH ? rl(C0.ub, s + DS) : rl(N.w0[1], s + DS - CH);
    Row<KPL> pa;
    uint32_t osa;
    if constexpr (FWD) {
      const uint32_t fl = rl(C0.flags, s);
      osa = rl(C0.sa, s);
      const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
#pragma unroll
      for (int e = 0; e < NV; ++e) pa.v[e] = vfma(kfb, plB.v[e], vfma(kfa, plA.v[e], RA[slot].v[e]));
    } else {
      osa = rl(C0.ua, s);
      pa = RA[slot];
    }
    const Row<KPL> pb = RB[slot];
    float c1 = dot_part<KPL>(pa, q), c2 = dot_part<KPL>(pb, q), g = dot_part<KPL>(pb, pa);
    wave_sum3(c1, c2, g);
    // wa = eta eA, wb = eta eB for every pair of the chunk at once (lane s holds pair s)
    const float wav = fmaf(c1, neta, C0.era);
    const float wbv = fmaf(fmaf(wav, g, C0.aa * c2), neta, C0.erb);
    const float wa = rlf(wav, s), wb = rlf(wbv, s);
    const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      const f2 q0 = q.v[e], a0 = pa.v[e], b0 = pb.v[e];
      const f2 q1 = vfma(wa, a0, aa * q0);
      plA.v[e] = vfma(wa, q0, ba * a0);
      plB.v[e] = vfma(wb, q1, bb * b0);
      q.v[e] = vfma(wb, b0, ab * q1);
    }
    st<KPL, UP>(urs, voff, osa, plA);
    st<KPL, UP>(urs, voff, rl(C0.ub, s), plB);
    RA[slot] = ld<KPL, UP>(urs, voff, noa);
    RB[slot] = ld<KPL, UP>(urs, voff, nob);
  };
  sweep_chunks<CH>(npairs, pair, [&](int c) { N = chunk_load<CH>(RR, c + 1, vlane); },
                           [&] { C0 = chunk_convert(N, eta); });
  keep_chunk(N);
  st<KPL, IP>(irs, voff, item_off, q);
}

// k = 64 (KPL = 1): one float of each row per lane.  Row<1> carries a row as a float pair with
// a zero high half, so every update of the generic code is a packed op on a half-empty register
// (and re-zeroing moves).  Here rows are plain floats, and the two updates that share a pattern
// run as one packed op: {plA, q1} = {ba, aa} * {pa, qa} + wa * {qa, pa} (v_pk_mul_f32, then
// v_pk_fma_f32 with the halves swapped), likewise {plB, q} from {pb, qb0}.  Same operation count
// per element as the generic step (one product, one fused multiply-add), but not the same rounding
// order: the generic step writes s*x + w*y and leaves the contraction to the compiler, this one
// rounds s*x first and fuses w*y into it.  Fast mode is judged on RMSE (tests/test_gpu_configs.py).
template <int POL = 0>
__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, off, POL));
}
template <int POL = 0>
__device__ __forceinline__ void st1(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, off, POL);
}
// {s0 * x + w * y, s1 * y + w * x}
__device__ __forceinline__ f2 pair_update(float s0, float s1, float w, float x, float y) {
  const f2 v = f2{x, y};
  return __builtin_elementwise_fma(f2{w, w}, v.yx, f2{s0, s1} * v);
}

template <int UP, bool FWD, int IP = kItemPolicy>
__device__ __forceinline__ void single_run_cell_k1(Chunk C0, __amdgpu_buffer_rsrc_t RR,
                                                   __amdgpu_buffer_rsrc_t urs, __amdgpu_buffer_rsrc_t irs, float eta,
                                                   uint32_t vlane, uint32_t voff, int npairs) {
  constexpr int CH = pair_chunk(1);
  constexpr int DS = pair_ring(1);
  const uint32_t item_off = rl(C0.ia, 0);
  float q = ld1<IP>(irs, voff, item_off);
  float RA[DS], RB[DS], plA = 0.f, plB = 0.f;
#pragma unroll
  for (int s = 0; s < DS; ++s) {
    RA[s] = ld1<UP>(urs, voff, rl(C0.ua, s));
    RB[s] = ld1<UP>(urs, voff, rl(C0.ub, s));
  }
  // no drain after the prefill (pair_device.hpp drain_vmem)
  const float neta = vgpr_of(-eta);
  ChunkRaw N{};  // the next chunk (sweep_chunks loads it when the current one starts)
  auto pair = [&](auto S) __attribute__((always_inline)) {
    constexpr int s = decltype(S)::value;
    const int slot = s % DS;
    const uint32_t noa = s + DS < CH ? rl(C0.ua, s + DS) : rl(N.w0[0], s + DS - CH);
    const uint32_t nob = s + DS < CH ? rl(C0.ub, s + DS) : rl(N.w0[1], s + DS - CH);
    float pa;
    uint32_t osa;
    if constexpr (FWD) {
      const uint32_t fl = rl(C0.flags, s);
      osa = rl(C0.sa, s);
      const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
      pa = kfb * plB + (kfa * plA + RA[slot]);
    } else {
      osa = rl(C0.ua, s);
      pa = RA[slot];
    }
    const float pb = RB[slot];
    float c1 = pa * q, c2 = pb * q, g = pb * pa;
    wave_sum3(c1, c2, g);
    const float wav = fmaf(c1, neta, C0.era);
    const float wbv = fmaf(fmaf(wav, g, C0.aa * c2), neta, C0.erb);
    const float wa = rlf(wav, s), wb = rlf(wbv, s);
    const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
    const f2 A = pair_update(ba, aa, wa, pa, q);    // {plA, q1}
    const f2 B = pair_update(bb, ab, wb, pb, A.y);  // {plB, q}
    plA = A.x;
    plB = B.x;
    q = B.y;
    st1<UP>(urs, voff, osa, plA);
    st1<UP>(urs, voff, rl(C0.ub, s), plB);
    RA[slot] = ld1<UP>(urs, voff, noa);
    RB[slot] = ld1<UP>(urs, voff, nob);
  };
  sweep_chunks<CH>(npairs, pair, [&](int c) { N = chunk_load<CH>(RR, c + 1, vlane); },
                           [&] { C0 = chunk_convert(N, eta); });
  keep_chunk(N);
  st1<IP>(irs, voff, item_off, q);
}

template <int D, int UP, int IP = kItemPolicy>
__device__ __forceinline__ void generic_cell_k1(Chunk C0, __amdgpu_buffer_rsrc_t RR,
                                                __amdgpu_buffer_rsrc_t urs, __amdgpu_buffer_rsrc_t irs, float eta,
                                                uint32_t vlane, uint32_t voff, int npairs) {
  constexpr int CH = pair_chunk(1);
  float plA = 0.f, plB = 0.f;
  float PA[D], PB[D], QA[D], QB[D];
#pragma unroll
  for (int s = 0; s < D; ++s) {
    PA[s] = ld1<UP>(urs, voff, rl(C0.ua, s));
    PB[s] = ld1<UP>(urs, voff, rl(C0.ub, s));
    QA[s] = ld1<IP>(irs, voff, rl(C0.ia, s));
    QB[s] = ld1<IP>(irs, voff, rl(C0.ib, s));
  }
  // no drain after the prefill (pair_device.hpp drain_vmem)
  const float neta = vgpr_of(-eta);
  float q = 0.f;
  ChunkRaw N{};  // the next chunk (sweep_chunks loads it when the current one starts)
  auto pair = [&](auto S) __attribute__((always_inline)) {
    constexpr int s = decltype(S)::value;
    const int slot = s % D;
    const uint32_t fl = rl(C0.flags, s);
    const uint32_t osa = rl(C0.sa, s), osb = rl(C0.sb, s), osia = rl(C0.sia, s), osi = rl(C0.si, s);
    const bool nin = s + D < CH;
    const uint32_t nua = nin ? rl(C0.ua, s + D) : rl(N.w0[0], s + D - CH);
    const uint32_t nub = nin ? rl(C0.ub, s + D) : rl(N.w0[1], s + D - CH);
    const uint32_t nia = nin ? rl(C0.ia, s + D) : rl(N.w0[2], s + D - CH);
    const uint32_t nib = nin ? rl(C0.ib, s + D) : rl(N.w0[3], s + D - CH);
    const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
    const float kq = static_cast<float>((fl >> 16) & 0xFFu);
    const float sr = rlf(C0.sr, s);
    const float pa = kfb * plB + (kfa * plA + PA[slot]);  // loads of forwarded rows return 0
    const float pb = PB[slot];
    const float qa = kq * q + QA[slot];
    const float qbd = sr * qa + QB[slot];  // B's item before A's update: q (run) or qB (split)
    float c1 = pa * qa, c2 = pb * qbd, g = pb * pa;
    wave_sum3(c1, c2, g);
    const float wav = fmaf(c1, neta, C0.era);
    const float wbv = fmaf(fmaf(C0.sr * wav, g, C0.m * c2), neta, C0.erb);
    const float wa = rlf(wav, s), wb = rlf(wbv, s);
    const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
    const f2 A = pair_update(ba, aa, wa, pa, qa);  // {plA, q1}
    const float qb0 = sr * A.y + QB[slot];
    const f2 B = pair_update(bb, ab, wb, pb, qb0);  // {plB, q}
    plA = A.x;
    plB = B.x;
    q = B.y;
    st1<UP>(urs, voff, osa, plA);
    st1<UP>(urs, voff, osb, plB);
    st1<IP>(irs, voff, osia, A.y);
    st1<IP>(irs, voff, osi, q);
    PA[slot] = ld1<UP>(urs, voff, nua);
    PB[slot] = ld1<UP>(urs, voff, nub);
    QA[slot] = ld1<IP>(irs, voff, nia);
    QB[slot] = ld1<IP>(irs, voff, nib);
  };
  sweep_chunks<CH>(npairs, pair, [&](int c) { N = chunk_load<CH>(RR, c + 1, vlane); },
                           [&] { C0 = chunk_convert(N, eta); });
  keep_chunk(N);
}

// One cell (WaveDesc d) of the pair schedule, swept by the calling wave.  UP = cache policy of
// the user-row loads and stores.  L0: the cell's first record chunk, loaded by the caller (the
// systolic sweep loads it while the previous cell's stores drain); sweep_chunks (pair_device.hpp)
// loads chunk c + 1 when chunk c starts.
template <int KPL, int D, int UP, int IP = kItemPolicy>
__device__ __forceinline__ void pair_cell(const WaveDesc d, const ChunkRaw& L0,
                                          const u4v* __restrict__ recs, __amdgpu_buffer_rsrc_t urs,
                                          __amdgpu_buffer_rsrc_t irs, float eta, int lane, uint64_t& wait_clk) {
  (void)wait_clk;
  constexpr int NV = Row<KPL>::NV;
  constexpr int CH = pair_chunk(KPL);
  static_assert(CH % D == 0, "ring slots must repeat every chunk");
  const int npairs = d.steps;
  const __amdgpu_buffer_rsrc_t RR = cell_records(recs, d.base, npairs);
  const uint32_t vlane = static_cast<uint32_t>(lane) * 64u;
  const uint32_t voff = static_cast<uint32_t>(lane) * KPL * 4u;

  Chunk C0 = chunk_convert(L0, eta);  // current chunk
  if constexpr (KPL == 1) {
    if (d.cells == kWaveSingleRun)
      single_run_cell_k1<UP, false>(C0, RR, urs, irs, eta, vlane, voff, npairs);
    else if (d.cells == kWaveSingleRunFwd)
      single_run_cell_k1<UP, true>(C0, RR, urs, irs, eta, vlane, voff, npairs);
    else
      generic_cell_k1<D, UP>(C0, RR, urs, irs, eta, vlane, voff, npairs);
    return;
  }
  if (d.cells == kWaveSingleRun) {
    single_run_cell<KPL, UP, false>(C0, RR, urs, irs, eta, vlane, voff, npairs, wait_clk);
    return;
  }
  if (d.cells == kWaveSingleRunFwd) {
    single_run_cell<KPL, UP, true>(C0, RR, urs, irs, eta, vlane, voff, npairs, wait_clk);
    return;
  }
  Row<KPL> plA, plB;  // the previous pair's updated user rows (forwarding)
#pragma unroll
  for (int e = 0; e < NV; ++e) plA.v[e] = plB.v[e] = f2{0.f, 0.f};

  {
    Row<KPL> PA[D], PB[D], QA[D], QB[D];
#define MF_PREFETCH(slot, UA, UB, IA, IB, YY)                                   \
    do {                                                                        \
      PA[slot] = ld<KPL, UP>(urs, voff, rl(UA, (YY)));                              \
      PB[slot] = ld<KPL, UP>(urs, voff, rl(UB, (YY)));                              \
      QA[slot] = ld<KPL, IP>(irs, voff, rl(IA, (YY)));                              \
      QB[slot] = ld<KPL, IP>(irs, voff, rl(IB, (YY)));                              \
    } while (0)
#pragma unroll
    for (int s = 0; s < D; ++s) MF_PREFETCH(s, C0.ua, C0.ub, C0.ia, C0.ib, s);
    if constexpr (KPL >= 4) drain_vmem();  // prefill_wait (pair_device.hpp)
    const float neta = vgpr_of(-eta);
    Row<KPL> q;
#pragma unroll
    for (int e = 0; e < NV; ++e) q.v[e] = f2{0.f, 0.f};

    ChunkRaw N{};  // the next chunk (sweep_chunks loads it when the current one starts)
  auto pair = [&](auto S) __attribute__((always_inline)) {
    constexpr int s = decltype(S)::value;
      const int slot = s % D;
#if defined(MFHIP_EXPERIMENTS) && defined(MFHIP_WAITPROBE)
      {  // experiment build: shader cycles spent waiting for this pair's prefetched rows
        const uint64_t a = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt((8 * (D - 1)) & 15 | (((8 * (D - 1)) >> 4) << 14) | 0x0F70 & ~0xF);
        wait_clk += __builtin_amdgcn_s_memtime() - a;
      }
#endif
      const uint32_t fl = rl(C0.flags, s);
      // store offsets named up front: the scheduler then reads them early instead of right
      // before each store (a v_readlane feeding a buffer store's soffset costs an s_nop 4)
      const uint32_t osa = rl(C0.sa, s), osb = rl(C0.sb, s), osia = rl(C0.sia, s), osi = rl(C0.si, s);
      const bool nin = s + D < CH;  // offsets of pair s + D (the ring's next rows)
      const uint32_t nua = nin ? rl(C0.ua, s + D) : rl(N.w0[0], s + D - CH);
      const uint32_t nub = nin ? rl(C0.ub, s + D) : rl(N.w0[1], s + D - CH);
      const uint32_t nia = nin ? rl(C0.ia, s + D) : rl(N.w0[2], s + D - CH);
      const uint32_t nib = nin ? rl(C0.ib, s + D) : rl(N.w0[3], s + D - CH);
      // byte flags -> float coefficients (v_cvt_f32_ubyteN): forwarding, keep q, split
      const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
      const float kq = static_cast<float>((fl >> 16) & 0xFFu);
      const float sr = rlf(C0.sr, s);  // 1 - split, from the chunk (one readlane, no convert + subtract)
      Row<KPL> pa, pb, qa, qbd;
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        pa.v[e] = vfma(kfb, plB.v[e], vfma(kfa, plA.v[e], PA[slot].v[e]));  // loads of forwarded rows return 0
        pb.v[e] = PB[slot].v[e];
        qa.v[e] = vfma(kq, q.v[e], QA[slot].v[e]);
        qbd.v[e] = vfma(sr, qa.v[e], QB[slot].v[e]);  // B's item before A's update: q (run) or qB (split)
      }
      float c1 = dot_part<KPL>(pa, qa), c2 = dot_part<KPL>(pb, qbd), g = dot_part<KPL>(pb, pa);
      wave_sum3(c1, c2, g);
#ifdef MFHIP_EXP_PAD_VALU  // sensitivity experiment: N extra VALU issue slots per mixed pair
#define MF_STR2(x) #x
#define MF_STR(x) MF_STR2(x)
      asm volatile(".rept " MF_STR(MFHIP_EXP_PAD_VALU) "\n\tv_nop\n\t.endr");
#endif
      // wa = eta eA, wb = eta eB in the chunk layout (lane s = pair s); a split pair has no
      // coupling to A's update (sr = 0, m = 1)
      const float wav = fmaf(c1, neta, C0.era);
      const float wbv = fmaf(fmaf(C0.sr * wav, g, C0.m * c2), neta, C0.erb);
      const float wa = rlf(wav, s), wb = rlf(wbv, s);
      const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
      Row<KPL> q1;
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        const f2 q0 = qa.v[e], a0 = pa.v[e], b0 = pb.v[e];
        q1.v[e] = vfma(wa, a0, aa * q0);
        plA.v[e] = vfma(wa, q0, ba * a0);
        const f2 qb0 = vfma(sr, q1.v[e], QB[slot].v[e]);
        plB.v[e] = vfma(wb, qb0, bb * b0);
        q.v[e] = vfma(wb, b0, ab * qb0);
      }
      st<KPL, UP>(urs, voff, osa, plA);
      st<KPL, UP>(urs, voff, osb, plB);
      st<KPL, IP>(irs, voff, osia, q1);
      st<KPL, IP>(irs, voff, osi, q);
      // rows of pair j+D (after this pair's stores)
      PA[slot] = ld<KPL, UP>(urs, voff, nua);
      PB[slot] = ld<KPL, UP>(urs, voff, nub);
      QA[slot] = ld<KPL, IP>(irs, voff, nia);
      QB[slot] = ld<KPL, IP>(irs, voff, nib);
  };
  sweep_chunks<CH>(npairs, pair, [&](int c) { N = chunk_load<CH>(RR, c + 1, vlane); },
                           [&] { C0 = chunk_convert(N, eta); });
    keep_chunk(N);
#undef MF_PREFETCH
  }
}

// One launch per sub-step: wave = cell (waves[] of the sub-step, longest first).
template <int KPL, int D>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_sweep_pair(
    const WaveDesc* __restrict__ waves, const u4v* __restrict__ recs, float* __restrict__ U, float* __restrict__ I,
    uint64_t u_bytes, uint64_t i_bytes, float eta, uint64_t* __restrict__ trace) {
  MF_LAUNCH_ACQUIRE();
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  const WaveDesc d = waves[blockIdx.x];
  const __amdgpu_buffer_rsrc_t rr = cell_records(recs, d.base, d.steps);
  const uint32_t vlane = threadIdx.x * 64u;
  uint64_t wait_clk = 0;
  pair_cell<KPL, D, 0>(d, chunk_load<pair_chunk(KPL)>(rr, 0, vlane), recs, raw_rsrc(U, u_bytes),
                       raw_rsrc(I, i_bytes), eta, threadIdx.x, wait_clk);
  MF_LAUNCH_RELEASE();
  if (trace && threadIdx.x == 0) {
    trace[2 * blockIdx.x] = t_start;
    trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// One persistent launch per superstep (systolic rotation).  Wave (j, g) sweeps the G_j cells of
// item group g of local rating block j in sub-step order; before cell t it waits until wave
// (j, g+1) has finished cell t-1, the only earlier user of user group (g+t) mod G_j in this
// superstep (item group g is this wave's alone).  Rating blocks are independent grids, each
// with its own G_j (choose_block_groups).  So a sub-step is no longer a grid-wide
// barrier: each cell starts when its two predecessors are done, and a long cell delays only
// the waves downstream of it.  Hand-off (MI355X_MICROARCH.md, valid forms, row 1): every
// user-row store and load is sc1, the wave drains its stores (vmcnt(0)), then lane 0 stores
// the progress word (agent-scope relaxed atomic = sc1 store); the consumer polls it with
// agent-scope relaxed loads (sc1).  Progress words are monotonic across launches (base), so
// they are never reset.  Every wave must be resident at once (the host checks occupancy); a
// poll that exceeds ~1 s sets err[0] and the wave gives up (the host then fails loudly).
// PRE: the next cell's first record chunk is loaded right after a cell's last stores are
// issued, so it arrives while those stores drain (vmcnt(4) waits for the stores only): a cell no
// longer starts with a record fetch on its critical path (an empty cell reads nothing; past the
// last cell the last cell's records are read again, unused).  The neighbour's progress is polled
// after the drain (read before the drain it was too often not yet there: an extra poll round trip,
// ML20M 5.98 vs 5.60 ms per epoch in round 3); EARLY also reads it once with the drain, and a
// neighbour already done then needs no poll (kEarlyPoll below).
template <int KPL, int D, bool PRE, bool EARLY>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_sweep_pair_sys(
    const SysWave* __restrict__ sw, const WaveDesc* __restrict__ sys, int nw, int lbase, const u4v* __restrict__ recs,
    float* __restrict__ U, float* __restrict__ I, uint64_t u_bytes, uint64_t i_bytes, float eta,
    int32_t* __restrict__ prog, uint32_t base, int32_t* __restrict__ err, uint64_t* __restrict__ trace,
    const int32_t* __restrict__ place) {
  MF_LAUNCH_ACQUIRE();
  const int lane = threadIdx.x;
  // blocks b and b+8 share an XCD: give each XCD a contiguous range of waves, so most hand-offs
  // (g+1 -> g) stay inside one L2 (speed only; correctness does not depend on it).  XCD x holds
  // nw/8 blocks, plus one when x < nw%8: a bijection for any nw.  sw = this launch's waves, the
  // superstep's waves from lbase on (progress words and SysWave::nbr count from the superstep's
  // first wave).
  // place (host-made, sys_placement): the same XCD ranges, permuted inside an XCD so that the
  // heaviest waves get the CUs with the fewest other waves (blocks k, k+32, k+64 of an XCD share a CU);
  // with empty blocks (-1) the heaviest wave of each XCD has its CU to itself (nw counts them too)
  const int b = static_cast<int>(blockIdx.x);
  const int x = b % 8, per = nw / 8, extra = nw % 8;
  const int L = place ? place[b] : x * per + min(x, extra) + b / 8;
  if (L < 0) return;  // an empty block of the placement (it only keeps a heavy wave's CU to itself)
  const SysWave w = sw[L];
  const WaveDesc* my = sys + w.cell0;
  int32_t* my_prog = prog + static_cast<int64_t>(lbase + L) * kProgStride;
  int32_t* nb_prog = prog + static_cast<int64_t>(w.nbr) * kProgStride;
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);
  const uint32_t vlane = static_cast<uint32_t>(lane) * 64u;
  auto first_chunks = [&](const WaveDesc& c, ChunkRaw& A) {  // an empty cell reads nothing
    A = chunk_load<pair_chunk(KPL)>(cell_records(recs, c.base, c.steps), 0, vlane);
  };
  WaveDesc d = my[0];
  ChunkRaw L0;
  if (PRE) first_chunks(d, L0);
  uint32_t seen = base;  // the neighbour's progress as last read
  for (int t = 0; t < w.G; ++t) {
    const WaveDesc dn = my[t + 1 < w.G ? t + 1 : t];  // scalar load, used after this cell
    if (t > 0 && w.G > 1 && static_cast<int32_t>(seen - (base + static_cast<uint32_t>(t))) < 0) {
      const uint32_t want = base + static_cast<uint32_t>(t);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
            __hip_atomic_load(nb_prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        if (static_cast<int32_t>(v - want) >= 0) break;
        // another wave gave up: its downstream waves would each spin their own second, so leave now
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
          return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 100 MHz clock: ~1 s
          if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const uint64_t c_start = __builtin_amdgcn_s_memrealtime();
    uint64_t c_clk = trace ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t wait_clk = 0;
    if (!PRE && d.steps > 0) first_chunks(d, L0);
    if (d.steps > 0) pair_cell<KPL, D, kSC1>(d, L0, recs, urs, irs, eta, lane, wait_clk);
    // EARLY: the neighbour's progress read together with this cell's store drain (issued after
    // the stores, completes with them), so a neighbour already done costs no poll round trip
    uint32_t early = 0;
    if (EARLY && t + 1 < w.G) early = __hip_atomic_load(nb_prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (PRE) {
      first_chunks(dn, L0);
      __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): the 4 loads above may fly, every older store has landed
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every user-row store of this wave has landed
    }
    if (EARLY && t + 1 < w.G) seen = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(early)));
    if (lane == 0)
      __hip_atomic_store(my_prog, static_cast<int32_t>(base + static_cast<uint32_t>(t) + 1u), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (trace && lane == 0) {  // {start, end} on the 100 MHz clock, shader-clock cycles, placement
      uint64_t* tr = trace + 4 * (w.cell0 + t);
      tr[0] = c_start;
      tr[1] = __builtin_amdgcn_s_memrealtime();
#if defined(MFHIP_EXPERIMENTS) && defined(MFHIP_WAITPROBE)
      tr[2] = wait_clk;  // experiment build: the trace's clock column carries the wait cycles
#else
      tr[2] = __builtin_amdgcn_s_memtime() - c_clk;
#endif
      // where the wave runs: XCC_ID (hwreg 20) and HW_ID (hwreg 4: wave, SIMD, CU, SH, SE)
      tr[3] = (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20)) << 32) |
              static_cast<uint32_t>(__builtin_amdgcn_s_getreg((31 << 11) | 4));
    }
    d = dn;
  }
  MF_LAUNCH_RELEASE();
}

// ev0 / ev1 (may be null): timed by the dispatch packet itself (no extra stream commands).
template <int KPL>
void dispatch(hipStream_t st, const WaveDesc* waves, int nwaves, const PairRec* recs, float* U, float* I,
              uint64_t ub, uint64_t ib, float eta, uint64_t* trace, hipEvent_t ev0, hipEvent_t ev1) {
  hipExtLaunchKernelGGL((k_sweep_pair<KPL, pair_ring(KPL)>), dim3(static_cast<unsigned>(nwaves)), dim3(64), 0, st, ev0, ev1,
                        0, waves, reinterpret_cast<const u4v*>(recs), U, I, ub, ib, eta, trace);
}

// Record preload across the cell boundary (PRE): on for every k since round 6 (ML20M 4.41-4.42 ->
// 4.26-4.27 ms per epoch, profiles/r06_ML20M_cell_ab.txt; off at k = 64 until then: 5.86-5.98 vs
// 5.59-5.60 ms in round 3, before the per-width rings).  EARLY (the neighbour's progress read with
// the drain): NFLX 20.00 / 19.98 -> 19.91 / 19.82 ms, ML20M 4.22 -> 4.25 / 4.26 ms -- k = 128 only.
template <int KPL>
constexpr bool kCellPreload = true;
template <int KPL>
constexpr bool kEarlyPoll = KPL == 2;

template <int KPL>
void dispatch_sys(hipStream_t st, const SysWave* sw, const WaveDesc* sys, int nw, int lbase, const PairRec* recs,
                  float* U, float* I, uint64_t ub, uint64_t ib, float eta, int32_t* prog, uint32_t base, int32_t* err,
                  uint64_t* trace, hipEvent_t ev0, hipEvent_t ev1, const int32_t* place) {
  hipExtLaunchKernelGGL((k_sweep_pair_sys<KPL, pair_ring(KPL), kCellPreload<KPL>, kEarlyPoll<KPL>>), dim3(static_cast<unsigned>(nw)),
                        dim3(64), 0, st, ev0, ev1, 0, sw, sys, nw, lbase, reinterpret_cast<const u4v*>(recs), U, I, ub,
                        ib, eta, prog, base, err, trace, place);
}

template <int KPL>
int sys_capacity() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sweep_pair_sys<KPL, pair_ring(KPL), kCellPreload<KPL>, kEarlyPoll<KPL>>, 64,
                                                   0) != hipSuccess)
    return 0;
  return cus * per_cu;
}

}  // namespace

bool pair_kernel_supports(int k) { return k == 64 || k == 128 || k == 256; }

int sweep_pair_sys_capacity(int k) {
  switch (k) {
    case 64: return sys_capacity<1>();
    case 128: return sys_capacity<2>();
    case 256: return sys_capacity<4>();
    default: return 0;
  }
}

void launch_sweep_pair_sys(hipStream_t st, const SysWave* sw, const WaveDesc* sys, int nw, int lbase,
                           const PairRec* recs, float* U, float* I, uint64_t u_bytes, uint64_t i_bytes, int k, float eta,
                           int32_t* prog, uint32_t base, int32_t* err, uint64_t* trace, hipEvent_t ev0, hipEvent_t ev1,
                           const int32_t* place) {
  if (nw <= 0) return;
#define MF_SYS(KPL) dispatch_sys<KPL>(st, sw, sys, nw, lbase, recs, U, I, u_bytes, i_bytes, eta, prog, base, err, trace, ev0, ev1, place)
  switch (k) {
    case 64: MF_SYS(1); break;
    case 128: MF_SYS(2); break;
    case 256: MF_SYS(4); break;
    default: break;
  }
#undef MF_SYS
}

void launch_sweep_pair(hipStream_t st, const WaveDesc* waves, int nwaves, const PairRec* recs, float* U, float* I,
                       uint64_t u_bytes, uint64_t i_bytes, int k, float eta, uint64_t* trace, hipEvent_t ev0,
                       hipEvent_t ev1) {
  if (nwaves <= 0) return;
  switch (k) {
    case 64: dispatch<1>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace, ev0, ev1); break;
    case 128: dispatch<2>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace, ev0, ev1); break;
    case 256: dispatch<4>(st, waves, nwaves, recs, U, I, u_bytes, i_bytes, eta, trace, ev0, ev1); break;
    default: break;
  }
}

#ifdef MFHIP_EXPERIMENTS
// Hot-item replicas (plan.hpp SplitItem), one workgroup per split item, any k.  fork: the item's
// row to its R-1 replica rows; join: q = (q + sum_r q_r) / R, replicas in order (deterministic).
__global__ __launch_bounds__(64) void k_split_fork(const SplitItem* __restrict__ sp, float* __restrict__ I, int k) {
  const SplitItem h = sp[blockIdx.x];
  const float* q = I + static_cast<size_t>(h.main_row) * k;
  float* dst = I + static_cast<size_t>(h.scratch_row) * k;
  for (int e = threadIdx.x; e < k; e += 64) {
    const float v = q[e];
    for (int r = 0; r < h.R - 1; ++r) dst[static_cast<size_t>(r) * k + e] = v;
  }
}

__global__ __launch_bounds__(64) void k_split_join(const SplitItem* __restrict__ sp, float* __restrict__ I, int k) {
  const SplitItem h = sp[blockIdx.x];
  float* q = I + static_cast<size_t>(h.main_row) * k;
  const float* rep = I + static_cast<size_t>(h.scratch_row) * k;
  const float inv = 1.0f / static_cast<float>(h.R);
  for (int e = threadIdx.x; e < k; e += 64) {
    float acc = q[e];
    for (int r = 0; r < h.R - 1; ++r) acc += rep[static_cast<size_t>(r) * k + e];
    q[e] = acc * inv;
  }
}

#endif

// Hot-item replicas exist only in a -DMFHIP_EXPERIMENTS build (the default build never plans any).
void launch_split_fork(hipStream_t st, const SplitItem* sp, int n, float* I, int k) {
#ifdef MFHIP_EXPERIMENTS
  if (n > 0) hipLaunchKernelGGL(k_split_fork, dim3(n), dim3(64), 0, st, sp, I, k);
#else
  (void)st; (void)sp; (void)n; (void)I; (void)k;
#endif
}

void launch_split_join(hipStream_t st, const SplitItem* sp, int n, float* I, int k) {
#ifdef MFHIP_EXPERIMENTS
  if (n > 0) hipLaunchKernelGGL(k_split_join, dim3(n), dim3(64), 0, st, sp, I, k);
#else
  (void)st; (void)sp; (void)n; (void)I; (void)k;
#endif
}

}  // namespace mfhip
