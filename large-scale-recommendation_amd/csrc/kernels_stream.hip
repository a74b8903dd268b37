// kernels_stream.hip -- fast-mode DSGD stream sweep (f32): one launch per superstep, one wave per
// item group, its cells as one continuous pair sequence with per-pair hand-offs (plan.hpp StreamWave).
// The pair step itself (two updates per reduction round, forwarding, out-of-range offsets for
// unused rows) is kernels_pair.hip's; see there.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

#include "pair_device.hpp"

// ---------------------------------------------------------------------------------------
// Stream sweep (plan.hpp StreamWave): one launch per superstep, one wave per item group of each
// local rating block, its K*G cells as ONE pair sequence.  The record chunks and the D-deep row
// ring run straight through cell boundaries; there is no per-cell drain, reload or wait.
//
// Hand-off, per pair instead of per cell:
//  * publish: after pair j's arithmetic the wave has waited for pair j's rows, which were loaded
//    after pair j-D's stores, and vmcnt retires in issue order, so the stores of pairs 0..j-D
//    have completed.  Lane 0 stores base + (j-D+1) to the wave's progress word (sc1) every pair.
//  * consume: pair j carries `need` (its cell's hand-off: the neighbour's pairs through its cell
//    t-K).  Before the rows of pair j+D are loaded the wave compares base + need(j+D) with the
//    largest neighbour progress seen so far; that value is refreshed every pair by a load that
//    rides in the ring beside the rows (so it costs no wait).  Only when it is short does the
//    wave poll synchronously (sc1 loads, ~1 s bound -> err[0]).
// Row traffic, forwarding and arithmetic are exactly pair_cell's (build_stream_plan keeps the
// window of 2D records along the whole stream, and never lets a pair span two cells).

// Progress words are read and written as agent-scope relaxed atomics (global_load / global_store
// sc1, k_sweep_pair_sys's proven hand-off form; an atomic is never hoisted out of a poll loop).
// A wave's slot is kStreamProgStride words: lane l stores the same value to word l and loads word l
// of the neighbour's slot, so each access is one coalesced 256-B line pair (64 lanes on ONE word
// serialise), with no lane-divergent branch in the ring; word 0 is the progress.
__device__ __forceinline__ uint32_t prog_load(const int32_t* w) {
  return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ int32_t prog_load_lanes(const int32_t* w) {  // VGPR result: read it later
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void prog_store(int32_t* w, uint32_t v) {
  __hip_atomic_store(w, static_cast<int32_t>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int CH>
__device__ __forceinline__ ChunkRaw chunk_load_n(const u4v* __restrict__ R, int c, int npairs, int lane) {
  const int64_t x = min(c * CH + min(lane, CH - 1), npairs - 1);
  return ChunkRaw{__builtin_nontemporal_load(R + 4 * x), __builtin_nontemporal_load(R + 4 * x + 1),
                  __builtin_nontemporal_load(R + 4 * x + 2), __builtin_nontemporal_load(R + 4 * x + 3)};
}

// Returns once the neighbour's progress has reached `want` (wrap-safe): at once when an earlier
// observation covers it, else by polling.  No early exit and no lane-divergent code: the fast path
// must stay one uniform branch so that the compiler's vmcnt tracking of the row ring survives it.
// Before it polls, the wave drains its stores and publishes `done` (every pair it has computed):
// a blocked wave then holds back only the pairs it has prefetched and not computed, which
// build_stream_plan keeps below the K-1 cells of slack (no cycle of waits around the ring).
// A poll that exceeds ~1 s sets err[0] (and the slot's diagnostics) and gives up; the wave then runs on
// with rows that may be stale -- the host turns err into MF_ERR_TIMEOUT and voids the fit.
struct WaitStats {
  uint32_t waits = 0;  // slow-path entries
  uint64_t ticks = 0;  // 100 MHz ticks spent in them
};

__device__ __forceinline__ void stream_wait(const int32_t* nb_prog, uint32_t want, uint32_t& seen, int32_t* my_prog,
                                            uint32_t done, uint32_t& pub, int32_t* err, int32_t slot, WaitStats& ws) {
  if (__builtin_expect(static_cast<int32_t>(seen - want) >= 0, 1)) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the stores of every computed pair have landed
  pub = done;
  prog_store(my_prog, done);
  ++ws.waits;
  for (;;) {
    const uint32_t v = prog_load(nb_prog);
    if (static_cast<int32_t>(v - seen) > 0) seen = v;
    if (static_cast<int32_t>(seen - want) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 100 MHz clock: ~1 s
      prog_store(err, 1u);
      int32_t* d = err + 4 + 8 * slot;  // diagnostics (err holds 4 + 8 * waves words): {seen, want, published, 1}
      prog_store(d, seen);
      prog_store(d + 1, want);
      prog_store(d + 2, done);
      prog_store(d + 3, 1u);
      seen = want;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  ws.ticks += __builtin_amdgcn_s_memrealtime() - t0;
}

template <int KPL, int D, int CH, int P>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_sweep_stream(
    const StreamWave* __restrict__ sws, int nw, int lbase, const u4v* __restrict__ recs, float* __restrict__ U,
    float* __restrict__ I, uint64_t u_bytes, uint64_t i_bytes, float eta, int32_t* __restrict__ prog, uint64_t prog_bytes,
    uint32_t base, int32_t* __restrict__ err) {
  constexpr int NV = Row<KPL>::NV;
  static_assert(CH % D == 0 && CH % P == 0, "ring slots and hand-off periods must repeat every chunk");
  const int lane = threadIdx.x;
  const int b = static_cast<int>(blockIdx.x);
  const int x = b % 8, per = nw / 8, extra = nw % 8;
  const int L = x * per + min(x, extra) + b / 8;  // XCD-contiguous waves (k_sweep_pair_sys)
  const StreamWave w = sws[L];
  const bool single = (w.nbr & kStreamSingleRun) != 0;
  const int nbr = w.nbr & ~kStreamSingleRun;
  const int npairs = w.npairs;
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);
  int32_t* my_prog = prog + static_cast<int64_t>(lbase + L) * kStreamProgStride + lane;
  const int32_t* nb_prog = prog + static_cast<int64_t>(nbr) * kStreamProgStride + lane;
  const uint32_t voff = static_cast<uint32_t>(lane) * KPL * 4u;
  uint32_t seen = base;  // largest neighbour progress observed (stale words from earlier launches are < base)
  uint32_t pub = base;   // largest value published (the progress word never moves back)
  WaitStats wst;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  prog_store(my_prog, base);  // 0 pairs done in this launch
  if (npairs <= 0) return;
  const u4v* R = recs + 4 * w.base;
  Chunk C0 = chunk_convert(chunk_load_n<CH>(R, 0, npairs, lane), eta);
  ChunkRaw C1 = chunk_load_n<CH>(R, 1, npairs, lane);
  // the prologue's D pairs: need is monotone along the stream, so the last of them has the largest
  stream_wait(nb_prog, base + rl(C0.need, min(D, npairs) - 1), seen, my_prog, base, pub, err, lbase + L, wst);
  Row<KPL> plA, plB;
#pragma unroll
  for (int e = 0; e < NV; ++e) plA.v[e] = plB.v[e] = f2{0.f, 0.f};
  int32_t PV[D];  // the neighbour's progress, loaded with each pair's rows

  if (single) {
    const uint32_t item_off = rl(C0.ia, 0);
    Row<KPL> q = ld<KPL>(irs, voff, item_off);
    Row<KPL> RA[D], RB[D];
    uint32_t ob[D];
#pragma unroll
    for (int s = 0; s < D; ++s) {
      ob[s] = rl(C0.ub, s);
      RA[s] = ld<KPL, kSC1>(urs, voff, rl(C0.ua, s));
      RB[s] = ld<KPL, kSC1>(urs, voff, ob[s]);
      PV[s] = prog_load_lanes(nb_prog);
    }
    drain_vmem();
    for (int c = 0;; ++c) {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int j = c * CH + s;
        if (j >= npairs) goto run_done;
        const int slot = s % D;
        const uint32_t fl = rl(C0.flags, s), osa = rl(C0.sa, s);
        const uint32_t noa = s + D < CH ? rl(C0.ua, s + D) : rl(C1.w0[0], s + D - CH);
        const uint32_t nob = s + D < CH ? rl(C0.ub, s + D) : rl(C1.w0[1], s + D - CH);
        const uint32_t nneed = s + D < CH ? rl(C0.need, s + D) : rl(C1.w3[3], s + D - CH);
        const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
        Row<KPL> pa;
        const Row<KPL> pb = RB[slot];
#pragma unroll
        for (int e = 0; e < NV; ++e) pa.v[e] = kfb * plB.v[e] + (kfa * plA.v[e] + RA[slot].v[e]);
        float c1 = dot_part<KPL>(pa, q), c2 = dot_part<KPL>(pb, q), g = dot_part<KPL>(pb, pa);
        wave_sum3(c1, c2, g);
        const float era = rlf(C0.era, s), erb = rlf(C0.erb, s);
        const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
        const float wa = fmaf(-eta, c1, era);
        const float wb = fmaf(-eta, fmaf(wa, g, aa * c2), erb);
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          const f2 q0 = q.v[e], a0 = pa.v[e], b0 = pb.v[e];
          const f2 q1 = aa * q0 + wa * a0;
          plA.v[e] = ba * a0 + wa * q0;
          plB.v[e] = bb * b0 + wb * q1;
          q.v[e] = ab * q1 + wb * b0;
        }
        st<KPL, kSC1>(urs, voff, osa, plA);
        st<KPL, kSC1>(urs, voff, ob[slot], plB);
        {  // hand-off: publish, refresh the neighbour's progress, gate the next loads
          const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(PV[slot]));
          if (static_cast<int32_t>(v - seen) > 0) seen = v;
          const uint32_t lag = base + static_cast<uint32_t>(max(j - D + 1, 0));  // stores of pairs <= j-D landed
          if (static_cast<int32_t>(lag - pub) > 0) pub = lag;
          if constexpr (P == 1) prog_store(my_prog, pub);
          else if (s % P == 0) prog_store(my_prog, pub);
          stream_wait(nb_prog, base + nneed, seen, my_prog, base + static_cast<uint32_t>(j + 1), pub, err, lbase + L, wst);
        }
        ob[slot] = nob;
        RA[slot] = ld<KPL, kSC1>(urs, voff, noa);
        RB[slot] = ld<KPL, kSC1>(urs, voff, ob[slot]);
        if (s % P == 0) PV[slot] = prog_load_lanes(nb_prog);
      }
      C0 = chunk_convert(C1, eta);
      C1 = chunk_load_n<CH>(R, c + 2, npairs, lane);
    }
  run_done:
    st<KPL>(irs, voff, item_off, q);
  } else {
    Row<KPL> PA[D], PB[D], QA[D], QB[D];
#pragma unroll
    for (int s = 0; s < D; ++s) {
      PA[s] = ld<KPL, kSC1>(urs, voff, rl(C0.ua, s));
      PB[s] = ld<KPL, kSC1>(urs, voff, rl(C0.ub, s));
      QA[s] = ld<KPL>(irs, voff, rl(C0.ia, s));
      QB[s] = ld<KPL>(irs, voff, rl(C0.ib, s));
      PV[s] = prog_load_lanes(nb_prog);
    }
    drain_vmem();
    Row<KPL> q;
#pragma unroll
    for (int e = 0; e < NV; ++e) q.v[e] = f2{0.f, 0.f};
    for (int c = 0;; ++c) {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const int j = c * CH + s;
        if (j >= npairs) goto gen_done;
        const int slot = s % D;
        const uint32_t fl = rl(C0.flags, s);
        const uint32_t osa = rl(C0.sa, s), osb = rl(C0.sb, s), osia = rl(C0.sia, s), osi = rl(C0.si, s);
        const bool nin = s + D < CH;
        const uint32_t nua = nin ? rl(C0.ua, s + D) : rl(C1.w0[0], s + D - CH);
        const uint32_t nub = nin ? rl(C0.ub, s + D) : rl(C1.w0[1], s + D - CH);
        const uint32_t nia = nin ? rl(C0.ia, s + D) : rl(C1.w0[2], s + D - CH);
        const uint32_t nib = nin ? rl(C0.ib, s + D) : rl(C1.w0[3], s + D - CH);
        const uint32_t nneed = nin ? rl(C0.need, s + D) : rl(C1.w3[3], s + D - CH);
        const float kfa = static_cast<float>(fl & 0xFFu), kfb = static_cast<float>((fl >> 8) & 0xFFu);
        const float kq = static_cast<float>((fl >> 16) & 0xFFu), sp = static_cast<float>(fl >> 24);
        const float sr = 1.f - sp;
        Row<KPL> pa, pb, qa, qbd;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          pa.v[e] = kfb * plB.v[e] + (kfa * plA.v[e] + PA[slot].v[e]);
          pb.v[e] = PB[slot].v[e];
          qa.v[e] = kq * q.v[e] + QA[slot].v[e];
          qbd.v[e] = sr * qa.v[e] + QB[slot].v[e];
        }
        float c1 = dot_part<KPL>(pa, qa), c2 = dot_part<KPL>(pb, qbd), g = dot_part<KPL>(pb, pa);
        wave_sum3(c1, c2, g);
        const float era = rlf(C0.era, s), erb = rlf(C0.erb, s);
        const float aa = rlf(C0.aa, s), ab = rlf(C0.ab, s), ba = rlf(C0.ba, s), bb = rlf(C0.bb, s);
        const float wa = fmaf(-eta, c1, era);
        const float m = fmaf(sr, aa - 1.f, 1.f), gw = sr * wa;
        const float wb = fmaf(-eta, fmaf(gw, g, m * c2), erb);
        Row<KPL> q1;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          const f2 q0 = qa.v[e], a0 = pa.v[e], b0 = pb.v[e];
          q1.v[e] = aa * q0 + wa * a0;
          plA.v[e] = ba * a0 + wa * q0;
          const f2 qb0 = sr * q1.v[e] + QB[slot].v[e];
          plB.v[e] = bb * b0 + wb * qb0;
          q.v[e] = ab * qb0 + wb * b0;
        }
        st<KPL, kSC1>(urs, voff, osa, plA);
        st<KPL, kSC1>(urs, voff, osb, plB);
        st<KPL>(irs, voff, osia, q1);
        st<KPL>(irs, voff, osi, q);
        {
          const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(PV[slot]));
          if (static_cast<int32_t>(v - seen) > 0) seen = v;
          const uint32_t lag = base + static_cast<uint32_t>(max(j - D + 1, 0));  // stores of pairs <= j-D landed
          if (static_cast<int32_t>(lag - pub) > 0) pub = lag;
          if constexpr (P == 1) prog_store(my_prog, pub);
          else if (s % P == 0) prog_store(my_prog, pub);
          stream_wait(nb_prog, base + nneed, seen, my_prog, base + static_cast<uint32_t>(j + 1), pub, err, lbase + L, wst);
        }
        PA[slot] = ld<KPL, kSC1>(urs, voff, nua);
        PB[slot] = ld<KPL, kSC1>(urs, voff, nub);
        QA[slot] = ld<KPL>(irs, voff, nia);
        QB[slot] = ld<KPL>(irs, voff, nib);
        if (s % P == 0) PV[slot] = prog_load_lanes(nb_prog);
      }
      C0 = chunk_convert(C1, eta);
      C1 = chunk_load_n<CH>(R, c + 2, npairs, lane);
    }
  gen_done:;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every store of this wave has landed
  prog_store(my_prog, base + static_cast<uint32_t>(npairs));
  {  // per-slot wait statistics (err words 4 + 8 * slot + 4 .. 7), accumulated over launches
    int32_t* d = err + 4 + 8 * (lbase + L) + 4;
    const uint32_t dt = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime() - t_start);
    if (lane == 0) {
      d[0] += static_cast<int32_t>(wst.waits);
      d[1] += static_cast<int32_t>(wst.ticks);
      d[2] += static_cast<int32_t>(dt);
      d[3] += npairs;
    }
  }
}

template <int KPL, int D, int CH, int P>
void dispatch_stream_d(hipStream_t st, const StreamWave* sw, int nw, int lbase, const PairRec* recs, float* U, float* I,
                       uint64_t ub, uint64_t ib, float eta, int32_t* prog, uint64_t prog_bytes, uint32_t base,
                       int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
  hipExtLaunchKernelGGL((k_sweep_stream<KPL, D, CH, P>), dim3(static_cast<unsigned>(nw)), dim3(64), 0, st, ev0, ev1, 0, sw,
                        nw, lbase, reinterpret_cast<const u4v*>(recs), U, I, ub, ib, eta, prog, prog_bytes, base, err);
}

// ring depth D with a record chunk of the largest multiple of D (and of P) that fits a wave (<= 60
// pairs); P = pairs between two hand-off word updates (1, 4 or 16)
template <int KPL>
void dispatch_stream(int ring, int period, hipStream_t st, const StreamWave* sw, int nw, int lbase, const PairRec* recs,
                     float* U, float* I, uint64_t ub, uint64_t ib, float eta, int32_t* prog, uint64_t prog_bytes,
                     uint32_t base, int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
#define MF_D(D, CH, P) \
  dispatch_stream_d<KPL, D, CH, P>(st, sw, nw, lbase, recs, U, I, ub, ib, eta, prog, prog_bytes, base, err, ev0, ev1)
  if (ring == 3 && period == 1) MF_D(3, 48, 1);
  else if (ring == 3 && period == 4) MF_D(3, 48, 4);
  else if (ring == 3 && period == 16) MF_D(3, 48, 16);
  else if (ring == 5 && period == 4) MF_D(5, 60, 4);
  else if (ring == 7 && period == 4) MF_D(7, 56, 4);
  else if (ring == 7 && period == 1) MF_D(7, 56, 1);
#undef MF_D
}

template <int KPL>
int stream_capacity() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  // the deepest ring holds the most registers: its occupancy bounds every depth
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sweep_stream<KPL, 7, 56, 1>, 64, 0) != hipSuccess) return 0;
  return cus * per_cu;
}

}  // namespace

int sweep_stream_capacity(int k) {
  switch (k) {
    case 64: return stream_capacity<1>();
    case 128: return stream_capacity<2>();
    case 256: return stream_capacity<4>();
    default: return 0;
  }
}

bool stream_ring_supported(int ring, int period) {
  return (ring == 3 && (period == 1 || period == 4 || period == 16)) || (ring == 5 && period == 4) ||
         (ring == 7 && (period == 1 || period == 4));
}

void launch_sweep_stream(int ring, int period, hipStream_t st, const StreamWave* sw, int nw, int lbase, const PairRec* recs,
                         float* U, float* I, uint64_t u_bytes, uint64_t i_bytes, int k, float eta, int32_t* prog,
                         uint64_t prog_bytes, uint32_t base, int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
  if (nw <= 0) return;
#define MF_ST(KPL) dispatch_stream<KPL>(ring, period, st, sw, nw, lbase, recs, U, I, u_bytes, i_bytes, eta, prog, prog_bytes, base, err, ev0, ev1)
  switch (k) {
    case 64: MF_ST(1); break;
    case 128: MF_ST(2); break;
    case 256: MF_ST(4); break;
    default: break;
  }
#undef MF_ST
}

}  // namespace mfhip
