// kernels_online_sweep.hip -- the f32 online micro-batch in one persistent launch
// (SGDUpdater.nextFactors in sequence order, core/FactorUpdater.scala:37-45, as FlinkOnlineMF.scala's
// item operator applies it: FlinkOnlineMF.scala:112-137).  k <= 256; the f64 batch and wider f32 rows
// keep k_online_sweep (kernels_det.hip).
//
// Schedule (kernels_online.hip, unchanged): wave w owns the items with row % W == w and applies
// their updates in sequence order; an update waits for its user's earlier updates (other waves)
// through a per-user ticket, the count of that user's updates done so far in the batch, and runs
// when the ticket equals its useq.  A wave's updates are in increasing sequence position, so the
// earliest unfinished update is always runnable: with every wave resident there is no deadlock.
//
// Pipeline (the hot item's wave is the batch's critical path, ~2.3k chained updates per NFLX 1M
// batch; the previous kernel spent ~1.3 us on each, almost all of it memory round trips in the
// chain: the ticket reads of the next updates were looked at after a ~128-add fold, the item row was
// loaded when the item changed, and the previous update's stores were drained every update):
//   * updates in chunks of 16 with the update's index a compile-time constant (every field a
//     constant-lane v_readlane), full chunks without exit tests;
//   * rows prefetched after the current update's stores: the general path's user AND item rows two
//     updates ahead (an item row is only ever written by this wave; an item that recurs after
//     another one was stored at the switch, before the prefetch, so a prefetched item row is always
//     current), a heavy item's wave (one item: its row loaded once, stored once) its user rows
//     kSingle updates ahead; a user row is prefetched only when its ticket is due, i.e. every
//     earlier update of that user, this wave's included, has landed;
//   * ticket polls read two (general) or kSingle (single item) updates after they are issued, and
//     tickets published as many updates late: update j waits only for update j - 2's (j - kSingle's)
//     stores (vmcnt(NW): the operations issued after them).  vmcnt counts in issue order, so
//     a wave waits, in effect, for the nearest of these distances: with every distance 2 the hot
//     item's wave (the batch's critical path) waited on each update's stores two updates later
//     (NFLX 1M batch 0.835 ms; profiles/r06_online_batch_timeline.txt).  A wave publishes every
//     pending ticket before it blocks;
//   * the dot product is online_f32.hpp's fixed tree (~10 dependent VALU operations, not a 128-add
//     chain); the level replay uses the same arithmetic, so both give the same factors bit for bit.
// Every update issues the same vector-memory operations (out-of-range offsets for rows it does not
// move), so NW is a constant: tools/isa_check.py checks it against the built code.
//
// Bytes per update: B_f32(k) = 16k + 20 (an item row held in registers across a run
// moves less) plus the 16-B update record, its 4-B useq and the ticket word.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

#include "online_f32.hpp"
#include "ticket_wait.hpp"

constexpr int kSC1 = 16;                // buffer cache policy: sc1 (L1 bypass, write-through)
constexpr uint32_t kOOB = 0xFFFFF000u;  // a row offset past the slab: the load returns 0, no store
constexpr int kOnChunk = 16;            // updates per register chunk
// The general path publishes a ticket two updates late, the single-item path kSingle late, and
// prefetches its user rows and reads its ticket polls kSingle updates on (tools/isa_check.py checks
// the built code against both).  Measured on NFLX 1M batches (gpurun_out/r6f, r6g): every wave at
// 2 -- 0.835 ms per launch; single 4 / general 4 -- 0.663 ms; single 8 / general 8 -- 0.806 ms
// (a ticket published late holds its consumers back, and the hot wave's users come from the
// general waves).
constexpr int kSingle = 4;

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xFFFFF000ull ? 0xFFFFF000u : static_cast<uint32_t>(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}
// One row of k floats as this lane's KPL elements (online_f32.hpp layout).  FULL: one access of
// 4 KPL bytes.  Else KPL 4-B accesses; a lane's element past k reads a clamped in-row address and
// is zeroed, and its store is masked off (a voffset past the slab would not do: with an
// out-of-range row offset in soffset the 32-bit sum can wrap back into range).
template <int KPL, bool FULL>
struct Rows {
  static constexpr int OPS = FULL ? 1 : KPL;  // vector-memory operations per row
  uint32_t voff[OPS];
  bool valid[OPS];
  __device__ Rows(int lane, int k) {
    if constexpr (FULL) {
      voff[0] = static_cast<uint32_t>(lane) * 4u * KPL;
      valid[0] = true;
    } else {
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        valid[c] = lane + 64 * c < k;
        voff[c] = static_cast<uint32_t>(valid[c] ? lane + 64 * c : k - 1) * 4u;
      }
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t off, float (&v)[KPL]) const {
    if constexpr (FULL && KPL == 1) {
      v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff[0], off, kSC1));
    } else if constexpr (FULL && KPL == 2) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff[0], off, kSC1);
      v[0] = __uint_as_float(x[0]);
      v[1] = __uint_as_float(x[1]);
    } else if constexpr (FULL && KPL == 4) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[0], off, kSC1);
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = __uint_as_float(x[c]);
    } else {
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        const float x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff[c], off, kSC1));
        v[c] = valid[c] ? x : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t rs, uint32_t off, const float (&v)[KPL]) const {
    if constexpr (FULL && KPL == 1) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), rs, voff[0], off, kSC1);
    } else if constexpr (FULL && KPL == 2) {
      using u2 = uint32_t __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(v[0]), __float_as_uint(v[1])}, rs, voff[0], off, kSC1);
    } else if constexpr (FULL && KPL == 4) {
      using u4 = uint32_t __attribute__((ext_vector_type(4)));
      const u4 d = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff[0], off, kSC1);
      // two wait states before the data VGPRs may be rewritten (gfx950 store-data hazard, pair_device.hpp)
      asm volatile("s_nop 1" ::"v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]));
    } else {
      // lane 0 is valid for every c (KPL = ceil(k / 64)), so every store issues
#pragma unroll
      for (int c = 0; c < KPL; ++c)
        if (valid[c]) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[c]), rs, voff[c], off, kSC1);
    }
  }
};

// Update x of a wave: lane (x % 16) of chunk x / 16 holds its record (user row, item row, rating,
// useq); records past the wave's end read as zeros (buffer range).
struct OnChunk {
  uint32_t u, i, q;
  float r;
};

__device__ __forceinline__ void publish(int32_t* t, int32_t v, int lane) {
  if (lane == 0) __hip_atomic_store(t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t poll_issue(const int32_t* t) {
  return __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70 & ~0xF);
}

// One wave's updates.  UD: user rows prefetched UD updates ahead (guarded by the user's ticket);
// TD: a ticket poll is read TD updates after it is issued; PD: tickets published PD updates late.
// vmcnt counts in issue order, so a wave waits, in effect, for the oldest of those distances --
// and for its item rows, prefetched two updates ahead (an item that recurs after a switch must be
// loaded after its store).  SINGLE: the wave holds one item (the plan's heavy-item waves), so the
// item row is loaded once and stored once, and every distance can be deeper: the hot item's chain
// -- the batch's critical path -- no longer waits for each update's row stores two updates later
// (NFLX 1M batch: 0.835-0.863 ms with every distance 2, the chain ~360 ns per update).
template <int KPL, bool FULL, int UD, int TD, int PD, bool SINGLE>
__device__ __forceinline__ void online_wave(const int64_t jb, const int32_t cnt, const DetEntry* __restrict__ ent,
                                            const uint32_t* __restrict__ useq, float* U, float* I, uint64_t u_bytes,
                                            uint64_t i_bytes, int k, float eta, int32_t* ticket, int32_t* dummy_ticket,
                                            int32_t* err) {
  using R = Rows<KPL, FULL>;
  constexpr int CH = kOnChunk;
  static_assert(UD + TD <= CH && 2 <= UD && 2 <= TD && 1 <= PD, "ring distances (s + UD + TD < 2 CH)");
  // operations issued after update j-PD's stores up to update j's publish: j-PD's loads and poll,
  // then PD-1 whole updates (publish, stores, loads, poll); SINGLE moves no item row per update
  constexpr int IO = SINGLE ? 0 : R::OPS;  // item-row operations per update (load, store)
  constexpr int NW = (R::OPS + IO + 1) + (PD - 1) * (1 + R::OPS + IO + R::OPS + IO + 1);
  static_assert(NW < 64, "vmcnt range");
  const int lane = threadIdx.x;
  const R rows(lane, k);
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);
  const __amdgpu_buffer_rsrc_t ers = raw_rsrc(ent + jb, static_cast<uint64_t>(cnt) * sizeof(DetEntry));
  const __amdgpu_buffer_rsrc_t qrs = raw_rsrc(useq + jb, static_cast<uint64_t>(cnt) * 4u);
  const uint32_t rowb = static_cast<uint32_t>(k) * 4u;
  auto chunk = [&](int c) {
    const uint32_t x = static_cast<uint32_t>(c * CH + (lane & (CH - 1)));
    const auto e = __builtin_amdgcn_raw_buffer_load_b128(ers, x * 16u, 0, 0);
    const double r = __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(e[3]) << 32) | e[2]));
    return OnChunk{e[0], e[1], __builtin_amdgcn_raw_buffer_load_b32(qrs, x * 4u, 0, 0), static_cast<float>(r)};
  };
  OnChunk C0 = chunk(0), C1 = chunk(1);
  auto fu = [&](int s) { return s < CH ? rl(C0.u, s) : rl(C1.u, s - CH); };
  auto fi = [&](int s) { return s < CH ? rl(C0.i, s) : rl(C1.i, s - CH); };
  auto fq = [&](int s) { return s < CH ? rl(C0.q, s) : rl(C1.q, s - CH); };
  auto fr = [&](int s) { return __uint_as_float(s < CH ? rl(__float_as_uint(C0.r), s) : rl(__float_as_uint(C1.r), s - CH)); };

  float P[UD][KPL], Q[2][KPL];
  int32_t okP[UD];  // the slot's user row was prefetched (its ticket was due)
  int32_t tk[TD];   // ticket polls, read TD updates after they are issued
  // prologue: the user rows of updates 0 .. UD-1 (their tickets read here), the item rows of
  // updates 0 and 1 (SINGLE: the one item row), polls of updates UD .. UD+TD-1
#pragma unroll
  for (int x = 0; x < UD; ++x) {
    const bool live = x < cnt;
    const uint32_t u = fu(x);
    okP[x] = !live || __builtin_amdgcn_readfirstlane(poll_issue(ticket + u)) == static_cast<int32_t>(fq(x));
    rows.load(urs, live && okP[x] ? u * rowb : kOOB, P[x]);
  }
  if constexpr (SINGLE) {
    rows.load(irs, fi(0) * rowb, Q[0]);  // (every entry of the wave has this item)
  } else {
#pragma unroll
    for (int x = 0; x < 2; ++x) rows.load(irs, x < cnt && (x == 0 || fi(1) != fi(0)) ? fi(x) * rowb : kOOB, Q[x]);
  }
#pragma unroll
  for (int x = 0; x < TD; ++x) tk[x] = poll_issue(x + UD < cnt ? ticket + fu(x + UD) : dummy_ticket);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  int32_t* pend[PD];  // the tickets of updates j-PD .. j-1 (word, value), published PD updates late
  int32_t pv[PD];
#pragma unroll
  for (int x = 0; x < PD; ++x) {
    pend[x] = dummy_ticket;
    pv[x] = 0;
  }
  auto publish_all = [&] {
#pragma unroll
    for (int x = 0; x < PD; ++x) {
      publish(pend[x], pv[x], lane);
      pend[x] = dummy_ticket;
    }
  };
  float q[KPL];  // the current item's row
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = SINGLE ? Q[0][c] : 0.f;
  uint32_t cur_i = 0;
  const uint32_t single_off = SINGLE ? fi(0) * rowb : 0u;  // (the chunks move on; the item does not)

  // update j (chunk-relative s, a compile-time constant once unrolled); s + UD + TD < 2 CH
  auto update = [&](const int s, const int32_t j) {
    const int slot = s & 1, us = s % UD, ts = s % TD;
    const uint32_t u = fu(s), i = fi(s);
    const int32_t qseq = static_cast<int32_t>(fq(s));
    const float r = fr(s);
    const uint32_t uD = fu(s + UD), qD = fq(s + UD), uT = fu(s + UD + TD);
    // 1. the user row, when its ticket was not due at prefetch time: publish the pending tickets
    //    (after their stores), wait for ours, load now
    if (!okP[us]) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      publish_all();
      wait_ticket_or_fail(ticket + u, qseq, err, lane);  // no early return (ticket_wait.hpp)
      rows.load(urs, u * rowb, P[us]);
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    // 2. the item row: prefetched when the item changed, else the one in registers
    if constexpr (!SINGLE) {
      if (j == 0 || i != cur_i) {
#pragma unroll
        for (int c = 0; c < KPL; ++c) q[c] = Q[slot][c];
      }
      cur_i = i;
    }
    // 3. the update (online_f32.hpp)
    float p[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) p[c] = P[us][c];
    const float le = f32_err(static_cast<double>(r), f32_wave_sum(f32_lane_dot<KPL>(p, q)), eta);
    f32_sgd_next<KPL>(p, q, le);
    // 4. update j-PD's stores have landed (NW younger operations may still fly): publish its ticket
    wait_vmcnt<NW>();
    publish(pend[0], pv[0], lane);
#pragma unroll
    for (int x = 0; x + 1 < PD; ++x) {
      pend[x] = pend[x + 1];
      pv[x] = pv[x + 1];
    }
    pend[PD - 1] = ticket + u;
    pv[PD - 1] = qseq + 1;
    // 5. stores: the user row, and the item row when the next update is on another item (or none)
    const bool live1 = j + 1 < cnt, live2 = j + 2 < cnt, liveD = j + UD < cnt;
    rows.store(urs, u * rowb, p);
    if constexpr (!SINGLE) {
      const uint32_t i1 = fi(s + 1);
      rows.store(irs, !live1 || i1 != i ? i * rowb : kOOB, q);
    }
    // 6. prefetch: update j+UD's user row into this user slot if its ticket (polled TD updates ago) is
    //    due -- every earlier update of that user, this wave's included, has landed -- and update
    //    j+2's item row if it starts another item's run
    const int32_t okN = !liveD || __builtin_amdgcn_readfirstlane(tk[ts]) == static_cast<int32_t>(qD);
    rows.load(urs, liveD && okN ? uD * rowb : kOOB, P[us]);
    if constexpr (!SINGLE) {
      const uint32_t i1 = fi(s + 1), i2 = fi(s + 2);
      rows.load(irs, live2 && i2 != i1 ? i2 * rowb : kOOB, Q[slot]);
    }
    okP[us] = okN;
    // 7. poll update j+UD+TD's ticket (read at j+TD)
    tk[ts] = poll_issue(j + UD + TD < cnt ? ticket + uT : dummy_ticket);
  };
  // full chunks run their updates with no exit test in between (ticket_wait.hpp, kernels_detsweep.hip)
  for (int32_t c0 = 0;; c0 += CH) {
    if (c0 + CH <= cnt) {
#pragma unroll
      for (int s = 0; s < CH; ++s) update(s, c0 + s);
    } else {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        if (c0 + s >= cnt) goto done;
        update(s, c0 + s);
      }
    }
    C0 = C1;
    C1 = chunk(c0 / CH + 2);
  }
done:
  if constexpr (SINGLE) rows.store(irs, single_off, q);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  publish_all();
}

// Waves [0, nsingle) hold one item each (the online plan's heavy-item waves, kernels_online.hip).
// skip (may be null): a non-zero count there -- ids the device lookup did not find -- makes every
// wave return at once (the host was not waiting for that count; it rebuilds the batch and runs it
// again).
template <int KPL, bool FULL>
__global__ __launch_bounds__(64) void k_online_f32(const int64_t* __restrict__ wbeg, const DetEntry* __restrict__ ent,
                                                   const uint32_t* __restrict__ useq, float* U, float* I,
                                                   uint64_t u_bytes, uint64_t i_bytes, int k, float eta,
                                                   int32_t* ticket, int32_t* dummy_ticket, int32_t* err, int nsingle,
                                                   const int32_t* __restrict__ skip) {
  if (skip && *skip != 0) return;
  const int64_t jb = wbeg[blockIdx.x];
  const int32_t cnt = static_cast<int32_t>(wbeg[blockIdx.x + 1] - jb);
  if (cnt <= 0) return;
  dummy_ticket += 16 * static_cast<int64_t>(blockIdx.x);  // this wave's own scratch line
  if (static_cast<int>(blockIdx.x) < nsingle)
    online_wave<KPL, FULL, kSingle, kSingle, kSingle, true>(jb, cnt, ent, useq, U, I, u_bytes, i_bytes, k, eta, ticket,
                                                            dummy_ticket, err);
  else
    online_wave<KPL, FULL, 2, 2, 2, false>(jb, cnt, ent, useq, U, I, u_bytes, i_bytes, k, eta, ticket, dummy_ticket,
                                           err);
}

template <int KPL, bool FULL>
int capacity_of() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_online_f32<KPL, FULL>, 64, 0) != hipSuccess) return 0;
  return cus * per_cu;
}

}  // namespace

bool online_f32_supports(int k) { return k >= 1 && k <= 256; }

// KPL = ceil(k / 64) floats per lane; FULL (contiguous, one access per row) when k == 64 KPL, KPL != 3
int online_f32_capacity(int k) {
  if (k <= 64) return k == 64 ? capacity_of<1, true>() : capacity_of<1, false>();
  if (k <= 128) return k == 128 ? capacity_of<2, true>() : capacity_of<2, false>();
  if (k <= 192) return capacity_of<3, false>();
  if (k <= 256) return k == 256 ? capacity_of<4, true>() : capacity_of<4, false>();
  return 0;
}

void launch_online_f32(hipStream_t st, int nw, const int64_t* wbeg, const DetEntry* ent, const uint32_t* useq, float* U,
                       float* I, uint64_t u_bytes, uint64_t i_bytes, int k, double eta, int32_t* ticket,
                       int32_t* dummy_ticket, int32_t* err, int nsingle, const int32_t* skip, hipEvent_t ev0,
                       hipEvent_t ev1) {
  if (nw <= 0 || !online_f32_supports(k)) return;
  const dim3 g(static_cast<unsigned>(nw)), b(64);
  const float e = static_cast<float>(eta);
#define MF_ON(KPL, FULL)                                                                                    \
  hipExtLaunchKernelGGL((k_online_f32<KPL, FULL>), g, b, 0, st, ev0, ev1, 0, wbeg, ent, useq, U, I, u_bytes, \
                        i_bytes, k, e, ticket, dummy_ticket, err, nsingle, skip)
  if (k == 64) MF_ON(1, true);
  else if (k < 64) MF_ON(1, false);
  else if (k == 128) MF_ON(2, true);
  else if (k < 128) MF_ON(2, false);
  else if (k <= 192) MF_ON(3, false);
  else if (k == 256) MF_ON(4, true);
  else MF_ON(4, false);
#undef MF_ON
}

}  // namespace mfhip
