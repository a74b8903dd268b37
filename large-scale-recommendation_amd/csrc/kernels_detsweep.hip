// kernels_detsweep.hip -- deterministic f64 DSGD superstep as ONE persistent launch (bit-exact
// with the reference's sequential order, DSGDforMF.scala:378-418).  Compiled with
// -ffp-contract=off: every a*b+c stays two rounded operations, as on the JVM.
//
// Schedule (plan.hpp DetSweepLayout / build_det_step): each item of a rating block belongs to
// one wave, which applies all updates of its items in the block's shuffled order (:392-393).
// An update depends on the previous update of its item (same wave: program order) and of its
// user (another wave, in general); the latter is awaited through a per-user ticket, the number
// of that user's updates done so far in this superstep.  The entry carries useq = how many
// earlier updates of its user the shuffled order has, so it runs when ticket[u] == useq and then
// publishes useq + 1.  Every wave's entries are in increasing shuffle position, so the unfinished
// entry with the smallest position is always runnable: with every wave resident there is no
// deadlock (the host launches at most the co-resident wave count).  Consecutive entries of the
// same item keep the item row in registers (the hot items' long chains).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms row 1): the user rows a
// wave publishes are stored sc1 (write-through), the wave drains them (s_waitcnt vmcnt(0)), then
// lane 0 stores the ticket with an agent-scope relaxed atomic; the consumer polls the ticket with
// agent-scope relaxed loads (sc1) and loads the user row with sc1 loads only after the poll has
// matched.  Item rows are touched by one wave only and are stored / reloaded with sc1 as well
// (the wave drains its stores before its next entry).  A wait longer than ~1 s sets err[0]; every
// wave then leaves (the host reports MF_ERR_TIMEOUT and refuses the partial model).
//
// Bytes per update: B_f64(k) = 32k + 24 plus the 20-B entry and the ticket word.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>


#include "kernels.hpp"

namespace mfhip {
namespace {

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ double rld(double v, int l) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffffu), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b >> 32), l));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

__device__ __forceinline__ double uniform(double v) { return rld(v, 0); }

#include "seq_fold.hpp"
#include "ticket_wait.hpp"

// Entry fields of a wave's entry list, 64 per lane-register chunk (the host pads every entry
// array by 64, so a chunk load never needs a bounds branch).
struct DetChunk {
  uint32_t u, i, q;
  double r;
};
__device__ __forceinline__ DetChunk det_chunk(const uint32_t* eu, const uint32_t* ei, const uint32_t* eq,
                                              const double* er, int64_t x) {
  return DetChunk{eu[x], ei[x], eq[x], er[x]};
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xFFFFF000ull ? 0xFFFFF000u : static_cast<uint32_t>(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}
constexpr int kSC1 = 16;                   // buffer cache policy: sc1 (L1 bypass, write-through)
constexpr uint32_t kOOB = 0xFFFFF000u;     // a row offset past the slab: the load returns 0, no store

// Ticket words and lambda / omega through raw buffers with the word's byte offset in an SGPR: one
// scalar shift per access instead of a 64-bit address and a select, and "none" is the out-of-range
// offset kOOB (the load returns 0, the store is dropped) instead of a per-wave dummy word.  Every
// lane touches the same word (same value): no exec mask around a publish.  sc1 loads and stores,
// the agent-scope relaxed atomics of the hand-off (MI355X_MICROARCH.md, valid forms: buffer_load_dword
// sc1 poll).
__device__ __forceinline__ int32_t poll_issue(__amdgpu_buffer_rsrc_t trs, uint32_t off) {
  return static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(trs, 0, off, kSC1));
}
__device__ __forceinline__ int32_t poll(__amdgpu_buffer_rsrc_t trs, uint32_t off) {
  return __builtin_amdgcn_readfirstlane(poll_issue(trs, off));
}
__device__ __forceinline__ void publish(__amdgpu_buffer_rsrc_t trs, uint32_t off, int32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(v), trs, 0, off, kSC1);
}
__device__ __forceinline__ double ld_reg(__amdgpu_buffer_rsrc_t rs, uint32_t row) {
  const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, 0, row * 8u, kSC1);
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(x[1]) << 32) | x[0]));
}

template <int KPL>
struct DRow {
  double v[KPL];
};
// f64 row of k: lane holds elements lane + 64c at byte voff[c] of the row (voff[c] is past any
// slab for elements >= k: those lanes load zeros and store nothing); an out-of-range row offset
// loads zeros and stores nothing.
template <int KPL>
__device__ __forceinline__ DRow<KPL> ldrow(__amdgpu_buffer_rsrc_t rs, const uint32_t (&voff)[KPL], uint32_t off) {
  DRow<KPL> r;
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff[c], off, kSC1);
    r.v[c] = __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(x[1]) << 32) | x[0]));
  }
  return r;
}
template <int KPL>
__device__ __forceinline__ void strow(__amdgpu_buffer_rsrc_t rs, const uint32_t (&voff)[KPL], uint32_t off,
                                      const double (&v)[KPL]) {
  using u2 = uint32_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const uint64_t b = static_cast<uint64_t>(__double_as_longlong(v[c]));
    __builtin_amdgcn_raw_buffer_store_b64(u2{static_cast<uint32_t>(b), static_cast<uint32_t>(b >> 32)}, rs, voff[c],
                                          off, kSC1);
  }
}

// vmcnt(N) in the gfx9 encoding (expcnt 7, lgkmcnt 15 left unconstrained).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70 & ~0xF);
}

// k_det_sweep2: per wave, the entries of its items in shuffled order, with a two-deep pipeline for
// the per-item chains (the hot item's wave is the superstep's critical path: ~26k chained updates
// per NFLX superstep):
//   * entries in chunks of kDetChunk with the entry index inside a chunk a compile-time constant
//     (unrolled), so every field is a v_readlane with a constant lane and the body is straight-line
//     code whose wait counts the compiler tracks exactly;
//   * rows prefetched TWO entries ahead (slot s % 2), issued after the current entry's stores, so
//     a prefetched item row always sees this wave's own earlier store; the user row of entry j+2 is
//     loaded only if its ticket -- polled two entries earlier still -- was already ready, else the
//     entry waits and loads when it runs (the rare slow path);
//   * a ticket is published TWO entries late: entry j waits only for entry j-2's stores
//     (vmcnt(6 KPL + 7): the operations issued after them), so a store's write-through latency
//     overlaps two entries of compute.  A wave publishes every pending ticket before it blocks on
//     one, so no published ticket ever waits on a blocked wave and the unfinished entry with the
//     smallest shuffle position stays runnable (no deadlock with every wave resident);
//   * FULL (k == 64 KPL): the dot's sequential fold in registers (seq_fold_dpp: permlane swaps and
//     DPP broadcasts, ~6.6 instead of ~11-13 cycles per f64 add), else through LDS (seq_fold).
constexpr int kDetChunk = 16;

// The update rule (AR) of an entry, both in the reference's rounding (no FMA):
//   kArDsgd: DSGDforMF.scala:405-410, lambda / omega per row (regU / regI);
//   kArNext: SGDUpdater.nextFactors (core/FactorUpdater.scala:37-45), the online micro-batch:
//            le = lr * e, p' = p + le * q, q' = q + le * p (old rows), no regularisation.  Its
//            lambda / omega buffers are empty ranges: the loads still issue (so every vmcnt the
//            hand-off counts is the same instruction count) but return 0 and touch no memory.
constexpr int kArDsgd = 0, kArNext = 1;
template <int AR>
constexpr uint64_t reg_bytes() {
  return AR == kArDsgd ? 0xFFFFF000ull : 0ull;
}
// (p', q') from the rows before the update, e = r - p.q
template <int AR>
__device__ __forceinline__ void update_pair(double p, double q, double e, double eta, double ru, double ri,
                                            double& pn, double& qn) {
  if constexpr (AR == kArDsgd) {
    pn = p - eta * (ru * p - e * q);  // :407-408
    qn = q - eta * (ri * q - e * p);  // :409-410 (old p)
  } else {
    const double le = eta * e;  // learningRate * e * i == (learningRate * e) * i
    pn = p + le * q;
    qn = q + le * p;
  }
}


// One wave's entries.  SINGLE (DetWave::flags & kDetWaveSingleItem): every entry updates the same
// item, so its row and lambda / omega are loaded once and stored once at the end, and an entry moves
// only its user row.  Vector-memory operations per entry, in issue order (the wait before a
// ticket is published counts on them -- change the entry, change NW):
//   generic: publish 1 | user store KPL, item store KPL | user load KPL, item load KPL, ru 1, ri 1, poll 1
//   SINGLE:  publish 1 | user store KPL                 | user load KPL,                ru 1,       poll 1
// NW = the operations issued after entry j-2's stores up to entry j's publish: entry j-2's loads plus
// all of entry j-1's: generic (2 KPL + 3) + (4 KPL + 4) = 6 KPL + 7, SINGLE (KPL + 2) + (2 KPL + 3) = 3 KPL + 5.
template <int KPL, bool FULL, bool SINGLE, int AR = kArDsgd>
__device__ __forceinline__ void det_wave(const DetWave d, const uint32_t* __restrict__ eu, const uint32_t* __restrict__ ei,
                                         const uint32_t* __restrict__ eq, const double* __restrict__ er, double* U,
                                         double* I, uint64_t u_bytes, uint64_t i_bytes, const double* __restrict__ regU,
                                         const double* __restrict__ regI, int k, double eta, int32_t* ticket,
                                         int32_t* dummy_ticket, int32_t* err, double* lds, int lane) {
  constexpr int CH = kDetChunk;
  constexpr int NW = SINGLE ? 3 * KPL + 5 : 6 * KPL + 7;
  static_assert(NW < 64, "vmcnt range");
  const int32_t cnt = d.count;  // 32-bit: the entry tests are scalar compares, not 64-bit VALU ones
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);
  const __amdgpu_buffer_rsrc_t trs = raw_rsrc(ticket, 0xFFFFF000ull);  // offsets are user rows * 4
  const __amdgpu_buffer_rsrc_t rus = raw_rsrc(regU, reg_bytes<AR>()), ris = raw_rsrc(regI, reg_bytes<AR>());
  uint32_t voff[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) voff[c] = lane + 64 * c < k ? static_cast<uint32_t>(lane + 64 * c) * 8u : 0x80000000u;
  const uint32_t rowb = static_cast<uint32_t>(k) * 8u;
  // chunk c: entry begin + CH c + (lane % CH) in every lane (entry arrays are padded past a wave's end)
  auto chunk = [&](int64_t c) { return det_chunk(eu, ei, eq, er, d.begin + c * CH + (lane & (CH - 1))); };
  DetChunk C0 = chunk(0), C1 = chunk(1);
  // field of entry s + dj of chunk C0 (C1 past the chunk), s + dj < 2 CH
  auto fu = [&](int s) { return s < CH ? rl(C0.u, s) : rl(C1.u, s - CH); };
  auto fi = [&](int s) { return s < CH ? rl(C0.i, s) : rl(C1.i, s - CH); };
  auto fq = [&](int s) { return s < CH ? rl(C0.q, s) : rl(C1.q, s - CH); };

  DRow<KPL> P[2], Q[2];
  double RU[2], RI[2];
  int32_t okP[2];  // the slot's user row was prefetched (its ticket was ready)
  int32_t tk[2];   // ticket polls, two entries ahead of the prefetch that reads them
  // prologue: entries 0 and 1 now (their tickets polled and read here), polls of entries 2 and 3
  const uint32_t item0 = fi(0);  // SINGLE: the wave's one item
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const bool live = x < cnt;
    const uint32_t u = fu(x), i = fi(x), q = fq(x);
    okP[x] = !live || poll(trs, u * 4u) == static_cast<int32_t>(q & kDetUseqMask);
    P[x] = ldrow<KPL>(urs, voff, live && okP[x] ? u * rowb : kOOB);
    RU[x] = ld_reg(rus, live ? u : 0u);
    if (!SINGLE || x == 0) {
      Q[x] = ldrow<KPL>(irs, voff, live && !(x > 0 && i == fi(x - 1)) ? i * rowb : kOOB);
      RI[x] = ld_reg(ris, live ? i : 0u);
    }
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) tk[x] = poll_issue(trs, x + 2 < cnt ? fu(x + 2) * 4u : kOOB);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  uint32_t pend0 = kOOB;  // entry j-2's ticket word (byte offset; kOOB: none) and value
  int32_t pv0 = 0;
  uint32_t pend1 = kOOB;  // entry j-1's
  int32_t pv1 = 0;
  double q[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = SINGLE ? Q[0].v[c] : 0.0;
  const double ri_single = SINGLE ? uniform(RI[0]) : 0.0;

  // one entry (chunk-relative s, a compile-time constant once unrolled)
#if defined(MFHIP_EXPERIMENTS) && defined(MFHIP_DET_PROBE)
  uint64_t pc[4] = {0, 0, 0, 0};  // experiment build: shader cycles per phase, printed by wave 0
  uint64_t pt = __builtin_amdgcn_s_memtime();
  auto stamp = [&](int x) { const uint64_t n = __builtin_amdgcn_s_memtime(); pc[x] += n - pt; pt = n; };
#else
  auto stamp = [](int) {};
#endif
  // keep / defer the item row (same item as the previous / the next entry of this wave): found
  // here from the entry fields, so the host build does not scan the entries for it
  uint32_t prev_i = 0xFFFFFFFFu;  // the previous entry's item (none before entry 0)
  auto entry = [&](const int s, const int32_t j) {
    const int slot = s & 1;
    const uint32_t u = fu(s), qf = fq(s);
    const uint32_t i = SINGLE ? item0 : fi(s);
    const bool keepq = !SINGLE && i == prev_i;
    const bool deferq = !SINGLE && j + 1 < cnt && fi(s + 1) == i;
    const double r = rld(s < CH ? C0.r : C1.r, s);
    const int32_t useq = static_cast<int32_t>(qf & kDetUseqMask);
    const uint32_t u2 = fu(s + 2), q2 = fq(s + 2), u4 = fu(s + 4);
    const uint32_t i2 = SINGLE ? item0 : fi(s + 2);
    // 1. the user row, when its ticket was not ready at prefetch time (rare): publish every
    //    pending ticket (after its stores), wait for ours, load now
    if (!okP[slot]) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      publish(trs, pend0, pv0);
      publish(trs, pend1, pv1);
      pend0 = pend1 = kOOB;
      wait_ticket_or_fail(ticket + u, useq, err, lane);  // no early return (ticket_wait.hpp)
      P[slot] = ldrow<KPL>(urs, voff, u * rowb);
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    // 2. compute entry j (DSGDforMF.scala:405-410, the reference's rounding, no FMA)
    if (!SINGLE && !keepq) {
#pragma unroll
      for (int c = 0; c < KPL; ++c) q[c] = Q[slot].v[c];
    }
    const double ru = uniform(RU[slot]), ri = SINGLE ? ri_single : uniform(RI[slot]);
    double pr[KPL], pn[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) pr[c] = P[slot].v[c] * q[c];
    stamp(0);
    double dot;
    if constexpr (FULL) dot = seq_fold_dpp<double, KPL>(pr);
    else dot = seq_fold<double, KPL>(pr, k, lds, lane);
    const double e = r - dot;  // :405
    stamp(1);
#pragma unroll
    for (int c = 0; c < KPL; ++c) update_pair<AR>(P[slot].v[c], q[c], e, eta, ru, ri, pn[c], q[c]);
    // 3. entry j-2's stores have landed (NW younger operations may still fly): publish its ticket
    wait_vmcnt<NW>();
    publish(trs, pend0, pv0);
    pend0 = pend1;
    pv0 = pv1;
    pend1 = u * 4u;
    pv1 = useq + 1;
    // 4. entry j's stores
    strow<KPL>(urs, voff, u * rowb, pn);
    if (!SINGLE) strow<KPL>(irs, voff, deferq ? kOOB : i * rowb, q);
    stamp(2);
    // 5. prefetch entry j+2 into this slot (after the stores: a reload of an item row this wave
    //    just stored sees it); its user row only if its ticket (polled at entry j-2) was ready
    const bool live2 = j + 2 < cnt;
    const int32_t okN = !live2 || __builtin_amdgcn_readfirstlane(tk[slot]) == static_cast<int32_t>(q2 & kDetUseqMask);
    P[slot] = ldrow<KPL>(urs, voff, live2 && okN ? u2 * rowb : kOOB);
    RU[slot] = ld_reg(rus, live2 ? u2 : 0u);
    if (!SINGLE) {
      Q[slot] = ldrow<KPL>(irs, voff, live2 && !(i2 == fi(s + 1)) ? i2 * rowb : kOOB);
      RI[slot] = ld_reg(ris, live2 ? i2 : 0u);
    }
    okP[slot] = okN;
    // 6. poll entry j+4's ticket (read at entry j+2)
    tk[slot] = poll_issue(trs, j + 4 < cnt ? u4 * 4u : kOOB);
    prev_i = i;
    stamp(3);
  };
  // Full chunks run their CH entries with no exit test in between: a per-entry "j >= cnt" exit
  // makes every entry's start a join with the path that skipped the previous entry, and the
  // compiler's wait counts then treat the rows loaded two entries back as just issued (vmcnt(3):
  // every entry waited for the previous entry's loads, a full memory round trip per update).
  // Only the last, partial chunk tests every entry.
  for (int32_t c0 = 0;; c0 += CH) {
    if (c0 + CH <= cnt) {
#pragma unroll
      for (int s = 0; s < CH; ++s) entry(s, c0 + s);
    } else {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        if (c0 + s >= cnt) goto done;
        entry(s, c0 + s);
      }
    }
    C0 = C1;
    C1 = chunk(c0 / CH + 2);
  }
done:
  if (SINGLE) strow<KPL>(irs, voff, item0 * rowb, q);  // the item row, once
  __builtin_amdgcn_s_waitcnt(0x0F70);
  publish(trs, pend0, pv0);
  publish(trs, pend1, pv1);
#if defined(MFHIP_EXPERIMENTS) && defined(MFHIP_DET_PROBE)
  if (blockIdx.x == 0 && lane == 0)
    printf("[det probe] wave 0: %lld entries, cycles per entry: pre-fold %.0f fold %.0f post-fold %.0f prefetch %.0f\n",
           (long long)cnt, double(pc[0]) / cnt, double(pc[1]) / cnt, double(pc[2]) / cnt, double(pc[3]) / cnt);
#endif
}

// ---------------------------------------------------------------------------------------------
// Split single-item chains (k == 64 KPL).  A single wave issues at most one instruction every
// ~4 shader cycles whatever its kind (profiles/r05_fold_fill_microbench.txt: one VALU, readlane,
// permlane or mov between two fold steps adds 4.0 cycles), so an update costs ~4 cycles per
// instruction of the wave that runs it: the 128-step fold (512 cycles at k = 128) plus ~170 more
// instructions of loads, ticket logic, the user-row update and stores -- ~1250 cycles, 521 ns per
// update of the hottest item's chain, which bounds the superstep.  The chain itself needs only the
// fold, e, the item-row update and the next products.  So a single-item wave is a pair of waves
// of one workgroup:
//   * the CHAIN wave (det_chain) runs the item recurrence -- products, fold, e = r - dot, the item
//     row update (DSGDforMF.scala:405, :409-410) -- and nothing else: its operands arrive in LDS;
//   * the HELPER wave (det_helper) does everything around it: entry fields, ticket polls, user-row
//     loads (issued kLinkLA entries ahead), the LDS hand-over, the user-row update (:407-408) with
//     the e the chain wave publishes in LDS, the stores, the tickets, and the item row at the end.
//     It repeats the item-row update itself (the same operations on the same bits, so its copy of
//     q is bitwise the chain wave's) rather than receiving q through LDS.
// LDS link, slot j % kLinkR per entry j (every array per lane, so no access conflicts):
//   helper -> chain: p (the user row), r, ru, then tag = j (the slot is filled);
//   chain -> helper: e (the error), then done = j + 1 (entries finished).
// LDS operations of one wave execute in order, so a reader that sees tag / done also sees the
// data written before it; volatile accesses keep the compiler from reordering them.
// Slot reuse: the helper refills slot j % R with entry j + R only after done > j (the chain has
// read everything of entry j), and the chain overwrites e of slot j % R at entry j + R, which needs
// entry j + R's tag, written after the helper read e_j.  No deadlock: the helper blocks on a ticket
// only for the entry it is about to finish (every earlier entry published first), as det_wave does.
constexpr int kLinkR = 4;   // LDS slots
constexpr int kLinkLA = 6;  // helper: user rows loaded this many entries before their LDS hand-over
constexpr int kLinkD = kLinkR + kLinkLA;  // load distance (entries)
constexpr int kLinkRing = 8;              // register slots of loaded rows (>= kLinkLA, divides kDetChunk)
static_assert(kDetChunk % kLinkRing == 0 && kLinkRing >= kLinkLA && kDetChunk % kLinkR == 0, "link ring sizes");
static_assert(kLinkD + 2 < 2 * kDetChunk, "fields of entry j + D + 2 must be in the two chunks");

// Per lane: its KPL row elements contiguous (ds_read/write_b128 at KPL >= 2), {r, ru} as one 16-B
// word; e, tag and done one word each.
template <int KPL>
struct DetLink {
  double p[kLinkR][64][KPL];
  double rr[kLinkR][64][2];  // {r, ru}
  double e[kLinkR][64];
  int32_t tag[kLinkR][64];
  int32_t done[64];
};
typedef double dbl2 __attribute__((ext_vector_type(2)));
// volatile LDS pointers (address space 3: ds_read / ds_write; through a generic pointer a volatile
// access becomes a flat access that waits for vmcnt and lgkmcnt both)
#define MFHIP_LDS(T) __attribute__((address_space(3))) volatile T
template <typename T>
__device__ __forceinline__ MFHIP_LDS(T) * lds(T* p) {
  return (MFHIP_LDS(T)*)p;
}
template <int KPL>
__device__ __forceinline__ void link_put_row(MFHIP_LDS(double) * at, const double (&v)[KPL]) {
  if constexpr (KPL == 1) {
    at[0] = v[0];
  } else {
#pragma unroll
    for (int c = 0; c < KPL; c += 2) ((MFHIP_LDS(dbl2)*)at)[c / 2] = dbl2{v[c], v[c + 1]};
  }
}
template <int KPL>
__device__ __forceinline__ void link_get_row(MFHIP_LDS(double) * at, double (&v)[KPL]) {
  if constexpr (KPL == 1) {
    v[0] = at[0];
  } else {
#pragma unroll
    for (int c = 0; c < KPL; c += 2) {
      const dbl2 x = ((MFHIP_LDS(dbl2)*)at)[c / 2];
      v[c] = x.x;
      v[c + 1] = x.y;
    }
  }
}

// The chain wave waits here whenever its helper is blocked on a user ticket, legitimately, for up
// to the ticket wait's own bound (poll_until: ~2^20 polls, 1-2 s).  So this bound is a clock, and
// longer (~4 s on the 100 MHz s_memrealtime): a helper that times out sets err itself, and the
// chain must not be the one to fail the launch first (its message would name the wrong wait).
// The clock is read only once the first check has failed: an s_memrealtime in flight is a
// scalar-memory operation, and those return out of order, so every LDS wait behind it waits with
// lgkmcnt(0) for the clock too -- read at every call, it cost the helper's per-entry hand-over
// ~45 ns (tools/det_chain_bench.py: 416 vs 370 ns per chained update, gpurun_out/r6y).
template <typename F>
__device__ __forceinline__ void link_wait(F v, int32_t want, int32_t* err, int lane) {
  if (__builtin_amdgcn_readfirstlane(v()) >= want) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_readfirstlane(v()) < want) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // the flag store is not a row store a ticket publishes
      break;
    }
  }
}

template <int KPL, int AR>
__device__ __forceinline__ void det_chain(const DetWave d, const uint32_t* __restrict__ ei, const double* I,
                                          uint64_t i_bytes, const double* __restrict__ regI, double eta,
                                          DetLink<KPL>& L, int32_t* err, int lane) {
  const int32_t cnt = d.count;
  const __amdgpu_buffer_rsrc_t irs = raw_rsrc(I, i_bytes);
  const __amdgpu_buffer_rsrc_t ris = raw_rsrc(regI, reg_bytes<AR>());
  uint32_t voff[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) voff[c] = static_cast<uint32_t>(lane + 64 * c) * 8u;
  const uint32_t item = __builtin_amdgcn_readfirstlane(ei[d.begin]);
  const DRow<KPL> Q0 = ldrow<KPL>(irs, voff, item * (64u * KPL * 8u));
  const double ri = uniform(ld_reg(ris, item));
  double q[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = Q0.v[c];
  MFHIP_LDS(int32_t)* tag = lds(&L.tag[0][0]);
  MFHIP_LDS(double)* lp = lds(&L.p[0][0][0]);
  MFHIP_LDS(double)* lrr = lds(&L.rr[0][0][0]);
  MFHIP_LDS(double)* le = lds(&L.e[0][0]);
  MFHIP_LDS(int32_t)* ldone = lds(&L.done[0]);
  double P[2][KPL], R[2];
  auto get = [&](int s, int sl) {  // slot sl's row and r into register slot s
    link_get_row<KPL>(lp + (sl * 64 + lane) * KPL, P[s]);
    R[s] = lrr[(sl * 64 + lane) * 2];
  };
  // entry m's operands from its slot (after its tag)
  auto fetch = [&](int s, int32_t m) {
    const int sl = m % kLinkR;
    link_wait([&] { return tag[sl * 64 + lane]; }, m, err, lane);
    __builtin_amdgcn_sched_barrier(0);
    get(s, sl);
  };
  // per register slot: an entry whose operands have to be read again when it starts (-1: none;
  // its slot was not filled yet when entry j - 2 ended -- rare).  Only the entry about to run may
  // block: the helper hands entry j over at the latest when it has finished entry j - 1.  A slot is
  // read right after its tag, unconditionally (the reads execute after the tag read, in order, so
  // they see the row whenever the tag did; stale data is read again).
  int32_t want[2] = {-1, -1};
  fetch(0, 0);
  {
    const int32_t t1 = tag[1 * 64 + lane];
    get(1, 1);
    if (cnt > 1 && __builtin_amdgcn_readfirstlane(t1) < 1) want[1] = 1;
  }
  auto entry = [&](const int s, const int32_t j) {
    if (want[s] == j) fetch(s, j);
    double pr[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) pr[c] = P[s][c] * q[c];
    const int sl2 = (j + 2) % kLinkR;
    const int32_t t2 = tag[sl2 * 64 + lane];  // read before the fold, tested after it
    const double dot = seq_fold_dpp<double, KPL>(pr);
    const double e = R[s] - dot;  // :405
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      if constexpr (AR == kArDsgd) q[c] = q[c] - eta * (ri * q[c] - e * P[s][c]);  // :409-410
      else q[c] = q[c] + (eta * e) * P[s][c];  // nextFactors (update_pair's le * p)
    }
    le[(j % kLinkR) * 64 + lane] = e;
    ldone[lane] = j + 1;
    // entry j + 2's operands into this register slot
    get(s, sl2);
    want[s] = (j + 2 < cnt && __builtin_amdgcn_readfirstlane(t2) < j + 2) ? j + 2 : -1;
  };
  for (int32_t c0 = 0;; c0 += 4) {
    if (c0 + 4 <= cnt) {
      entry(0, c0);
      entry(1, c0 + 1);
      entry(0, c0 + 2);
      entry(1, c0 + 3);
    } else {
      if (c0 < cnt) entry(0, c0);
      if (c0 + 1 < cnt) entry(1, c0 + 1);
      if (c0 + 2 < cnt) entry(0, c0 + 2);
      break;
    }
  }
}

template <int KPL, int AR>
__device__ __forceinline__ void det_helper(const DetWave d, const uint32_t* __restrict__ eu, const uint32_t* __restrict__ ei,
                                           const uint32_t* __restrict__ eq, const double* __restrict__ er, double* U,
                                           double* I, uint64_t u_bytes, uint64_t i_bytes,
                                           const double* __restrict__ regU, const double* __restrict__ regI,
                                           double eta, int32_t* ticket, DetLink<KPL>& L, int32_t* err, int lane) {
  constexpr int CH = kDetChunk, R = kLinkR, D = kLinkD, RING = kLinkRing;
  // vector-memory operations per entry, in issue order (the wait before a ticket is published
  // counts on them -- change the entry, change NW):
  //   publish 1 | user store KPL | user load KPL, ru 1 | poll 1
  // NW = the operations issued after entry j-2's stores up to entry j's publish: entry j-2's loads
  // and poll, all of entry j-1's: (KPL + 2) + (2 KPL + 3).
  constexpr int NW = 3 * KPL + 5;
  static_assert(NW < 64, "vmcnt range");
  const int32_t cnt = d.count;
  const __amdgpu_buffer_rsrc_t urs = raw_rsrc(U, u_bytes), irs = raw_rsrc(I, i_bytes);
  const __amdgpu_buffer_rsrc_t trs = raw_rsrc(ticket, 0xFFFFF000ull);
  const __amdgpu_buffer_rsrc_t rus = raw_rsrc(regU, reg_bytes<AR>()), ris = raw_rsrc(regI, reg_bytes<AR>());
  uint32_t voff[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) voff[c] = static_cast<uint32_t>(lane + 64 * c) * 8u;
  constexpr uint32_t rowb = 64u * KPL * 8u;
  auto chunk = [&](int64_t c) { return det_chunk(eu, ei, eq, er, d.begin + c * CH + (lane & (CH - 1))); };
  DetChunk C0 = chunk(0), C1 = chunk(1);
  auto fu = [&](int s) { return s < CH ? rl(C0.u, s) : rl(C1.u, s - CH); };
  auto fq = [&](int s) { return s < CH ? rl(C0.q, s) : rl(C1.q, s - CH); };
  auto fr = [&](int s) { return rld(s < CH ? C0.r : C1.r, s < CH ? s : s - CH); };
  const uint32_t item = rl(C0.i, 0);
  const DRow<KPL> Q0 = ldrow<KPL>(irs, voff, item * rowb);
  const double ri = uniform(ld_reg(ris, item));
  double q[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = Q0.v[c];
  MFHIP_LDS(int32_t)* tag = lds(&L.tag[0][0]);
  MFHIP_LDS(double)* lp = lds(&L.p[0][0][0]);
  MFHIP_LDS(double)* lrr = lds(&L.rr[0][0][0]);
  MFHIP_LDS(double)* le = lds(&L.e[0][0]);
  MFHIP_LDS(int32_t)* ldone = lds(&L.done[0]);
  auto put = [&](int32_t m, const double (&p)[KPL], double r, double ru) {  // entry m into its slot
    const int sl = m % R;
    link_put_row<KPL>(lp + (sl * 64 + lane) * KPL, p);
    ((MFHIP_LDS(dbl2)*)lrr)[sl * 64 + lane] = dbl2{r, ru};
    tag[sl * 64 + lane] = m;  // last: the slot is filled
  };
  double PR[RING][KPL], RU[RING];  // loaded user rows of entries j + R .. j + D - 1 (slot m % RING)
  uint32_t okR = 0;                // bit m % RING: entry m's row was loaded (its ticket was ready)
  uint32_t later = 0;              // bit m % R: entry m is not in its slot yet (handed over when it runs)
  int32_t tk[2];                   // polls of entries j + D and j + D + 1
  // prologue (entries 0 .. D-1): rows of entries with a ready ticket; 0 .. R-1 go to their slots
  for (int x = 0; x < D; ++x) {
    const bool live = x < cnt;
    const uint32_t u = fu(x);
    const bool ok = live && poll(trs, u * 4u) == static_cast<int32_t>(fq(x) & kDetUseqMask);
    const DRow<KPL> p = ldrow<KPL>(urs, voff, ok ? u * rowb : kOOB);
    const double ru = ld_reg(rus, live ? u : 0u);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if (x < R) {
      if (ok) put(x, p.v, fr(x), ru);
      else if (live) later |= 1u << (x % R);
    } else {
#pragma unroll
      for (int c = 0; c < KPL; ++c) PR[x % RING][c] = p.v[c];
      RU[x % RING] = ru;
      if (ok) okR |= 1u << (x % RING);
    }
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) tk[x] = poll_issue(trs, D + x < cnt ? fu(D + x) * 4u : kOOB);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  uint32_t pend0 = kOOB, pend1 = kOOB;  // entries j-2 / j-1: ticket word byte offsets (kOOB: none)
  int32_t pv0 = 0, pv1 = 0;
  auto entry = [&](const int s, const int32_t j) {
    const uint32_t u = fu(s), qf = fq(s);
    const int32_t useq = static_cast<int32_t>(qf & kDetUseqMask);
    // a. entry j's row when its ticket was not ready in time: publish every pending ticket
    //    (after its stores), wait for ours, hand the row over now
    if (later & (1u << (j % R))) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      publish(trs, pend0, pv0);
      publish(trs, pend1, pv1);
      pend0 = pend1 = kOOB;
      wait_ticket_or_fail(ticket + u, useq, err, lane);
      const DRow<KPL> p = ldrow<KPL>(urs, voff, u * rowb);
      const double ru = ld_reg(rus, u);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      put(j, p.v, fr(s), ru);
      later &= ~(1u << (j % R));
    }
    // b. the chain wave's e of entry j
    link_wait([&] { return ldone[lane]; }, j + 1, err, lane);
    __builtin_amdgcn_sched_barrier(0);
    const int sl = j % R;
    const double e = le[sl * 64 + lane];
    const double ru = lrr[(sl * 64 + lane) * 2 + 1];
    double p[KPL], pn[KPL];
    link_get_row<KPL>(lp + (sl * 64 + lane) * KPL, p);
    // c. the user row (:407-408) and this wave's copy of the item row (:409-410, old p)
#pragma unroll
    for (int c = 0; c < KPL; ++c) update_pair<AR>(p[c], q[c], e, eta, ru, ri, pn[c], q[c]);
    // d. entry j-2's stores have landed: publish its ticket; entry j's stores
    wait_vmcnt<NW>();
    publish(trs, pend0, pv0);
    pend0 = pend1;
    pv0 = pv1;
    pend1 = u * 4u;
    pv1 = useq + 1;
    strow<KPL>(urs, voff, u * rowb, pn);
    // e. entry j + R into slot j % R (the chain wave is done with entry j)
    const int32_t m = j + R;
    if (m < cnt) {
      if (okR & (1u << (m % RING))) put(m, PR[m % RING], fr(s + R), RU[m % RING]);
      else later |= 1u << (m % R);
    }
    // f. load entry j + D's row if its ticket (polled two entries ago) is ready
    const int32_t m2 = j + D;
    const bool ok2 = m2 < cnt && __builtin_amdgcn_readfirstlane(tk[j & 1]) == static_cast<int32_t>(fq(s + D) & kDetUseqMask);
    const uint32_t u2 = fu(s + D);
    const DRow<KPL> p2 = ldrow<KPL>(urs, voff, ok2 ? u2 * rowb : kOOB);
#pragma unroll
    for (int c = 0; c < KPL; ++c) PR[m2 % RING][c] = p2.v[c];
    RU[m2 % RING] = ld_reg(rus, m2 < cnt ? u2 : 0u);
    okR = ok2 ? (okR | (1u << (m2 % RING))) : (okR & ~(1u << (m2 % RING)));
    // g. poll entry j + D + 2's ticket
    tk[j & 1] = poll_issue(trs, m2 + 2 < cnt ? fu(s + D + 2) * 4u : kOOB);
  };
  for (int32_t c0 = 0;; c0 += CH) {
    if (c0 + CH <= cnt) {
#pragma unroll
      for (int s = 0; s < CH; ++s) entry(s, c0 + s);
    } else {
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        if (c0 + s >= cnt) goto done;
        entry(s, c0 + s);
      }
    }
    C0 = C1;
    C1 = chunk(c0 / CH + 2);
  }
done:
  // the loads of the last entries' look-ahead (rows, lambda/omega, polls past the wave's end) are
  // used here, so the compiler keeps every one of them on the path through the last chunk: the
  // wait before each publish counts them
#pragma unroll
  for (int x = 0; x < RING; ++x) {
#pragma unroll
    for (int c = 0; c < KPL; ++c) asm volatile("" ::"v"(PR[x][c]));
    asm volatile("" ::"v"(RU[x]));
  }
  asm volatile("" ::"v"(tk[0]), "v"(tk[1]));
  strow<KPL>(irs, voff, item * rowb, q);  // the item row, once
  __builtin_amdgcn_s_waitcnt(0x0F70);
  publish(trs, pend0, pv0);
  publish(trs, pend1, pv1);
}

// Blocks of two wave slots: slots[2b + w] is wave w's descriptor.  A single-item wave's slot 1 is
// its helper (kDetWaveHelper: the same entries); any other slot runs det_wave (count 0: nothing).
template <int KPL, int AR = kArDsgd>
__global__ __launch_bounds__(128) void k_det_sweep_split(const DetWave* __restrict__ slots, const uint32_t* __restrict__ eu,
                                                         const uint32_t* __restrict__ ei, const uint32_t* __restrict__ eq,
                                                         const double* __restrict__ er, double* U, double* I,
                                                         uint64_t u_bytes, uint64_t i_bytes,
                                                         const double* __restrict__ regU,
                                                         const double* __restrict__ regI, double eta, int32_t* ticket,
                                                         int32_t* err) {
  __shared__ __attribute__((aligned(16))) DetLink<KPL> link;
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = static_cast<int>(threadIdx.x) & 63;
  const DetWave d0 = slots[2 * blockIdx.x];
  const DetWave d = slots[2 * blockIdx.x + w];
  if ((d0.flags & kDetWaveSingleItem) && d0.count > 0) {  // a chain / helper pair (both waves)
    if (w == 1) {
#pragma unroll
      for (int sl = 0; sl < kLinkR; ++sl) link.tag[sl][lane] = -1;
      link.done[lane] = 0;
    }
    __syncthreads();
    if (w == 0) det_chain<KPL, AR>(d0, ei, I, i_bytes, regI, eta, link, err, lane);
    else det_helper<KPL, AR>(d0, eu, ei, eq, er, U, I, u_bytes, i_bytes, regU, regI, eta, ticket, link, err, lane);
    return;
  }
  if (d.count == 0) return;
  det_wave<KPL, true, false, AR>(d, eu, ei, eq, er, U, I, u_bytes, i_bytes, regU, regI, 64 * KPL, eta, ticket, nullptr,
                                 err, nullptr, lane);
}

template <int KPL, bool FULL>
__global__ __launch_bounds__(64) void k_det_sweep2(const DetWave* __restrict__ waves, const uint32_t* __restrict__ eu,
                                                   const uint32_t* __restrict__ ei, const uint32_t* __restrict__ eq,
                                                   const double* __restrict__ er, double* U, double* I,
                                                   uint64_t u_bytes, uint64_t i_bytes, const double* __restrict__ regU,
                                                   const double* __restrict__ regI, int k, double eta,
                                                   int32_t* ticket, int32_t* dummy_ticket, int32_t* err) {
  __shared__ __attribute__((aligned(16))) double lds[64 * KPL];
  (void)dummy_ticket;  // "no ticket" is the out-of-range offset kOOB now
  const DetWave d = waves[blockIdx.x];
  if (d.count == 0) return;
  if (d.flags & kDetWaveSingleItem)
    det_wave<KPL, FULL, true>(d, eu, ei, eq, er, U, I, u_bytes, i_bytes, regU, regI, k, eta, ticket, dummy_ticket, err, lds,
                              static_cast<int>(threadIdx.x));
  else
    det_wave<KPL, FULL, false>(d, eu, ei, eq, er, U, I, u_bytes, i_bytes, regU, regI, k, eta, ticket, dummy_ticket, err,
                               lds, static_cast<int>(threadIdx.x));
}

template <int KPL>
int det_capacity(bool full) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  const hipError_t st = full ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_det_sweep2<KPL, true>, 64, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_det_sweep2<KPL, false>, 64, 0);
  return st == hipSuccess ? cus * per_cu : 0;
}

template <int KPL, int AR = kArDsgd>
int det_split_cap() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_det_sweep_split<KPL, AR>, 128, 0) != hipSuccess) return 0;
  return 2 * cus * per_cu;
}

}  // namespace

int det_split_capacity(int k) {
  if (k == 64) return det_split_cap<1>();
  if (k == 128) return det_split_cap<2>();
  if (k == 256) return det_split_cap<4>();
  return 0;
}

void launch_det_sweep_split(hipStream_t st, const DetWave* slots, int nslots, const uint32_t* eu, const uint32_t* ei,
                            const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes,
                            uint64_t i_bytes, const double* regU, const double* regI, int k, double eta,
                            int32_t* ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
  if (nslots <= 0) return;
  const dim3 g(static_cast<unsigned>(nslots / 2)), b(128);
#define MF_DETS(KPL)                                                                                           \
  hipExtLaunchKernelGGL((k_det_sweep_split<KPL>), g, b, 0, st, ev0, ev1, 0, slots, eu, ei, eq, er, U, I, u_bytes, \
                        i_bytes, regU, regI, eta, ticket, err)
  if (k == 64) MF_DETS(1);
  else if (k == 128) MF_DETS(2);
  else if (k == 256) MF_DETS(4);
#undef MF_DETS
}

// The online f64 micro-batch (SGDUpdater.nextFactors in sequence order, core/FactorUpdater.scala:37-45)
// on the deterministic sweep: the same per-item waves, per-user tickets and hand-off, kArNext's
// update rule.  Slots as launch_det_sweep_split's; k = 64, 128, 256 only (0: not supported).
int online_det_capacity(int k) {
  if (k == 64) return det_split_cap<1, kArNext>();
  if (k == 128) return det_split_cap<2, kArNext>();
  if (k == 256) return det_split_cap<4, kArNext>();
  return 0;
}

void launch_online_det(hipStream_t st, const DetWave* slots, int nslots, const uint32_t* eu, const uint32_t* ei,
                       const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes, uint64_t i_bytes,
                       int k, double eta, int32_t* ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
  if (nslots <= 0) return;
  const dim3 g(static_cast<unsigned>(nslots / 2)), b(128);
  const double* none = nullptr;  // kArNext: no lambda / omega (empty buffer ranges)
#define MF_ONDET(KPL)                                                                                                 \
  hipExtLaunchKernelGGL((k_det_sweep_split<KPL, kArNext>), g, b, 0, st, ev0, ev1, 0, slots, eu, ei, eq, er, U, I,     \
                        u_bytes, i_bytes, none, none, eta, ticket, err)
  if (k == 64) MF_ONDET(1);
  else if (k == 128) MF_ONDET(2);
  else if (k == 256) MF_ONDET(4);
#undef MF_ONDET
}

// the co-resident wave count of the instance launch_det_sweep picks for k
int det_sweep_capacity(int k) {
  if (k <= 64) return det_capacity<1>(k == 64);
  if (k <= 128) return det_capacity<2>(k == 128);
  if (k <= 256) return det_capacity<4>(k == 256);
  return det_capacity<8>(k == 512);
}

void launch_det_sweep(hipStream_t st, const DetWave* waves, int nw, const uint32_t* eu, const uint32_t* ei,
                      const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes, uint64_t i_bytes,
                      const double* regU, const double* regI, int k, double eta, int32_t* ticket,
                      int32_t* dummy_ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1) {
  if (nw <= 0) return;
  const dim3 g(static_cast<unsigned>(nw)), b(64);
#define MF_DET(KPL)                                                                                                  \
  do {                                                                                                               \
    if (k == 64 * (KPL))                                                                                             \
      hipExtLaunchKernelGGL((k_det_sweep2<KPL, true>), g, b, 0, st, ev0, ev1, 0, waves, eu, ei, eq, er, U, I, u_bytes, \
                            i_bytes, regU, regI, k, eta, ticket, dummy_ticket, err);                                 \
    else                                                                                                             \
      hipExtLaunchKernelGGL((k_det_sweep2<KPL, false>), g, b, 0, st, ev0, ev1, 0, waves, eu, ei, eq, er, U, I,       \
                            u_bytes, i_bytes, regU, regI, k, eta, ticket, dummy_ticket, err);                        \
  } while (0)
  if (k <= 64) MF_DET(1);
  else if (k <= 128) MF_DET(2);
  else if (k <= 256) MF_DET(4);
  else MF_DET(8);
#undef MF_DET
}

}  // namespace mfhip
