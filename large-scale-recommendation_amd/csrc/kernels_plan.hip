// kernels_plan.hip -- the fast pair schedule's per-cell work on the device: the greedy emission of
// every cell (plan.cpp build_fast_plan, phase 2) and the pair records of every wave
// (build_pair_plan), one thread per cell / wave.  The host keeps phase 1 (LPT groups, cell-major
// order, spreading of repeated users) and the wave tables; the records never cross PCIe.  The
// result is bitwise the host plan (tests/test_gpu_dsgd.py: plan digests and factors compared).
//
// A cell's emission is a sequential greedy over its entries (continue the item run, or the user
// run, else the item with most pending ratings whose row and some pending user row are free,
// else a no-op record), so a cell is one thread's serial program; cells are independent (the
// window counts along a cell), so the launch is as wide as the cell count (~1M on NFLX).  Its
// scratch (groups, the per-cell user table, taken flags, hazard positions) lives in global
// memory at the cell's entry range.  Integer work, latency-bound: no MFMA, no LDS staging.
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <climits>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"
#include "plan.hpp"

namespace mfhip {
namespace {

constexpr int kPlanThreads = 64;
constexpr int32_t kNever = INT32_MIN / 2;  // hazard position of a row not emitted yet in the cell

struct EmitArgs {
  const PlanEnt* E;        // entries of all blocks, in cell order (cells indexed like fp.cell_off)
  const int64_t* cstart;   // ncells + 1
  const int32_t* cblk;     // cell -> block (index into the per-block tables)
  const uint32_t* bub;     // per block: first user row
  const int64_t* bregu;    // per block: offset into regu
  const int64_t* bvit;     // per block: offset into regi / vrow
  const float* regu;
  const float* regi;
  const uint32_t* vrow;
  int32_t* ug;             // scratch, per entry: user group / item group / user list / order
  int32_t* ig;
  int32_t* ulist;
  int32_t* iorder;
  uint8_t* taken;
  int32_t* igB;            // per group (at the cell's entry range): [beg, end), head, left, row
  int32_t* igE;
  int32_t* igH;
  int32_t* igL;
  uint32_t* igRow;
  int32_t* ugB;
  int32_t* ugE;
  int32_t* ugH;
  int32_t* ugL;
  int32_t* lastu;          // hazard position per user / item group
  int32_t* lasti;
  int32_t* hkey;           // per-cell open-addressing table local user -> user group (2 slots per entry)
  int32_t* hval;
  int64_t ncells;
  int32_t window;
  uint32_t row_bytes;
  uint32_t dummy;
  const int64_t* recbase;  // write pass: first record of each cell
  FastRec* recs;           // write pass output (null: count pass)
  int32_t* nrec;           // count pass: records per cell; write pass: unused
  int32_t* npads;          // count pass: no-op records per cell
  int32_t* npairs;         // write pass: pair steps per cell
  int32_t* err;            // set when a cell's emission ran past its bound
};

// The emission of one cell (plan.cpp build_fast_plan, phase 2, per-cell streams).  Returns the
// record count; writes the records when A.recs is set.
__device__ int64_t emit_cell(const EmitArgs& A, int64_t gc, int64_t& pads) {
  const int64_t c0 = A.cstart[gc];
  const int32_t m = static_cast<int32_t>(A.cstart[gc + 1] - c0);
  pads = 0;
  if (m == 0) return 0;
  const int32_t bx = A.cblk[gc];
  const uint32_t ub = A.bub[bx];
  const float* regu = A.regu + A.bregu[bx];
  const float* regi = A.regi + A.bvit[bx];
  const uint32_t* vrow = A.vrow + A.bvit[bx];
  const PlanEnt* E = A.E + c0;
  int32_t *ug = A.ug + c0, *ig = A.ig + c0, *ulist = A.ulist + c0, *iorder = A.iorder + c0;
  uint8_t* taken = A.taken + c0;
  int32_t *igB = A.igB + c0, *igE = A.igE + c0, *igH = A.igH + c0, *igL = A.igL + c0;
  uint32_t* igRow = A.igRow + c0;
  int32_t *ugB = A.ugB + c0, *ugE = A.ugE + c0, *ugH = A.ugH + c0, *ugL = A.ugL + c0;
  int32_t *lastu = A.lastu + c0, *lasti = A.lasti + c0;
  int32_t *hkey = A.hkey + 2 * c0, *hval = A.hval + 2 * c0;
  const uint32_t hcap = 2u * static_cast<uint32_t>(m);
  for (uint32_t h = 0; h < hcap; ++h) hkey[h] = -1;
  // groups: an item group is a run of equal items (contiguous), a user group is numbered by the
  // user's first appearance in the cell
  int32_t nig = 0, nug = 0;
  for (int32_t e = 0; e < m; ++e) {
    const PlanEnt pe = E[e];
    if (nig == 0 || igRow[nig - 1] != pe.vil) {
      igRow[nig] = pe.vil;
      igB[nig] = igH[nig] = e;
      ++nig;
    }
    uint32_t h = static_cast<uint32_t>((static_cast<uint64_t>(pe.ul) * 0x9E3779B1u) % hcap);
    while (hkey[h] != -1 && hkey[h] != static_cast<int32_t>(pe.ul)) h = h + 1 == hcap ? 0 : h + 1;
    int32_t g;
    if (hkey[h] == -1) {
      hkey[h] = static_cast<int32_t>(pe.ul);
      hval[h] = g = nug;
      ugE[nug] = 0;
      ++nug;
    } else {
      g = hval[h];
    }
    ug[e] = g;
    ig[e] = nig - 1;
    igE[nig - 1] = e + 1;
    ugE[g]++;  // count for now
  }
  {  // user groups: counts -> CSR ranges, entries in cell order
    int32_t acc = 0;
    for (int32_t g = 0; g < nug; ++g) {
      const int32_t n2 = ugE[g];
      ugB[g] = ugH[g] = acc;
      acc += n2;
      ugE[g] = acc;
      ugL[g] = ugB[g];  // fill cursor
    }
    for (int32_t e = 0; e < m; ++e) ulist[ugL[ug[e]]++] = e;
  }
  for (int32_t e = 0; e < m; ++e) taken[e] = 0;
  for (int32_t g = 0; g < nig; ++g) { igL[g] = igE[g] - igB[g]; lasti[g] = kNever; }
  for (int32_t g = 0; g < nug; ++g) { ugL[g] = ugE[g] - ugB[g]; lastu[g] = kNever; }
  // item groups by pending ratings, most first (stable)
  for (int32_t z = 0; z < nig; ++z) {
    const int32_t v = z, sv = igE[z] - igB[z];
    int32_t y = z - 1;
    while (y >= 0 && igE[iorder[y]] - igB[iorder[y]] < sv) { iorder[y + 1] = iorder[y]; --y; }
    iorder[y + 1] = v;
  }
  // (plan.hpp plan_window_pack) a single-item cell with a run window: no user within W records,
  // not even the next one
  const bool run_cell = plan_window_strict_runs(A.window) && nig == 1;
  const int32_t W = nig == 1 ? plan_window_run(A.window) : plan_window_mixed(A.window);
  FastRec* out = A.recs ? A.recs + A.recbase[gc] : nullptr;
  int32_t iorder_head = 0, prev_ug = -1, prev_ig = -1, left = m;
  int32_t pos = 0;
  uint32_t prev_irow = 0;
  const int32_t limit = 4 * W;
  // at most W no-op records in a row (after W of them every row is free again): a longer
  // emission is a bug -- stop and report it instead of spinning
  const int64_t max_pos = static_cast<int64_t>(m) * (W + 1) + 64;
  while (left > 0) {
    if (pos > max_pos) {
      pads = -1;
      return pos;
    }
    // the first untaken entries of an item group (at most 4 * window) whose user row is free
    // (or is the current user)
    auto scan_item = [&](int32_t g2, bool any_user) -> int32_t {
      int32_t& head = igH[g2];
      const int32_t end = igE[g2];
      while (head < end && taken[head]) ++head;
      int32_t seen = 0;
      for (int32_t y = head; y < end && seen < limit; ++y) {
        if (taken[y]) continue;
        ++seen;
        if ((!any_user && !run_cell && ug[y] == prev_ug) || pos - lastu[ug[y]] >= W) return y;
      }
      return -1;
    };
    auto try_item = [&]() -> int32_t {
      if (prev_ig < 0 || igL[prev_ig] == 0) return -1;
      return scan_item(prev_ig, false);
    };
    auto try_user = [&]() -> int32_t {
      if (run_cell || prev_ug < 0 || ugL[prev_ug] == 0) return -1;
      int32_t& head = ugH[prev_ug];
      const int32_t end = ugE[prev_ug];
      while (head < end && taken[ulist[head]]) ++head;
      int32_t seen = 0;
      for (int32_t y = head; y < end && seen < limit; ++y) {
        const int32_t e = ulist[y];
        if (taken[e]) continue;
        ++seen;
        if (ig[e] == prev_ig || pos - lasti[ig[e]] >= W) return e;
      }
      return -1;
    };
    const bool user_first = prev_ug >= 0 && prev_ig >= 0 && ugL[prev_ug] > igL[prev_ig];
    int32_t pick = user_first ? try_user() : try_item();
    if (pick < 0) pick = user_first ? try_item() : try_user();
    if (pick < 0) {  // fresh start: both rows free
      while (iorder_head < nig && igL[iorder[iorder_head]] == 0) ++iorder_head;
      int tried = 0;
      for (int32_t z = iorder_head; z < nig && tried < 64; ++z) {
        const int32_t g2 = iorder[z];
        if (igL[g2] == 0) continue;
        ++tried;
        if (pos - lasti[g2] < W) continue;
        pick = scan_item(g2, true);
        if (pick >= 0) break;
      }
    }
    if (pick < 0) {  // no-op record: zero user row, the current item (forwarded)
      if (out)
        out[pos] = FastRec{A.dummy * A.row_bytes, prev_irow * A.row_bytes, 0.f, 0.f, 0.f, A.dummy, prev_irow | kPadBit, 0};
      ++pads;
      if (prev_ig >= 0) lasti[prev_ig] = pos;
      prev_ug = -1;
      ++pos;
      continue;
    }
    taken[pick] = 1;
    --left;
    const int32_t pg = ug[pick], pi = ig[pick];
    igL[pi]--;
    ugL[pg]--;
    lastu[pg] = pos;
    lasti[pi] = pos;
    prev_ug = pg;
    prev_ig = pi;
    const PlanEnt pe = E[pick];
    const uint32_t urow = pe.ul + ub;
    prev_irow = vrow[pe.vil];
    if (out)
      out[pos] = FastRec{urow * A.row_bytes, prev_irow * A.row_bytes, pe.r, regu[pe.ul], regi[pe.vil], urow, prev_irow, 0};
    ++pos;
  }
  return pos;
}

__global__ __launch_bounds__(kPlanThreads) void k_emit_cells(EmitArgs A) {
  for (int64_t gc = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; gc < A.ncells;
       gc += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t pads = 0;
    const int64_t n = emit_cell(A, gc, pads);
    if (pads < 0) A.err[0] = 1;
    if (!A.recs) {
      A.nrec[gc] = static_cast<int32_t>(n);
      A.npads[gc] = static_cast<int32_t>(pads);
    } else {  // pair steps of the cell: two records with distinct users, or one
      const FastRec* f = A.recs + A.recbase[gc];
      int32_t np = 0;
      for (int64_t x = 0; x < n; ++np) x += (x + 1 < n && f[x + 1].u != f[x].u) ? 2 : 1;
      A.npairs[gc] = np;
    }
  }
}

struct PairArgs {
  const FastRec* recs;
  const int64_t* recbase;    // per cell
  const int32_t* nrec;       // per cell
  const int64_t* wave_cell;  // per wave
  const int64_t* wave_base;  // per wave: first pair record
  PairRec* out;
  int32_t* kind;             // per wave: kWaveGeneric / kWaveSingleRun / kWaveSingleRunFwd
  int32_t* noops;            // per wave: no-op halves
  double* bytes;             // per wave: requested bytes
  int64_t nwaves;
  double row_bytes;
  int32_t ring;  // the sweep's ring depth for this k (plan.hpp pair_ring)
};

// build_pair_plan's per-cell body (plan.cpp), one thread per wave.
__global__ __launch_bounds__(kPlanThreads) void k_pair_waves(PairArgs A) {
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w < A.nwaves;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t gc = A.wave_cell[w];
    const FastRec* f = A.recs + A.recbase[gc];
    const int64_t len = A.nrec[gc];
    PairRec* const first = A.out + A.wave_base[w];
    PairRec* out = first;
    auto item_of = [](const FastRec& r) { return r.i & ~kPadBit; };
    auto is_pad = [](const FastRec& r) { return (r.i & kPadBit) != 0; };
    int32_t noop = 0;
    uint32_t last_u = kOffOOB, last_half = 0;
    for (int64_t x = 0; x < len;) {
      const FastRec& a = f[x];
      const bool has_b = x + 1 < len && f[x + 1].u != a.u;
      const int64_t nx = x + (has_b ? 2 : 1);
      PairRec pr{};
      uint32_t flags = 0;
      const bool a_pad = is_pad(a);
      if (!a_pad && last_u == a.u_off) flags |= last_half;
      if (x > 0 && item_of(f[x - 1]) == item_of(a)) flags |= kPairKeepQ;
      pr.ua = (a_pad || (flags & (kPairFwdA | kPairFwdB))) ? kOffOOB : a.u_off;
      pr.ia = (flags & kPairKeepQ) ? kOffOOB : a.i_off;
      pr.sa = a_pad ? kOffOOB : a.u_off;
      pr.ra = a.r;
      pr.rua = a.ru;
      pr.ria = a.ri;
      if (a_pad) noop++;
      pr.ib = pr.ub = pr.sb = pr.sia = kOffOOB;
      const FastRec* tail = &a;
      if (has_b) {
        const FastRec& b = f[x + 1];
        tail = &b;
        if (item_of(b) != item_of(a)) {
          flags |= kPairSplit;
          pr.sia = a.i_off;
          pr.ib = b.i_off;
        }
        if (!is_pad(b)) {
          pr.ub = pr.sb = b.u_off;
          pr.rb = b.r;
          pr.rub = b.ru;
          pr.rib = b.ri;
        } else {
          noop++;
        }
      } else {
        noop++;
      }
      pr.si = (nx >= len || item_of(f[nx]) != item_of(*tail)) ? tail->i_off : kOffOOB;
      pr.flags = flags;
      *out++ = pr;
      if (has_b) {
        last_u = is_pad(f[x + 1]) ? kOffOOB : f[x + 1].u_off;
        last_half = kPairFwdB;
      } else {
        last_u = a_pad ? kOffOOB : a.u_off;
        last_half = kPairFwdA;
      }
      x = nx;
    }
    bool single = first[0].ia != kOffOOB && !(first[0].flags & (kPairKeepQ | kPairSplit));
    for (const PairRec* r = first; single && r < out; ++r)
      single = !(r->flags & kPairSplit) && (r == first || (r->flags & kPairKeepQ)) && r->ub == r->sb &&
               (r + 1 < out ? r->si == kOffOOB : r->si == first[0].ia);
    if (single) {  // the lean path's ring: a loaded user row was stored >= A.ring pairs back
      const int kR = A.ring - 1;
      uint32_t ring[kPairPlanRing][2];
      for (auto& rr : ring) rr[0] = rr[1] = kOffOOB;
      for (const PairRec* r = first; single && r < out; ++r) {
        const int64_t j = r - first;
        const uint32_t offs[2] = {r->ua, r->ub};
        for (uint32_t off : offs) {
          if (off == kOffOOB) continue;
          for (int y = 0; y < kR; ++y)
            if (ring[y][0] == off || ring[y][1] == off) single = false;
        }
        if (kR > 0) {
          ring[j % kR][0] = r->sa;
          ring[j % kR][1] = r->sb;
        }
      }
    }
    int64_t rows = 0;
    for (const PairRec* r = first; r < out; ++r) {
      if (single) {
        rows += (r->ua != kOffOOB) + 2 * (r->ub != kOffOOB) + (r->sa != kOffOOB);
      } else {
        const uint32_t offs[8] = {r->ua, r->ub, r->ia, r->ib, r->sa, r->sb, r->sia, r->si};
        for (uint32_t off : offs) rows += off != kOffOOB;
      }
    }
    if (single && out > first) rows += 2;
    bool fwd = false;  // A rows forwarded from the previous pair: the lean path's FWD instance
    for (const PairRec* r = first; single && r < out; ++r) fwd = fwd || (r->flags & (kPairFwdA | kPairFwdB));
    A.kind[w] = single ? (fwd ? kWaveSingleRunFwd : kWaveSingleRun) : kWaveGeneric;
    A.noops[w] = noop;
    A.bytes[w] = 64.0 * static_cast<double>(out - first) + A.row_bytes * static_cast<double>(rows);
  }
}

unsigned plan_grid(int64_t n) {
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + kPlanThreads - 1) / kPlanThreads, 1 << 20)));
}

template <class T>
T* upload(DevBuf& d, const T* h, size_t n, hipStream_t st) {
  d.alloc(std::max<size_t>(n, 1) * sizeof(T));
  if (n) MF_HIP(hipMemcpyAsync(d.get(), h, n * sizeof(T), hipMemcpyHostToDevice, st));
  return d.as<T>();
}

// ---------------------------------------------------------------------------------------------
// Phase 1 on the device (build_fast_plan's per-block work for the default plan: no hot-item
// replicas, K = 1, per-cell streams).  Ratings stay in the rating blocks' device order (x).

inline int bits_of(uint64_t maxval) {
  int b = 1;
  while (b < 64 && (maxval >> b) != 0) ++b;
  return b;
}

__device__ __forceinline__ uint32_t mix32d(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

// per rating: its block, local user / item, and the per-block user / item histograms
__global__ void k_p1_local(const uint32_t* __restrict__ urow, const uint32_t* __restrict__ irow, int64_t n,
                           const int64_t* __restrict__ bstart, int64_t nb2, int32_t nb, const int64_t* __restrict__ ubs,
                           const int64_t* __restrict__ ibs, const int64_t* __restrict__ uoff,
                           const int64_t* __restrict__ ioff, int32_t* __restrict__ blk, uint32_t* __restrict__ ul,
                           uint32_t* __restrict__ il, int32_t* __restrict__ ucnt, int32_t* __restrict__ icnt) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t lo = 0, hi = nb2;  // block b: bstart[b] <= x < bstart[b+1]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (bstart[mid] <= x) lo = mid;
      else hi = mid;
    }
    const int32_t b = static_cast<int32_t>(lo), p = b / nb, q = b % nb;
    const uint32_t u = urow[x] - static_cast<uint32_t>(ubs[p]), i = irow[x] - static_cast<uint32_t>(ibs[q]);
    blk[x] = b;
    ul[x] = u;
    il[x] = i;
    atomicAdd(ucnt + uoff[b] + u, 1);
    atomicAdd(icnt + ioff[b] + i, 1);
  }
}

// cell-major key (cell, item rank in the cell's item group), stable in x by the sort
__global__ void k_p1_cellkey(const int32_t* __restrict__ blk, const uint32_t* __restrict__ ul,
                             const uint32_t* __restrict__ il, int64_t n, const int32_t* __restrict__ Gb,
                             const int64_t* __restrict__ cbase, const int64_t* __restrict__ uoff,
                             const int64_t* __restrict__ ioff, const int32_t* __restrict__ gu,
                             const int32_t* __restrict__ gi, const int32_t* __restrict__ irank, uint64_t R,
                             uint64_t* __restrict__ key, int32_t* __restrict__ val, int32_t* __restrict__ ccount) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t b = blk[x], G = Gb[b];
    const int32_t g = gi[ioff[b] + il[x]], h = gu[uoff[b] + ul[x]];
    const int32_t d = h - g;
    const int64_t gc = cbase[b] + static_cast<int64_t>(d < 0 ? d + G : d) * G + g;
    key[x] = static_cast<uint64_t>(gc) * R + static_cast<uint64_t>(irank[ioff[b] + il[x]]);
    val[x] = static_cast<int32_t>(x);
    atomicAdd(ccount + gc, 1);
  }
}

__global__ void k_p1_heads64(const uint64_t* __restrict__ k, int64_t n, int32_t* __restrict__ head) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < n;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x)
    head[y] = (y == 0 || k[y] != k[y - 1]) ? 1 : 0;
}

// (run, local user) key of position y of the cell-major order
__global__ void k_p1_runuser(const int32_t* __restrict__ runid1, const int32_t* __restrict__ O1,
                             const uint32_t* __restrict__ ul, int64_t n, uint64_t NU, uint64_t* __restrict__ key,
                             int32_t* __restrict__ val) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < n;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    key[y] = static_cast<uint64_t>(runid1[y] - 1) * NU + ul[O1[y]];
    val[y] = static_cast<int32_t>(y);
  }
}

__global__ void k_p1_segstart(const int32_t* __restrict__ head, const int32_t* __restrict__ segid1, int64_t n,
                              int64_t* __restrict__ segstart) {
  for (int64_t z = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; z < n;
       z += static_cast<int64_t>(gridDim.x) * blockDim.x)
    if (head[z]) segstart[segid1[z] - 1] = z;
}

// spreading key of position y: the o-th of a user's m ratings in its item run goes to
// (o + h_u) / m (24 bits), ties by a second per-user hash (16 bits); x breaks the rest (stable)
__global__ void k_p1_pos(const int32_t* __restrict__ segid1, const int64_t* __restrict__ segstart,
                         const int32_t* __restrict__ P2, const int32_t* __restrict__ O1,
                         const uint32_t* __restrict__ urow, int64_t n, uint64_t order_seed,
                         uint64_t* __restrict__ pos, int32_t* __restrict__ val) {
  for (int64_t z = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; z < n;
       z += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t sg = segid1[z] - 1;
    const int64_t s0 = segstart[sg], m = segstart[sg + 1] - s0, o = z - s0;
    const int32_t y = P2[z];
    const uint32_t u = urow[O1[y]];
    const double h = static_cast<double>(mix32d(order_seed * 0x2545F4914F6CDD1DULL ^ u)) * (1.0 / 4294967296.0);
    const double frac = (static_cast<double>(o) + h) / static_cast<double>(m);
    const uint64_t tie = mix32d(order_seed ^ (static_cast<uint64_t>(u) << 20)) & 0xFFFFu;
    pos[y] = (static_cast<uint64_t>(frac * 16777216.0) << 16) | tie;
    val[y] = y;
  }
}

__global__ void k_p1_runkey(const int32_t* __restrict__ Q1, const int32_t* __restrict__ runid1, int64_t n,
                            uint32_t* __restrict__ key) {
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w < n;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x)
    key[w] = static_cast<uint32_t>(runid1[Q1[w]] - 1);
}

__global__ void k_p1_gather(const int32_t* __restrict__ F, const int32_t* __restrict__ O1,
                            const int32_t* __restrict__ blk, const int64_t* __restrict__ bstart,
                            const uint32_t* __restrict__ ul, const uint32_t* __restrict__ il,
                            const double* __restrict__ r, int64_t n, PlanEnt* __restrict__ E) {
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w < n;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t x = O1[F[w]];
    E[w] = PlanEnt{static_cast<uint32_t>(x - bstart[blk[x]]), ul[x], il[x], static_cast<float>(r[x])};
  }
}

struct SortTemp {
  DevBuf buf;
  void* get(size_t bytes) {
    buf.alloc(std::max<size_t>(bytes, 256));
    return buf.get();
  }
};

template <class K>
void sort_pairs(hipStream_t st, SortTemp& tmp, const K* kin, K* kout, const int32_t* vin, int32_t* vout, int64_t n,
                int bits) {
  size_t tb = 0;
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, static_cast<int>(n), 0, bits, st));
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, kin, kout, vin, vout, static_cast<int>(n), 0, bits, st));
}

void inclusive_sum(hipStream_t st, SortTemp& tmp, const int32_t* in, int32_t* out, int64_t n) {
  size_t tb = 0;
  MF_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out, static_cast<int>(n), st));
  MF_HIP(hipcub::DeviceScan::InclusiveSum(tmp.get(tb), tb, in, out, static_cast<int>(n), st));
}

// Per-block host metadata of the plan (blocks with ratings, ascending b) and the device inputs
// of the emission: the entries in cell order and the cell starts (cells indexed like
// fp.cell_off: GG cells + one empty slot per block).
struct PlanBlocks {
  std::vector<int64_t> b, GG, nu, nv, len;
  std::vector<uint32_t> ub;
  std::vector<int64_t> uoff, voff;  // nblk + 1: offsets into regu / regi, vrow
  std::vector<float> regu, regi;
  std::vector<uint32_t> vrow;
  int64_t total = 0;
};

void emit_and_pair(hipStream_t st, const PlanBlocks& pb, DevBuf& dE, DevBuf& dcs, FastPlan& fp, int32_t nb, int32_t c,
                   int32_t shard, int32_t k, uint32_t dummy_row, int32_t window, bool substep_waves, PairPlan& pp,
                   DevBuf& d_pairs) {
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  const int64_t nblk = static_cast<int64_t>(pb.b.size());
  std::vector<int64_t> coff(nblk + 1, 0);
  for (int64_t bx = 0; bx < nblk; ++bx) coff[bx + 1] = coff[bx] + pb.GG[bx] + 1;
  const int64_t total = pb.total, ncells = coff[nblk];
  std::vector<int32_t> cblk(ncells);
  fp.cell_base.assign(nb2, -1);
  fp.rec_base.assign(nb2, -1);
  for (int64_t bx = 0; bx < nblk; ++bx) {
    fp.cell_base[pb.b[bx]] = coff[bx];
    for (int64_t cc = 0; cc <= pb.GG[bx]; ++cc) cblk[coff[bx] + cc] = static_cast<int32_t>(bx);
  }
  DevBuf dcb, dbub, dbregu, dbvit, dregu, dregi, dvrow;
  EmitArgs A{};
  A.E = dE.as<PlanEnt>();
  A.cstart = dcs.as<int64_t>();
  A.cblk = upload(dcb, cblk.data(), cblk.size(), st);
  A.bub = upload(dbub, pb.ub.data(), pb.ub.size(), st);
  A.bregu = upload(dbregu, pb.uoff.data(), static_cast<size_t>(nblk), st);
  A.bvit = upload(dbvit, pb.voff.data(), static_cast<size_t>(nblk), st);
  A.regu = upload(dregu, pb.regu.data(), pb.regu.size(), st);
  A.regi = upload(dregi, pb.regi.data(), pb.regi.size(), st);
  A.vrow = upload(dvrow, pb.vrow.data(), pb.vrow.size(), st);
  const size_t ne = static_cast<size_t>(std::max<int64_t>(total, 1));
  DevBuf s_ug, s_ig, s_ul, s_io, s_tk, s_igB, s_igE, s_igH, s_igL, s_igR, s_ugB, s_ugE, s_ugH, s_ugL, s_lu, s_li, s_hk, s_hv;
  auto i32 = [&](DevBuf& d) { d.alloc(ne * 4); return d.as<int32_t>(); };
  A.ug = i32(s_ug); A.ig = i32(s_ig); A.ulist = i32(s_ul); A.iorder = i32(s_io);
  s_tk.alloc(ne); A.taken = s_tk.as<uint8_t>();
  A.igB = i32(s_igB); A.igE = i32(s_igE); A.igH = i32(s_igH); A.igL = i32(s_igL);
  s_igR.alloc(ne * 4); A.igRow = s_igR.as<uint32_t>();
  A.ugB = i32(s_ugB); A.ugE = i32(s_ugE); A.ugH = i32(s_ugH); A.ugL = i32(s_ugL);
  A.lastu = i32(s_lu); A.lasti = i32(s_li);
  s_hk.alloc(2 * ne * 4); A.hkey = s_hk.as<int32_t>();
  s_hv.alloc(2 * ne * 4); A.hval = s_hv.as<int32_t>();
  A.ncells = ncells;
  A.window = window;
  A.row_bytes = static_cast<uint32_t>(k) * 4u;
  A.dummy = dummy_row;
  DevBuf dnrec, dnpads, dnpairs, drecbase, drecs, derr;
  dnrec.alloc(static_cast<size_t>(std::max<int64_t>(ncells, 1)) * 4);
  dnpads.alloc(static_cast<size_t>(std::max<int64_t>(ncells, 1)) * 4);
  A.nrec = dnrec.as<int32_t>();
  A.npads = dnpads.as<int32_t>();
  derr.alloc(4);
  MF_HIP(hipMemsetAsync(derr.get(), 0, 4, st));
  A.err = derr.as<int32_t>();
  hipLaunchKernelGGL(k_emit_cells, dim3(plan_grid(ncells)), dim3(kPlanThreads), 0, st, A);
  MF_HIP(hipGetLastError());
  std::vector<int32_t> nrec(ncells), npads(ncells);
  MF_HIP(hipMemcpyAsync(nrec.data(), A.nrec, ncells * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipMemcpyAsync(npads.data(), A.npads, ncells * 4, hipMemcpyDeviceToHost, st));
  int32_t err = 0;
  MF_HIP(hipMemcpyAsync(&err, A.err, 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  MF_REQUIRE(err == 0, "device plan: a cell's emission ran past its bound");
  // records: per block contiguous, cells in order (the host plan's layout)
  std::vector<int64_t> recbase(ncells);
  fp.cell_off.assign(ncells, 0);
  fp.pads = 0;
  int64_t nrecs = 0;
  for (int64_t bx = 0; bx < nblk; ++bx) {
    fp.rec_base[pb.b[bx]] = nrecs;
    int64_t acc = 0;
    for (int64_t cc = 0; cc <= pb.GG[bx]; ++cc) {
      const int64_t gc = coff[bx] + cc;
      recbase[gc] = nrecs + acc;
      fp.cell_off[gc] = static_cast<int32_t>(acc);
      acc += nrec[gc];
      fp.pads += npads[gc];
    }
    nrecs += acc;
  }
  A.recbase = upload(drecbase, recbase.data(), recbase.size(), st);
  drecs.alloc(static_cast<size_t>(std::max<int64_t>(nrecs, 1)) * sizeof(FastRec));
  A.recs = drecs.as<FastRec>();
  dnpairs.alloc(static_cast<size_t>(std::max<int64_t>(ncells, 1)) * 4);
  A.npairs = dnpairs.as<int32_t>();
  hipLaunchKernelGGL(k_emit_cells, dim3(plan_grid(ncells)), dim3(kPlanThreads), 0, st, A);
  MF_HIP(hipGetLastError());
  std::vector<int32_t> cell_pairs(ncells);
  MF_HIP(hipMemcpyAsync(cell_pairs.data(), A.npairs, ncells * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  // the emission scratch is done
  for (DevBuf* d : {&s_ug, &s_ig, &s_ul, &s_io, &s_tk, &s_igB, &s_igE, &s_igH, &s_igL, &s_igR, &s_ugB, &s_ugE, &s_ugH,
                    &s_ugL, &s_lu, &s_li, &s_hk, &s_hv, &dE})
    d->release();
  // wave tables on the host, pair records on the device
  build_pair_plan(pp, fp, nb, c, shard, k, substep_waves, &cell_pairs);
  const int64_t nwaves = static_cast<int64_t>(pp.waves.size());
  std::vector<int64_t> wave_base(nwaves);
  int64_t npairs_total = 0;
  for (int64_t w = 0; w < nwaves; ++w) {
    wave_base[w] = pp.waves[w].base;
    npairs_total = std::max<int64_t>(npairs_total, pp.waves[w].base + pp.waves[w].steps);
  }
  DevBuf dwc, dwb, dkind, dnoop, dbytes;
  PairArgs P{};
  P.recs = A.recs;
  P.recbase = A.recbase;
  P.nrec = A.nrec;
  P.wave_cell = upload(dwc, pp.wave_cell.data(), pp.wave_cell.size(), st);
  P.wave_base = upload(dwb, wave_base.data(), wave_base.size(), st);
  d_pairs.alloc(static_cast<size_t>(std::max<int64_t>(npairs_total, 1)) * sizeof(PairRec));
  P.out = d_pairs.as<PairRec>();
  dkind.alloc(static_cast<size_t>(std::max<int64_t>(nwaves, 1)) * 4);
  dnoop.alloc(static_cast<size_t>(std::max<int64_t>(nwaves, 1)) * 4);
  dbytes.alloc(static_cast<size_t>(std::max<int64_t>(nwaves, 1)) * 8);
  P.kind = dkind.as<int32_t>();
  P.noops = dnoop.as<int32_t>();
  P.bytes = dbytes.as<double>();
  P.nwaves = nwaves;
  P.row_bytes = 4.0 * k;
  P.ring = pair_ring(pair_kpl(k));
  if (nwaves > 0) {
    hipLaunchKernelGGL(k_pair_waves, dim3(plan_grid(nwaves)), dim3(kPlanThreads), 0, st, P);
    MF_HIP(hipGetLastError());
  }
  std::vector<int32_t> kind(nwaves), noops(nwaves);
  std::vector<double> bytes(nwaves);
  if (nwaves > 0) {
    MF_HIP(hipMemcpyAsync(kind.data(), P.kind, nwaves * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(noops.data(), P.noops, nwaves * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(bytes.data(), P.bytes, nwaves * 8, hipMemcpyDeviceToHost, st));
  }
  MF_HIP(hipStreamSynchronize(st));
  // per-wave results into the tables, sums in the host path's order
  const int64_t nsub = static_cast<int64_t>(pp.sub_off.size()) - 1;
  std::vector<double> sub_bytes(nsub, 0.0);
  pp.noop_halves = 0;
  for (int64_t x = 0; x < nsub; ++x)
    for (int64_t w = pp.sub_off[x]; w < pp.sub_off[x + 1]; ++w) {
      pp.waves[w].cells = kind[w];
      if (pp.wave_sys[w] >= 0) pp.sys[pp.wave_sys[w]] = pp.waves[w];
      pp.noop_halves += noops[w];
      sub_bytes[x] += bytes[w];
    }
  pp.sm_bytes.assign(nb, 0.0);
  for (int64_t x = 0; x < nsub; ++x) pp.sm_bytes[substep_waves ? x / fp.G : x] += sub_bytes[x];
}

// per rating of the shard's blocks: the per-block item histogram (the group model's top counts)
__global__ void k_item_hist(const uint32_t* __restrict__ irow, int64_t n, const int64_t* __restrict__ bstart,
                            int64_t nb2, int32_t nb, const int64_t* __restrict__ ibs, const int64_t* __restrict__ ioff,
                            int32_t* __restrict__ icnt) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t lo = 0, hi = nb2;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (bstart[mid] <= x) lo = mid;
      else hi = mid;
    }
    const int32_t b = static_cast<int32_t>(lo);
    atomicAdd(icnt + ioff[b] + (irow[x] - static_cast<uint32_t>(ibs[b % nb])), 1);
  }
}

}  // namespace

std::vector<int64_t> device_block_tops(hipStream_t st, const DevRatingBlocks& dr, const RatingBlocks& rb,
                                       const SideLayout& I) {
  const int32_t nb = rb.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  std::vector<int64_t> ioff(nb2, 0), top(nb2, 0);
  int64_t isum = 0;
  for (int64_t b = 0; b < nb2; ++b) {
    ioff[b] = isum;
    if (rb.size(b) > 0) isum += I.block_start[b % nb + 1] - I.block_start[b % nb];
  }
  if (dr.total == 0 || isum == 0) return top;
  DevBuf dbs, dibs, dio, dcnt;
  upload(dbs, rb.start.data(), rb.start.size(), st);
  upload(dibs, I.block_start.data(), I.block_start.size(), st);
  upload(dio, ioff.data(), ioff.size(), st);
  dcnt.alloc(static_cast<size_t>(isum) * 4);
  MF_HIP(hipMemsetAsync(dcnt.get(), 0, dcnt.bytes(), st));
  hipLaunchKernelGGL(k_item_hist, dim3(plan_grid(dr.total)), dim3(256), 0, st, dr.irow.as<uint32_t>(), dr.total,
                     dbs.as<int64_t>(), nb2, nb, dibs.as<int64_t>(), dio.as<int64_t>(), dcnt.as<int32_t>());
  MF_HIP(hipGetLastError());
  std::vector<int32_t> cnt(isum);
  MF_HIP(hipMemcpyAsync(cnt.data(), dcnt.get(), isum * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  for (int64_t b = 0; b < nb2; ++b) {
    if (rb.size(b) == 0) continue;
    const int64_t ni = I.block_start[b % nb + 1] - I.block_start[b % nb];
    int32_t mx = 0;
    for (int64_t il = 0; il < ni; ++il) mx = std::max(mx, cnt[ioff[b] + il]);
    top[b] = mx;
  }
  return top;
}

void fetch_rating_blocks(hipStream_t st, const DevRatingBlocks& dr, RatingBlocks& rb) {
  resize_huge(rb.urow, dr.total);
  resize_huge(rb.irow, dr.total);
  resize_huge(rb.r, dr.total);
  if (dr.total > 0) {
    MF_HIP(hipMemcpyAsync(rb.urow.data(), dr.urow.get(), dr.total * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(rb.irow.data(), dr.irow.get(), dr.total * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(rb.r.data(), dr.r.get(), dr.total * 8, hipMemcpyDeviceToHost, st));
  }
  MF_HIP(hipStreamSynchronize(st));
}

void device_pair_schedule(hipStream_t st, std::vector<FastBlockWork>& work, FastPlan& fp, int32_t nb, int32_t c,
                          int32_t shard, int32_t k, uint32_t dummy_row, int32_t window, bool substep_waves,
                          PairPlan& pp, DevBuf& d_pairs) {
  const int64_t nblk = static_cast<int64_t>(work.size());
  PlanBlocks pb;
  pb.uoff.assign(nblk + 1, 0);
  pb.voff.assign(nblk + 1, 0);
  std::vector<int64_t> eoff(nblk + 1, 0);
  for (int64_t bx = 0; bx < nblk; ++bx) {
    const FastBlockWork& W = work[bx];
    pb.b.push_back(W.b);
    pb.GG.push_back(W.GG);
    pb.nu.push_back(W.nu);
    pb.nv.push_back(W.nv);
    pb.len.push_back(W.len);
    pb.ub.push_back(static_cast<uint32_t>(W.ub));
    pb.uoff[bx + 1] = pb.uoff[bx] + W.nu;
    pb.voff[bx + 1] = pb.voff[bx] + W.nv;
    eoff[bx + 1] = eoff[bx] + W.len;
    pb.regu.insert(pb.regu.end(), W.regu.begin(), W.regu.end());
    pb.regi.insert(pb.regi.end(), W.regi.begin(), W.regi.end());
    pb.vrow.insert(pb.vrow.end(), W.vrow.begin(), W.vrow.end());
  }
  pb.total = eoff[nblk];
  std::vector<int64_t> cstart;
  for (int64_t bx = 0; bx < nblk; ++bx)
    for (int64_t cc = 0; cc <= work[bx].GG; ++cc) cstart.push_back(eoff[bx] + work[bx].cstart[cc]);
  cstart.push_back(pb.total);
  DevBuf dE, dcs;
  dE.alloc(std::max<int64_t>(pb.total, 1) * sizeof(PlanEnt));
  for (int64_t bx = 0; bx < nblk; ++bx)
    if (work[bx].len)
      MF_HIP(hipMemcpyAsync(dE.as<PlanEnt>() + eoff[bx], work[bx].e.data(), work[bx].len * sizeof(PlanEnt),
                            hipMemcpyHostToDevice, st));
  upload(dcs, cstart.data(), cstart.size(), st);
  emit_and_pair(st, pb, dE, dcs, fp, nb, c, shard, k, dummy_row, window, substep_waves, pp, d_pairs);
}

void device_fast_schedule(hipStream_t st, const DevRatingBlocks& dr, const RatingBlocks& rb, const SideLayout& U,
                          const SideLayout& I, const std::vector<int32_t>& Gb, double lambda, uint64_t order_seed,
                          FastPlan& fp, int32_t c, int32_t shard, int32_t k, uint32_t dummy_row, int32_t window,
                          PairPlan& pp, DevBuf& d_pairs) {
  const int32_t nb = rb.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  const int64_t n = dr.total;
  MF_REQUIRE(n > 0 && n == rb.start[nb2] && n < (int64_t{1} << 31), "device schedule: rating blocks do not match (or none)");
  PlanBlocks pb;
  std::vector<int64_t> uoffb(nb2, 0), ioffb(nb2, 0), cbase(nb2, 0);
  std::vector<int32_t> Gblk(nb2, 1);
  int64_t usum = 0, isum = 0, csum = 0;
  for (int64_t b = 0; b < nb2; ++b) {
    if (rb.size(b) == 0) continue;
    const int32_t p = static_cast<int32_t>(b / nb), q = static_cast<int32_t>(b % nb);
    const int64_t nu = U.block_start[p + 1] - U.block_start[p], ni = I.block_start[q + 1] - I.block_start[q];
    const int64_t G = Gb[b];
    pb.b.push_back(b);
    pb.GG.push_back(G * G);
    pb.nu.push_back(nu);
    pb.nv.push_back(ni);
    pb.len.push_back(rb.size(b));
    pb.ub.push_back(static_cast<uint32_t>(U.block_start[p]));
    uoffb[b] = usum;
    ioffb[b] = isum;
    cbase[b] = csum;
    Gblk[b] = static_cast<int32_t>(G);
    usum += nu;
    isum += ni;
    csum += G * G + 1;
  }
  const int64_t nblk = static_cast<int64_t>(pb.b.size());
  pb.total = n;
  // 1. local rows and the per-block histograms
  DevBuf dbs, dubs, dibs, duo, dio, dblk, dul, dil, ducnt, dicnt;
  upload(dbs, rb.start.data(), rb.start.size(), st);
  upload(dubs, U.block_start.data(), U.block_start.size(), st);
  upload(dibs, I.block_start.data(), I.block_start.size(), st);
  upload(duo, uoffb.data(), uoffb.size(), st);
  upload(dio, ioffb.data(), ioffb.size(), st);
  const size_t nn = static_cast<size_t>(std::max<int64_t>(n, 1));
  dblk.alloc(nn * 4);
  dul.alloc(nn * 4);
  dil.alloc(nn * 4);
  ducnt.alloc(static_cast<size_t>(std::max<int64_t>(usum, 1)) * 4);
  dicnt.alloc(static_cast<size_t>(std::max<int64_t>(isum, 1)) * 4);
  MF_HIP(hipMemsetAsync(ducnt.get(), 0, ducnt.bytes(), st));
  MF_HIP(hipMemsetAsync(dicnt.get(), 0, dicnt.bytes(), st));
  hipLaunchKernelGGL(k_p1_local, dim3(plan_grid(n)), dim3(256), 0, st, dr.urow.as<uint32_t>(), dr.irow.as<uint32_t>(), n,
                     dbs.as<int64_t>(), nb2, nb, dubs.as<int64_t>(), dibs.as<int64_t>(), duo.as<int64_t>(),
                     dio.as<int64_t>(), dblk.as<int32_t>(), dul.as<uint32_t>(), dil.as<uint32_t>(), ducnt.as<int32_t>(),
                     dicnt.as<int32_t>());
  MF_HIP(hipGetLastError());
  std::vector<int32_t> ucnt(usum), icnt(isum);
  if (usum) MF_HIP(hipMemcpyAsync(ucnt.data(), ducnt.get(), usum * 4, hipMemcpyDeviceToHost, st));
  if (isum) MF_HIP(hipMemcpyAsync(icnt.data(), dicnt.get(), isum * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  // 2. LPT groups per block on the host (build_fast_plan phase 1), item ranks inside a group
  std::vector<int32_t> gu(usum), gi(isum), irank(isum);
  std::vector<int32_t> gmax(nblk, 0);
  pb.uoff.assign(nblk + 1, 0);
  pb.voff.assign(nblk + 1, 0);
  for (int64_t bx = 0; bx < nblk; ++bx) {
    pb.uoff[bx + 1] = pb.uoff[bx] + pb.nu[bx];
    pb.voff[bx + 1] = pb.voff[bx] + pb.nv[bx];
  }
  pb.regu.resize(usum);
  pb.regi.resize(isum);
  pb.vrow.resize(isum);
  parallel_tasks(nblk, [&](int64_t bx) {
    const int64_t b = pb.b[bx];
    const int32_t G = Gblk[b];
    const int32_t p = static_cast<int32_t>(b / nb), q = static_cast<int32_t>(b % nb);
    const int64_t nu = pb.nu[bx], ni = pb.nv[bx];
    std::vector<int64_t> lu(ucnt.begin() + uoffb[b], ucnt.begin() + uoffb[b] + nu);
    std::vector<int64_t> li(icnt.begin() + ioffb[b], icnt.begin() + ioffb[b] + ni);
    std::vector<int32_t> g1, g2;
    lpt_assign(lu, G, g1);
    lpt_assign(li, G, g2);
    std::copy(g1.begin(), g1.end(), gu.begin() + uoffb[b]);
    std::copy(g2.begin(), g2.end(), gi.begin() + ioffb[b]);
    std::vector<int32_t> gsize(G, 0);
    for (int64_t il = 0; il < ni; ++il) irank[ioffb[b] + il] = gsize[g2[il]]++;
    gmax[bx] = *std::max_element(gsize.begin(), gsize.end());
    const int64_t ub = U.block_start[p], ib = I.block_start[q];
    for (int64_t ul = 0; ul < nu; ++ul)
      pb.regu[pb.uoff[bx] + ul] = static_cast<float>(lambda / static_cast<double>(U.omega[ub + ul]));
    for (int64_t il = 0; il < ni; ++il) {
      pb.regi[pb.voff[bx] + il] = static_cast<float>(lambda / static_cast<double>(I.omega[ib + il]));
      pb.vrow[pb.voff[bx] + il] = static_cast<uint32_t>(ib + il);
    }
  });
  int32_t R = 1;
  for (int32_t g : gmax) R = std::max(R, g + 1);
  const int64_t ncells = csum;
  // 3. cell-major order (cell, item rank, x)
  DevBuf dGb, dcb, dgu, dgi, dir, dk1, dk1s, dv1, dO1, dcc, dcs;
  upload(dGb, Gblk.data(), Gblk.size(), st);
  upload(dcb, cbase.data(), cbase.size(), st);
  upload(dgu, gu.data(), gu.size(), st);
  upload(dgi, gi.data(), gi.size(), st);
  upload(dir, irank.data(), irank.size(), st);
  dk1.alloc(nn * 8);
  dk1s.alloc(nn * 8);
  dv1.alloc(nn * 4);
  dO1.alloc(nn * 4);
  dcc.alloc(static_cast<size_t>(ncells + 1) * 4);
  MF_HIP(hipMemsetAsync(dcc.get(), 0, dcc.bytes(), st));
  hipLaunchKernelGGL(k_p1_cellkey, dim3(plan_grid(n)), dim3(256), 0, st, dblk.as<int32_t>(), dul.as<uint32_t>(),
                     dil.as<uint32_t>(), n, dGb.as<int32_t>(), dcb.as<int64_t>(), duo.as<int64_t>(), dio.as<int64_t>(),
                     dgu.as<int32_t>(), dgi.as<int32_t>(), dir.as<int32_t>(), static_cast<uint64_t>(R),
                     dk1.as<uint64_t>(), dv1.as<int32_t>(), dcc.as<int32_t>());
  MF_HIP(hipGetLastError());
  SortTemp tmp;
  sort_pairs<uint64_t>(st, tmp, dk1.as<uint64_t>(), dk1s.as<uint64_t>(), dv1.as<int32_t>(), dO1.as<int32_t>(), n,
                       bits_of(static_cast<uint64_t>(ncells) * R));
  // cell starts: inclusive scan of the cell counts (one extra zero slot at the end)
  std::vector<int64_t> cstart(ncells + 1, 0);
  {
    DevBuf incl;
    incl.alloc(static_cast<size_t>(ncells + 1) * 4);
    inclusive_sum(st, tmp, dcc.as<int32_t>(), incl.as<int32_t>(), ncells + 1);
    std::vector<int32_t> h(ncells + 1);
    MF_HIP(hipMemcpyAsync(h.data(), incl.get(), (ncells + 1) * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipStreamSynchronize(st));
    for (int64_t gc = 0; gc < ncells; ++gc) cstart[gc + 1] = h[gc];
  }
  upload(dcs, cstart.data(), cstart.size(), st);
  // 4. runs (cell, item) of that order; within a run each user's ratings counted (o of m)
  DevBuf dhead, drun, dk2, dk2s, dv2, dP2, dseg, dsegs;
  dhead.alloc(nn * 4);
  drun.alloc(nn * 4);
  hipLaunchKernelGGL(k_p1_heads64, dim3(plan_grid(n)), dim3(256), 0, st, dk1s.as<uint64_t>(), n, dhead.as<int32_t>());
  inclusive_sum(st, tmp, dhead.as<int32_t>(), drun.as<int32_t>(), n);
  int32_t nruns = 0;
  MF_HIP(hipMemcpyAsync(&nruns, drun.as<int32_t>() + n - 1, 4, hipMemcpyDeviceToHost, st));
  int64_t numax = 1;
  for (int64_t bx = 0; bx < nblk; ++bx) numax = std::max(numax, pb.nu[bx] + 1);
  MF_HIP(hipStreamSynchronize(st));
  dk1.release();
  dk2.alloc(nn * 8);
  dk2s.alloc(nn * 8);
  dv2.alloc(nn * 4);
  dP2.alloc(nn * 4);
  hipLaunchKernelGGL(k_p1_runuser, dim3(plan_grid(n)), dim3(256), 0, st, drun.as<int32_t>(), dO1.as<int32_t>(),
                     dul.as<uint32_t>(), n, static_cast<uint64_t>(numax), dk2.as<uint64_t>(), dv2.as<int32_t>());
  sort_pairs<uint64_t>(st, tmp, dk2.as<uint64_t>(), dk2s.as<uint64_t>(), dv2.as<int32_t>(), dP2.as<int32_t>(), n,
                       bits_of(static_cast<uint64_t>(nruns) * numax));
  hipLaunchKernelGGL(k_p1_heads64, dim3(plan_grid(n)), dim3(256), 0, st, dk2s.as<uint64_t>(), n, dhead.as<int32_t>());
  dseg.alloc(nn * 4);
  inclusive_sum(st, tmp, dhead.as<int32_t>(), dseg.as<int32_t>(), n);
  int32_t nseg = 0;
  MF_HIP(hipMemcpyAsync(&nseg, dseg.as<int32_t>() + n - 1, 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  dsegs.alloc(static_cast<size_t>(nseg + 1) * 8);
  hipLaunchKernelGGL(k_p1_segstart, dim3(plan_grid(n)), dim3(256), 0, st, dhead.as<int32_t>(), dseg.as<int32_t>(), n,
                     dsegs.as<int64_t>());
  const int64_t nend = n;
  MF_HIP(hipMemcpyAsync(dsegs.as<int64_t>() + nseg, &nend, 8, hipMemcpyHostToDevice, st));
  // 5. spreading positions, then the final order: by position, then (stably) by run
  DevBuf dpos, dposs, dv3, dQ1, dk3, dk3s, dF;
  dpos.alloc(nn * 8);
  dposs.alloc(nn * 8);
  dv3.alloc(nn * 4);
  dQ1.alloc(nn * 4);
  hipLaunchKernelGGL(k_p1_pos, dim3(plan_grid(n)), dim3(256), 0, st, dseg.as<int32_t>(), dsegs.as<int64_t>(),
                     dP2.as<int32_t>(), dO1.as<int32_t>(), dr.urow.as<uint32_t>(), n, order_seed, dpos.as<uint64_t>(),
                     dv3.as<int32_t>());
  MF_HIP(hipGetLastError());
  sort_pairs<uint64_t>(st, tmp, dpos.as<uint64_t>(), dposs.as<uint64_t>(), dv3.as<int32_t>(), dQ1.as<int32_t>(), n, 40);
  dk3.alloc(nn * 4);
  dk3s.alloc(nn * 4);
  dF.alloc(nn * 4);
  hipLaunchKernelGGL(k_p1_runkey, dim3(plan_grid(n)), dim3(256), 0, st, dQ1.as<int32_t>(), drun.as<int32_t>(), n,
                     dk3.as<uint32_t>());
  sort_pairs<uint32_t>(st, tmp, dk3.as<uint32_t>(), dk3s.as<uint32_t>(), dQ1.as<int32_t>(), dF.as<int32_t>(), n,
                       bits_of(static_cast<uint64_t>(nruns)));
  DevBuf dE;
  dE.alloc(nn * sizeof(PlanEnt));
  hipLaunchKernelGGL(k_p1_gather, dim3(plan_grid(n)), dim3(256), 0, st, dF.as<int32_t>(), dO1.as<int32_t>(),
                     dblk.as<int32_t>(), dbs.as<int64_t>(), dul.as<uint32_t>(), dil.as<uint32_t>(), dr.r.as<double>(), n,
                     dE.as<PlanEnt>());
  MF_HIP(hipGetLastError());
  MF_HIP(hipStreamSynchronize(st));
  for (DevBuf* d : {&dk1s, &dv1, &dO1, &dhead, &drun, &dk2, &dk2s, &dv2, &dP2, &dseg, &dsegs, &dpos, &dposs, &dv3, &dQ1,
                    &dk3, &dk3s, &dF, &dblk, &dul, &dil, &dcc})
    d->release();
  fp.Gb.assign(Gblk.begin(), Gblk.end());
  fp.G = *std::max_element(fp.Gb.begin(), fp.Gb.end());
  fp.split_off.assign(nb2 + 1, 0);
  fp.splits.clear();
  fp.scratch_rows = 0;
  emit_and_pair(st, pb, dE, dcs, fp, nb, c, shard, k, dummy_row, window, false, pp, d_pairs);
}

}  // namespace mfhip
