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
  const int32_t W = A.window;
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
        if ((!any_user && ug[y] == prev_ug) || pos - lastu[ug[y]] >= W) return y;
      }
      return -1;
    };
    auto try_item = [&]() -> int32_t {
      if (prev_ig < 0 || igL[prev_ig] == 0) return -1;
      return scan_item(prev_ig, false);
    };
    auto try_user = [&]() -> int32_t {
      if (prev_ug < 0 || ugL[prev_ug] == 0) return -1;
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
  int32_t* kind;             // per wave: kWaveGeneric / kWaveSingleRun
  int32_t* noops;            // per wave: no-op halves
  double* bytes;             // per wave: requested bytes
  int64_t nwaves;
  double row_bytes;
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
    if (single) {  // the lean path's ring: a loaded user row was stored >= kPairRingSingle pairs back
      constexpr int kR = kPairRingSingle - 1;
      uint32_t ring[kR > 0 ? kR : 1][2];
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
    A.kind[w] = single ? kWaveSingleRun : kWaveGeneric;
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

}  // namespace

void device_pair_schedule(hipStream_t st, std::vector<FastBlockWork>& work, FastPlan& fp, int32_t nb, int32_t c,
                          int32_t shard, int32_t k, uint32_t dummy_row, int32_t window, bool substep_waves,
                          PairPlan& pp, DevBuf& d_pairs) {
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  const int64_t nblk = static_cast<int64_t>(work.size());
  // cells indexed like fp.cell_off: per block GG cells + one empty slot
  std::vector<int64_t> eoff(nblk + 1, 0), coff(nblk + 1, 0), vitoff(nblk + 1, 0), uoff(nblk + 1, 0);
  for (int64_t bx = 0; bx < nblk; ++bx) {
    eoff[bx + 1] = eoff[bx] + work[bx].len;
    coff[bx + 1] = coff[bx] + work[bx].GG + 1;
    vitoff[bx + 1] = vitoff[bx] + work[bx].nv;
    uoff[bx + 1] = uoff[bx] + work[bx].nu;
  }
  const int64_t total = eoff[nblk], ncells = coff[nblk];
  std::vector<int64_t> cstart(ncells + 1);
  std::vector<int32_t> cblk(ncells);
  std::vector<uint32_t> bub(nblk);
  std::vector<float> regu(uoff[nblk]), regi(vitoff[nblk]);
  std::vector<uint32_t> vrow(vitoff[nblk]);
  fp.cell_base.assign(nb2, -1);
  fp.rec_base.assign(nb2, -1);
  for (int64_t bx = 0; bx < nblk; ++bx) {
    const FastBlockWork& W = work[bx];
    fp.cell_base[W.b] = coff[bx];
    for (int64_t cc = 0; cc <= W.GG; ++cc) {
      cstart[coff[bx] + cc] = eoff[bx] + W.cstart[cc];
      if (cc < W.GG) cblk[coff[bx] + cc] = static_cast<int32_t>(bx);
    }
    cblk[coff[bx] + W.GG] = static_cast<int32_t>(bx);
    bub[bx] = static_cast<uint32_t>(W.ub);
    std::copy(W.regu.begin(), W.regu.end(), regu.begin() + uoff[bx]);
    std::copy(W.regi.begin(), W.regi.end(), regi.begin() + vitoff[bx]);
    std::copy(W.vrow.begin(), W.vrow.end(), vrow.begin() + vitoff[bx]);
  }
  cstart[ncells] = total;
  DevBuf dE, dcs, dcb, dbub, dbregu, dbvit, dregu, dregi, dvrow;
  dE.alloc(std::max<int64_t>(total, 1) * sizeof(PlanEnt));
  for (int64_t bx = 0; bx < nblk; ++bx)
    if (work[bx].len)
      MF_HIP(hipMemcpyAsync(dE.as<PlanEnt>() + eoff[bx], work[bx].e.data(), work[bx].len * sizeof(PlanEnt),
                            hipMemcpyHostToDevice, st));
  EmitArgs A{};
  A.E = dE.as<PlanEnt>();
  A.cstart = upload(dcs, cstart.data(), cstart.size(), st);
  A.cblk = upload(dcb, cblk.data(), cblk.size(), st);
  A.bub = upload(dbub, bub.data(), bub.size(), st);
  A.bregu = upload(dbregu, uoff.data(), static_cast<size_t>(nblk), st);
  A.bvit = upload(dbvit, vitoff.data(), static_cast<size_t>(nblk), st);
  A.regu = upload(dregu, regu.data(), regu.size(), st);
  A.regi = upload(dregi, regi.data(), regi.size(), st);
  A.vrow = upload(dvrow, vrow.data(), vrow.size(), st);
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
  DevBuf dnrec, dnpads, dnpairs, drecbase, drecs;
  dnrec.alloc(static_cast<size_t>(ncells) * 4);
  dnpads.alloc(static_cast<size_t>(ncells) * 4);
  A.nrec = dnrec.as<int32_t>();
  A.npads = dnpads.as<int32_t>();
  DevBuf derr;
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
    fp.rec_base[work[bx].b] = nrecs;
    int64_t acc = 0;
    for (int64_t cc = 0; cc <= work[bx].GG; ++cc) {
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
  dnpairs.alloc(static_cast<size_t>(ncells) * 4);
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

}  // namespace mfhip
