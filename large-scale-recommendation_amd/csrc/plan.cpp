// plan.cpp -- host-side DSGD blocking and device schedules (see plan.hpp).
#include "plan.hpp"

#include <sys/mman.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>
#include <atomic>
#include <cmath>
#include <numeric>
#include <queue>
#include <random>
#include <string>

#include "common.hpp"
#include "jvm_random.hpp"

namespace mfhip {

namespace {

// Dense id->row table used while blocking when the id range is compact.
struct DenseMap {
  int32_t lo = 0;
  std::vector<int32_t> rows;  // id - lo -> row or -1
  bool ok() const { return !rows.empty(); }
  int32_t find(int32_t id) const {
    int64_t x = static_cast<int64_t>(id) - lo;
    return (x >= 0 && x < static_cast<int64_t>(rows.size())) ? rows[x] : -1;
  }
};

void minmax(const int32_t* ids, int64_t n, int32_t& mn, int32_t& mx) {
  int w = host_threads();
  std::vector<int32_t> a(w, INT32_MAX), b(w, INT32_MIN);
  parallel_for(n, [&](int64_t s, int64_t e, int t) {
    int32_t lo = INT32_MAX, hi = INT32_MIN;
    for (int64_t j = s; j < e; ++j) { lo = std::min(lo, ids[j]); hi = std::max(hi, ids[j]); }
    a[t] = lo; b[t] = hi;
  }, w);
  mn = *std::min_element(a.begin(), a.end());
  mx = *std::max_element(b.begin(), b.end());
}

bool dense_ok(int32_t mn, int32_t mx, int64_t n) {
  const int64_t range = static_cast<int64_t>(mx) - mn + 1;
  return range <= std::max<int64_t>(4 * n, 1 << 22) && range <= (int64_t{1} << 30);
}

}  // namespace

// initFactorBlockAndIndices (DSGDforMF.scala:513-588): distinct ids (:520), block per id
// (:531-533), omega = rating count (:537-541), ids sorted within a block when seeded (:556).
void build_side(SideLayout& s, const int32_t* ids, int64_t n, int32_t nb, int64_t seed, bool has_seed,
                Blocking blocking) {
  s = SideLayout();
  s.n_blocks = nb;
  std::vector<int32_t> distinct, counts;
  if (n > 0) {
    int32_t mn, mx;
    minmax(ids, n, mn, mx);
    if (dense_ok(mn, mx, n)) {
      const int64_t range = static_cast<int64_t>(mx) - mn + 1;
      std::vector<int32_t> cnt(range, 0);
      int32_t* c = cnt.data();
      parallel_for(n, [&](int64_t b, int64_t e, int) {
        for (int64_t j = b; j < e; ++j) __atomic_fetch_add(&c[static_cast<int64_t>(ids[j]) - mn], 1, __ATOMIC_RELAXED);
      });
      for (int64_t x = 0; x < range; ++x)
        if (cnt[x]) { distinct.push_back(static_cast<int32_t>(x + mn)); counts.push_back(cnt[x]); }
    } else {
      std::vector<int32_t> tmp(ids, ids + n);
      std::sort(tmp.begin(), tmp.end());
      for (int64_t j = 0; j < n; ++j) {
        if (j == 0 || tmp[j] != tmp[j - 1]) { distinct.push_back(tmp[j]); counts.push_back(0); }
        counts.back()++;
      }
    }
  }
  const int64_t d = static_cast<int64_t>(distinct.size());
  std::vector<int32_t> blk(d);
  if (blocking == Blocking::kBalanced) {
    std::vector<int64_t> order(d);
    std::vector<uint64_t> tie(d);
    for (int64_t x = 0; x < d; ++x) {
      order[x] = x;
      uint64_t h = static_cast<uint64_t>(static_cast<int64_t>(distinct[x]) ^ seed) * 0x9E3779B97F4A7C15ULL;
      tie[x] = h ^ (h >> 29);
    }
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      return counts[a] != counts[b] ? counts[a] > counts[b] : tie[a] < tie[b];
    });
    using E = std::pair<int64_t, int32_t>;  // (load, block)
    std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
    for (int32_t b = 0; b < nb; ++b) pq.emplace(0, b);
    for (int64_t x : order) {
      E e = pq.top();
      pq.pop();
      blk[x] = e.second;
      e.first += counts[x];
      pq.push(e);
    }
  } else if (has_seed) {
    parallel_for(d, [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x) {
        JavaRandom rng(static_cast<int64_t>(distinct[x]) ^ seed);
        blk[x] = rng.nextInt(nb);
      }
    });
  } else {
    std::random_device rd;
    JavaRandom rng((static_cast<int64_t>(rd()) << 32) ^ rd());
    for (int64_t x = 0; x < d; ++x) blk[x] = rng.nextInt(nb);
  }
  s.block_start.assign(nb + 1, 0);
  for (int64_t x = 0; x < d; ++x) s.block_start[blk[x] + 1]++;
  for (int32_t b = 0; b < nb; ++b) s.block_start[b + 1] += s.block_start[b];
  std::vector<int64_t> fill(s.block_start.begin(), s.block_start.end() - 1);
  s.row_id.resize(d);
  s.omega.resize(d);
  s.row_block.resize(d);
  s.index.reserve(d);
  for (int64_t x = 0; x < d; ++x) {  // ascending ids => ascending within each block
    const int64_t row = fill[blk[x]]++;
    s.row_id[row] = distinct[x];
    s.omega[row] = counts[x];
    s.row_block[row] = blk[x];
    s.index.insert(distinct[x], static_cast<int32_t>(row));
  }
}

void lookup_rows(const SideLayout& s, const int32_t* ids, int64_t n, std::vector<uint32_t>& rows) {
  rows.resize(n);
  DenseMap dm;
  if (s.rows() > 0) {
    int32_t mn = *std::min_element(s.row_id.begin(), s.row_id.end());
    int32_t mx = *std::max_element(s.row_id.begin(), s.row_id.end());
    if (dense_ok(mn, mx, s.rows())) {
      dm.lo = mn;
      dm.rows.assign(static_cast<int64_t>(mx) - mn + 1, -1);
      for (int64_t r = 0; r < s.rows(); ++r) dm.rows[static_cast<int64_t>(s.row_id[r]) - mn] = static_cast<int32_t>(r);
    }
  }
  parallel_for(n, [&](int64_t b, int64_t e, int) {
    if (dm.ok()) for (int64_t j = b; j < e; ++j) rows[j] = static_cast<uint32_t>(dm.find(ids[j]));
    else for (int64_t j = b; j < e; ++j) rows[j] = static_cast<uint32_t>(s.index.find(ids[j]));
  });
}

// Rating blocks (DSGDforMF.scala:301-327): block ub*n+ib, sorted by (user, item) when seeded.
void build_rating_blocks(RatingBlocks& rb, const SideLayout& U, const SideLayout& I,
                         const int32_t* u, const int32_t* i, const double* r, int64_t n,
                         int32_t ub_lo, int32_t ub_hi, bool sort_ui, bool keep_src) {
  const int32_t nb = U.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  rb = RatingBlocks();
  rb.n_blocks = nb;
  std::vector<uint32_t> ur, ir;
  lookup_rows(U, u, n, ur);
  lookup_rows(I, i, n, ir);
  const int w = host_threads();
  const int64_t chunk = (n + w - 1) / std::max(w, 1);
  std::vector<std::vector<int64_t>> hist(w, std::vector<int64_t>(nb2 + 1, 0));
  auto block_of = [&](int64_t j) -> int64_t {
    const int32_t ub = U.row_block[ur[j]];
    if (ub < ub_lo || ub >= ub_hi) return -1;
    return static_cast<int64_t>(ub) * nb + I.row_block[ir[j]];
  };
  parallel_for(n, [&](int64_t b, int64_t e, int t) {
    for (int64_t j = b; j < e; ++j) { int64_t k = block_of(j); if (k >= 0) hist[t][k]++; }
  }, w, chunk);
  rb.start.assign(nb2 + 1, 0);
  for (int64_t k = 0; k < nb2; ++k)
    for (int t = 0; t < w; ++t) rb.start[k + 1] += hist[t][k];
  for (int64_t k = 0; k < nb2; ++k) rb.start[k + 1] += rb.start[k];
  const int64_t total = rb.start[nb2];
  // per (worker, block) write cursors: worker t writes after workers < t (stable)
  for (int64_t k = 0; k < nb2; ++k) {
    int64_t pos = rb.start[k];
    for (int t = 0; t < w; ++t) { int64_t c = hist[t][k]; hist[t][k] = pos; pos += c; }
  }
  rb.urow.resize(total);
  rb.irow.resize(total);
  rb.r.resize(total);
  if (keep_src) rb.src.resize(total);
  std::vector<uint64_t> key;
  if (sort_ui) key.resize(total);
  parallel_for(n, [&](int64_t b, int64_t e, int t) {
    for (int64_t j = b; j < e; ++j) {
      int64_t k = block_of(j);
      if (k < 0) continue;
      int64_t pos = hist[t][k]++;
      rb.urow[pos] = ur[j];
      rb.irow[pos] = ir[j];
      rb.r[pos] = r[j];
      if (keep_src) rb.src[pos] = j;
      if (sort_ui)
        key[pos] = (static_cast<uint64_t>(static_cast<uint32_t>(u[j]) ^ 0x80000000u) << 32) |
                   (static_cast<uint32_t>(i[j]) ^ 0x80000000u);
    }
  }, w, chunk);
  if (!sort_ui) return;
  parallel_tasks(nb2, [&](int64_t k) {
    const int64_t s = rb.start[k], len = rb.start[k + 1] - s;
    if (len < 2) return;
    std::vector<int32_t> idx(len);
    std::iota(idx.begin(), idx.end(), 0);
    const uint64_t* kk = key.data() + s;
    std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return kk[a] < kk[b]; });
    std::vector<uint32_t> tu(len), ti(len);
    std::vector<double> tr(len);
    std::vector<int64_t> ts(keep_src ? len : 0);
    for (int64_t x = 0; x < len; ++x) {
      tu[x] = rb.urow[s + idx[x]]; ti[x] = rb.irow[s + idx[x]]; tr[x] = rb.r[s + idx[x]];
      if (keep_src) ts[x] = rb.src[s + idx[x]];
    }
    std::copy(tu.begin(), tu.end(), rb.urow.begin() + s);
    std::copy(ti.begin(), ti.end(), rb.irow.begin() + s);
    std::copy(tr.begin(), tr.end(), rb.r.begin() + s);
    if (keep_src) std::copy(ts.begin(), ts.end(), rb.src.begin() + s);
  });
}

// Level schedule: level(j) = 1 + max(level of the previous update of the same user row,
// level of the previous update of the same item row) along each sequence's order.  Updates
// of one level touch pairwise-distinct rows, so running a level in parallel and the levels
// in order reproduces the sequential result bit for bit.
void build_level_plan(const std::vector<OrderedSeq>& seqs, LevelPlan& out, std::vector<int32_t>* src) {
  const int64_t ns = static_cast<int64_t>(seqs.size());
  std::vector<std::vector<int32_t>> lvl(ns);
  std::vector<std::vector<int64_t>> cnt(ns);
  parallel_tasks(ns, [&](int64_t x) {
    const OrderedSeq& q = seqs[x];
    std::vector<int32_t> lu(q.u_hi - q.u_lo, 0), li(q.i_hi - q.i_lo, 0);
    lvl[x].resize(q.len);
    int32_t maxl = 0;
    for (int64_t j = 0; j < q.len; ++j) {
      const int64_t e = q.order ? q.order[j] : j;
      int32_t& a = lu[q.u[e] - q.u_lo];
      int32_t& b = li[q.i[e] - q.i_lo];
      const int32_t l = std::max(a, b) + 1;
      a = l;
      b = l;
      lvl[x][j] = l;
      maxl = std::max(maxl, l);
    }
    cnt[x].assign(maxl + 1, 0);
    for (int64_t j = 0; j < q.len; ++j) cnt[x][lvl[x][j]]++;
  });
  int64_t L = 0;
  for (auto& c : cnt) L = std::max<int64_t>(L, static_cast<int64_t>(c.size()) - 1);
  out.level_start.assign(L + 1, 0);
  // cursor[x][l] = where sequence x writes its level-l entries (level-major, then sequence order)
  std::vector<std::vector<int64_t>> cur(ns);
  int64_t pos = 0;
  for (int64_t l = 1; l <= L; ++l) {
    out.level_start[l - 1] = pos;
    for (int64_t x = 0; x < ns; ++x) {
      if (cur[x].empty()) cur[x].assign(cnt[x].size(), 0);
      if (l < static_cast<int64_t>(cnt[x].size())) { cur[x][l] = pos; pos += cnt[x][l]; }
    }
  }
  out.level_start[L] = pos;
  out.entries.resize(pos);
  if (src) src->resize(pos);
  parallel_tasks(ns, [&](int64_t x) {
    const OrderedSeq& q = seqs[x];
    for (int64_t j = 0; j < q.len; ++j) {
      const int64_t e = q.order ? q.order[j] : j;
      const int64_t at = cur[x][lvl[x][j]]++;
      out.entries[at] = DetEntry{q.u[e], q.i[e], q.r[e]};
      if (src) (*src)[at] = static_cast<int32_t>(e);
    }
  });
}

// ---------------------------------------------------------------------------------------
// Deterministic persistent sweep (plan.hpp DetSweepLayout).
void build_det_layout(DetSweepLayout& L, const RatingBlocks& rb, const SideLayout& U, const SideLayout& I, int32_t c,
                      int32_t shard, int32_t waves_per_superstep) {
  (void)U;
  const int32_t nb = rb.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  L.block_waves.assign(nb2, 0);
  L.item_wave.assign(nb2, {});
  L.wave_single.assign(nb2, {});
  // per superstep sm: the shard's blocks (p, (p+sm) mod n) share the wave budget by size
  for (int32_t sm = 0; sm < nb; ++sm) {
    int64_t total = 0;
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j;
      total += rb.size(static_cast<int64_t>(p) * nb + (p + sm) % nb);
    }
    if (total == 0) continue;
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j;
      const int64_t b = static_cast<int64_t>(p) * nb + (p + sm) % nb;
      if (rb.size(b) == 0) continue;
      L.block_waves[b] = static_cast<int32_t>(
          std::max<int64_t>(1, static_cast<int64_t>(waves_per_superstep) * rb.size(b) / total));
    }
  }
  parallel_tasks(nb2, [&](int64_t b) {
    if (L.block_waves[b] == 0) return;
    const int32_t q = static_cast<int32_t>(b % nb);
    const int64_t i0 = I.block_start[q], ni = I.block_start[q + 1] - i0;
    std::vector<int64_t> cnt(ni, 0);
    for (int64_t x = rb.start[b]; x < rb.start[b + 1]; ++x) cnt[rb.irow[x] - i0]++;
    std::vector<int32_t> items;
    for (int64_t x = 0; x < ni; ++x)
      if (cnt[x] > 0) items.push_back(static_cast<int32_t>(x));
    const int32_t W = std::max<int32_t>(1, std::min<int32_t>(L.block_waves[b], static_cast<int32_t>(items.size())));
    L.block_waves[b] = W;
    // LPT: heaviest item first onto the least-loaded wave (ties: lower wave), so the hottest
    // items sit alone in their waves
    std::stable_sort(items.begin(), items.end(), [&](int32_t a, int32_t c2) { return cnt[a] > cnt[c2]; });
    using Load = std::pair<int64_t, int32_t>;
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
    for (int32_t w = 0; w < W; ++w) heap.emplace(0, w);
    auto& iw = L.item_wave[b];
    iw.assign(ni, -1);
    std::vector<int32_t> nitems(W, 0);
    for (int32_t it : items) {
      Load top = heap.top();
      heap.pop();
      iw[it] = top.second;
      nitems[top.second]++;
      top.first += cnt[it];
      heap.push(top);
    }
    auto& ws = L.wave_single[b];
    ws.assign(W, 0);
    for (int32_t w = 0; w < W; ++w) ws[w] = nitems[w] == 1;
  });
}

// MFHIP_TIMING: wall time of build_det_step's phases, summed over calls (det_build_phase_ns)
std::atomic<int64_t> g_det_phase_ns[5];
int64_t det_build_phase_ns(int ph) { return g_det_phase_ns[ph]; }

void build_det_step(const RatingBlocks& rb, const SideLayout& U, const SideLayout& I, const DetSweepLayout& L,
                    const std::vector<int64_t>& blocks, const std::vector<int64_t>& seeds, bool seeded,
                    const DetStepOut& out, DetStepScratch* scratch) {
  auto ph_t = std::chrono::steady_clock::now();
  auto lap = [&](int ph) {
    const auto now = std::chrono::steady_clock::now();
    g_det_phase_ns[ph] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - ph_t).count();
    ph_t = now;
  };
  const int32_t nb = rb.n_blocks;
  const int64_t nbk = static_cast<int64_t>(blocks.size());
  DetStepScratch local;
  DetStepScratch& sc = scratch ? *scratch : local;
  for (auto* v : {&sc.order, &sc.wv}) if (static_cast<int64_t>(v->size()) < nbk) v->resize(nbk);
  for (auto* v : {&sc.gu, &sc.gi}) if (static_cast<int64_t>(v->size()) < nbk) v->resize(nbk);
  if (static_cast<int64_t>(sc.gr.size()) < nbk) sc.gr.resize(nbk);
  std::vector<int64_t> e0(nbk + 1, 0), w0(nbk + 1, 0);  // entry / wave offsets of each block
  for (int64_t x = 0; x < nbk; ++x) {
    e0[x + 1] = e0[x] + rb.size(blocks[x]);
    w0[x + 1] = w0[x] + L.block_waves[blocks[x]];
  }
  std::vector<uint64_t> rseeds(nbk);
  if (!seeded) {
    std::random_device rd;
    for (auto& v : rseeds) v = (static_cast<uint64_t>(rd()) << 32) ^ rd();
  }
  // 1. the shuffle of each block (serial within a block: one JavaRandom stream)
  auto& order = sc.order;
  parallel_tasks(nbk, [&](int64_t x) {
    const int64_t len = rb.size(blocks[x]);
    if (len == 0) return;
    order[x].resize(len);
    JavaRandom rng(seeded ? seeds[x] : static_cast<int64_t>(rseeds[x]));
    scala_shuffle(rng, order[x].data(), len);  // DSGDforMF.scala:392-393
  });
  lap(0);
  // the rest runs over chunks of shuffle positions, so a large block does not hold up the step
  constexpr int64_t kChunk = int64_t{1} << 18;
  struct Chunk {
    int64_t x, j0, j1;
  };
  std::vector<Chunk> ch;
  std::vector<int64_t> ch0(nbk + 1, 0);
  for (int64_t x = 0; x < nbk; ++x) {
    ch0[x] = static_cast<int64_t>(ch.size());
    const int64_t len = rb.size(blocks[x]);
    for (int64_t j = 0; j < len; j += kChunk) ch.push_back(Chunk{x, j, std::min(len, j + kChunk)});
  }
  ch0[nbk] = static_cast<int64_t>(ch.size());
  auto& gu = sc.gu;
  auto& gi = sc.gi;
  auto& gr = sc.gr;
  auto& wv = sc.wv;
  for (int64_t x = 0; x < nbk; ++x) {
    const int64_t len = rb.size(blocks[x]);
    gu[x].resize(len);
    gi[x].resize(len);
    gr[x].resize(len);
    wv[x].resize(len);
  }
  auto block_geom = [&](int64_t x, int64_t& st, int64_t& u0, int64_t& nu, int64_t& i0) {
    const int64_t b = blocks[x];
    const int32_t p = static_cast<int32_t>(b / nb), q = static_cast<int32_t>(b % nb);
    st = rb.start[b];
    u0 = U.block_start[p];
    nu = U.block_start[p + 1] - u0;
    i0 = I.block_start[q];
  };
  // 2. per chunk: the ratings in shuffle order, gathered once (the only random reads), their
  // waves, and per-chunk counts of waves and users
  std::vector<std::vector<int64_t>> wcur(ch.size());
  std::vector<std::vector<int32_t>> ucur(ch.size());
  const DetEntry* const aos = rb.det_aos.empty() ? nullptr : rb.det_aos.data();
  parallel_tasks(static_cast<int64_t>(ch.size()), [&](int64_t t) {
    const Chunk c = ch[t];
    int64_t st, u0, nu, i0;
    block_geom(c.x, st, u0, nu, i0);
    const auto& iw = L.item_wave[blocks[c.x]];
    const int32_t* ord = order[c.x].data();
    wcur[t].assign(L.block_waves[blocks[c.x]], 0);
    ucur[t].assign(nu, 0);
    constexpr int64_t kAhead = 64;  // the rating arrays are far larger than the caches
    for (int64_t j = c.j0; j < c.j1; ++j) {
      if (j + kAhead < c.j1) {
        const int64_t ea = st + ord[j + kAhead];
        if (aos) {
          __builtin_prefetch(aos + ea);
        } else {
          __builtin_prefetch(&rb.urow[ea]);
          __builtin_prefetch(&rb.irow[ea]);
          __builtin_prefetch(&rb.r[ea]);
        }
      }
      const int64_t e = st + ord[j];
      uint32_t ur, ir;
      if (aos) {
        const DetEntry& de = aos[e];
        ur = de.u;
        ir = de.i;
        gr[c.x][j] = de.r;
      } else {
        ur = rb.urow[e];
        ir = rb.irow[e];
        gr[c.x][j] = rb.r[e];
      }
      gu[c.x][j] = ur;
      gi[c.x][j] = ir;
      const int32_t w = iw[ir - i0];
      wv[c.x][j] = w;
      wcur[t][w]++;
      ucur[t][ur - u0]++;
    }
  });
  lap(1);
  // 3. per block: wave offsets, and each chunk's start per wave and per user (its counts turned
  // into exclusive prefixes over the block's chunks)
  parallel_tasks(nbk, [&](int64_t x) {
    const int32_t W = L.block_waves[blocks[x]];
    if (rb.size(blocks[x]) == 0) return;
    int64_t st, u0, nu, i0;
    block_geom(x, st, u0, nu, i0);
    int64_t at = e0[x];
    for (int32_t w = 0; w < W; ++w) {
      const int64_t wbeg = at;
      for (int64_t t = ch0[x]; t < ch0[x + 1]; ++t) {
        const int64_t cnt = wcur[t][w];
        wcur[t][w] = at;
        at += cnt;
      }
      out.waves[w0[x] + w] = DetWave{wbeg, static_cast<int32_t>(at - wbeg), 0};
    }
    for (int64_t uu = 0; uu < nu; ++uu) {
      int32_t run = 0;
      for (int64_t t = ch0[x]; t < ch0[x + 1]; ++t) {
        const int32_t cnt = ucur[t][uu];
        ucur[t][uu] = run;
        run += cnt;
      }
    }
  });
  lap(2);
  // 4. per chunk: the scatter into wave-major order; useq = the user's count of earlier ratings
  // in shuffle order
  parallel_tasks(static_cast<int64_t>(ch.size()), [&](int64_t t) {
    const Chunk c = ch[t];
    int64_t st, u0, nu, i0;
    block_geom(c.x, st, u0, nu, i0);
    std::vector<int64_t>& cur = wcur[t];
    std::vector<int32_t>& useq = ucur[t];
    for (int64_t j = c.j0; j < c.j1; ++j) {
      const uint32_t ur = gu[c.x][j];
      const int64_t at = cur[wv[c.x][j]]++;
      out.u[at] = ur;
      out.i[at] = gi[c.x][j];
      out.qf[at] = static_cast<uint32_t>(useq[ur - u0]++);
      out.r[at] = gr[c.x][j];
    }
  });
  lap(3);
  // 5. a wave that holds one item of its block is a single-item wave (the layout's, static)
  for (int64_t x = 0; x < nbk; ++x) {
    const auto& ws = L.wave_single[blocks[x]];
    for (int32_t w = 0; w < L.block_waves[blocks[x]]; ++w)
      out.waves[w0[x] + w].flags = ws[w] ? kDetWaveSingleItem : 0;  // the sweep's lean / split path
  }
  lap(4);
}

// G trades launch/cell overhead and the record padding forced by heavy users (large G) against
// cell imbalance (small G).  The per-superstep critical path is the sum over sub-steps of the
// longest cell; on the NFLX-shaped synthetic it is minimal near ~150 ratings per average cell
// for the one-update-per-step kernel (G = 96 for 1.4M-rating blocks).  The pair kernel does
// best near 1024 waves per sub-step with cells of >= ~40 ratings (NFLX: G = 128; ML20M, 281k
// ratings per block: G = 80), the cell_target / default_waves the caller passes.
int32_t choose_groups(int64_t avg_block_ratings, int32_t blocks_per_device, int32_t fast_waves, double cell_target,
                      int32_t default_waves) {
  if (fast_waves < 0) return std::clamp(-fast_waves, 1, 4096);
  const int32_t waves = fast_waves > 0 ? fast_waves : default_waves;
  int64_t g = waves / std::max(blocks_per_device, 1);
  const int64_t cap = static_cast<int64_t>(std::sqrt(std::max<double>(avg_block_ratings, 1.0) / cell_target));
  g = std::min(g, cap);
  g = (g / 4) * 4;
  return static_cast<int32_t>(std::clamp<int64_t>(g, 4, 1024));
}

void hugepage_hint(void* p, size_t bytes) {
  constexpr uintptr_t kHuge = uintptr_t{1} << 21;
  const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
  if (e > a) madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

namespace {
// Longest-processing-time greedy: heaviest rows first into the least-loaded group.
void lpt_groups(const std::vector<int64_t>& load, int32_t G, std::vector<int32_t>& group) {
  const int64_t n = static_cast<int64_t>(load.size());
  group.assign(n, 0);
  std::vector<int32_t> order;
  order.reserve(n);
  for (int64_t x = 0; x < n; ++x) if (load[x] > 0) order.push_back(static_cast<int32_t>(x));
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return load[a] != load[b] ? load[a] > load[b] : a < b;
  });
  using E = std::pair<int64_t, int32_t>;
  std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
  for (int32_t g = 0; g < G; ++g) pq.emplace(0, g);
  for (int32_t x : order) {
    E e = pq.top();
    pq.pop();
    group[x] = e.second;
    e.first += load[x];
    pq.push(e);
  }
}

// MFHIP_TIMING: build_fast_plan's per-phase thread time (summed over blocks), on stderr
struct PhaseTimes {
  std::atomic<int64_t> ns[5];
  const char* names[5] = {"groups", "keys+sort", "spread", "emit", "other"};
};
PhaseTimes g_fp_times;
struct PhaseTick {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(int phase) {
    const auto now = std::chrono::steady_clock::now();
    g_fp_times.ns[phase] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
    t = now;
  }
};

inline uint32_t mix32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return static_cast<uint32_t>(x);
}
}  // namespace

// Fast-mode rotation schedule.  Within rating block (p, q): items of block q are split into
// G groups and users of block p into G groups (both LPT-balanced by rating count in the
// block); cell (t, g) holds the ratings with item group g and user group (g + t) mod G.
// Cells of one sub-step t share no user or item row.  Inside a cell the ratings are ordered
// by item (one contiguous run per item, so the item row stays in registers) and by a hash
// of the user inside an item run.
void build_fast_plan(FastPlan& fp, const RatingBlocks& rb, const SideLayout& U, const SideLayout& I,
                     int32_t G0, int32_t k, double lambda, uint64_t order_seed, uint32_t dummy_row,
                     std::vector<int64_t>* rec_src, int32_t window, const std::vector<int32_t>* block_groups,
                     int32_t split_run, uint32_t scratch_base, std::vector<FastBlockWork>* entries_out) {
  // (plan.hpp plan_window_pack: mixed cells' window, single-item cells' window)
  const int64_t kHazardWindow = plan_window_mixed(window);  // shadows the default for this plan
  const int64_t kRunWindow = plan_window_run(window);
  const bool strict_runs = plan_window_strict_runs(window);
  const uint32_t row_bytes = static_cast<uint32_t>(k) * 4u;
  const int32_t nb = rb.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  fp = FastPlan();
  fp.G = G0;
  fp.Gb.assign(nb2, G0);
  if (block_groups) {
    for (int64_t b = 0; b < nb2; ++b) fp.Gb[b] = (*block_groups)[b] > 0 ? (*block_groups)[b] : G0;
    fp.G = *std::max_element(fp.Gb.begin(), fp.Gb.end());
  }
  fp.rec_base.assign(nb2, -1);
  fp.cell_base.assign(nb2, -1);
  std::vector<int64_t> blocks;
  for (int64_t b = 0; b < nb2; ++b)
    if (rb.size(b) > 0) blocks.push_back(b);
  const int64_t nblk = static_cast<int64_t>(blocks.size());
  std::vector<int64_t> pads(nblk, 0);
  // hot-item replicas: per block, the items with more than split_run ratings and their R
  std::vector<std::vector<std::pair<uint32_t, int32_t>>> hot(nblk);
  if (split_run > 0)
    parallel_tasks(nblk, [&](int64_t bx) {
      const int64_t b = blocks[bx];
      const int32_t q = static_cast<int32_t>(b % nb);
      const int64_t ib = I.block_start[q], ni = I.block_start[q + 1] - ib;
      std::vector<int32_t> cnt(ni, 0);
      for (int64_t j = rb.start[b]; j < rb.start[b + 1]; ++j) cnt[rb.irow[j] - ib]++;
      for (int64_t il = 0; il < ni; ++il)
        if (cnt[il] > split_run)
          hot[bx].push_back({static_cast<uint32_t>(il), static_cast<int32_t>((cnt[il] + split_run - 1) / split_run)});
    });
  fp.split_off.assign(nb2 + 1, 0);
  std::vector<int64_t> split_first(nblk, 0);
  {
    uint32_t cursor = 0;
    for (int64_t bx = 0, b = 0; b < nb2; ++b) {
      fp.split_off[b + 1] = fp.split_off[b];
      if (bx < nblk && blocks[bx] == b) {
        const int32_t q = static_cast<int32_t>(b % nb);
        split_first[bx] = static_cast<int64_t>(fp.splits.size());
        for (const auto& h : hot[bx]) {
          fp.splits.push_back(SplitItem{static_cast<uint32_t>(I.block_start[q]) + h.first, scratch_base + cursor, h.second});
          cursor += static_cast<uint32_t>(h.second - 1);
        }
        fp.split_off[b + 1] = static_cast<int64_t>(fp.splits.size());
        ++bx;
      }
    }
    fp.scratch_rows = cursor;
  }
  for (auto& x : g_fp_times.ns) x = 0;
  // Phase 1, per block: virtual items, LPT groups, cell-major order and the spreading of
  // repeated users.  Its result (the block's entries in final cell order, as flat arrays) feeds
  // phase 2, which emits cells in independent chunks.
  using BlockWork = FastBlockWork;
  std::vector<BlockWork> work(nblk);
  const auto wall0 = std::chrono::steady_clock::now();
  auto wall = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - wall0).count(); };
  parallel_tasks(nblk, [&](int64_t bx) {
    PhaseTick tick;
    BlockWork& W = work[bx];
    const int64_t b = blocks[bx];
    const int32_t G = fp.Gb[b];
    const int64_t T = G;       // sub-steps = user groups
    const int64_t GG = T * G;  // cells
    const int32_t p = static_cast<int32_t>(b / nb), q = static_cast<int32_t>(b % nb);
    const int64_t ub = U.block_start[p], nu = U.block_start[p + 1] - ub;
    const int64_t ib = I.block_start[q], ni = I.block_start[q + 1] - ib;
    const int64_t s = rb.start[b], len = rb.size(b);
    // virtual local items: 0..ni-1 the block's items, ni.. the replicas 1..R-1 of its hot items
    // (a hot item's ratings go round-robin to its R chains in block order)
    std::vector<uint32_t> vil(len), vrow;     // rating -> virtual item; virtual item -> global row
    std::vector<uint32_t> vreal;              // virtual item -> the item's own global row (omega)
    int64_t nv = ni;
    {
      std::vector<int32_t> hix(ni, -1), seen;
      std::vector<int64_t> vbase;
      const auto& hb = hot[bx];
      for (size_t h = 0; h < hb.size(); ++h) {
        hix[hb[h].first] = static_cast<int32_t>(h);
        vbase.push_back(nv);
        nv += hb[h].second - 1;
      }
      seen.assign(hb.size(), 0);
      vrow.resize(nv);
      vreal.resize(nv);
      for (int64_t il = 0; il < ni; ++il) vrow[il] = vreal[il] = static_cast<uint32_t>(ib + il);
      for (size_t h = 0; h < hb.size(); ++h)
        for (int32_t r = 1; r < hb[h].second; ++r) {
          vrow[vbase[h] + r - 1] = fp.splits[split_first[bx] + h].scratch_row + static_cast<uint32_t>(r - 1);
          vreal[vbase[h] + r - 1] = static_cast<uint32_t>(ib + hb[h].first);
        }
      for (int64_t x = 0; x < len; ++x) {
        const uint32_t il = rb.irow[s + x] - static_cast<uint32_t>(ib);
        const int32_t h = hix[il];
        if (h < 0) { vil[x] = il; continue; }
        const int32_t r = seen[h]++ % hb[h].second;
        vil[x] = r == 0 ? il : static_cast<uint32_t>(vbase[h] + r - 1);
      }
    }
    std::vector<uint32_t> ulx(len);  // local user of every rating (x order)
    for (int64_t x = 0; x < len; ++x) ulx[x] = rb.urow[s + x] - static_cast<uint32_t>(ub);
    std::vector<int64_t> lu(nu, 0), li(nv, 0);
    for (int64_t x = 0; x < len; ++x) { lu[ulx[x]]++; li[vil[x]]++; }
    std::vector<int32_t> gu, gi;
    lpt_groups(lu, static_cast<int32_t>(T), gu);
    lpt_groups(li, G, gi);
    tick.lap(0);
    // Cell-major order (cell, item, x): two stable counting sorts, by item and then by cell.  The
    // spreading below depends only on each user's ratings of a run in x order, so this is the
    // plan of sorting the block by (cell, item, per-user hash, x).  The entries are gathered into
    // flat arrays in that order, so everything after reads them sequentially.
    W.cstart.assign(GG + 1, 0);
    std::vector<int64_t>& cstart = W.cstart;
    RecVec<PlanEnt>& E = W.e;
    resize_huge(E, len);
    {
      std::vector<int32_t> cell_of(len);
      for (int64_t x = 0; x < len; ++x) {
        const int32_t g = gi[vil[x]], h = gu[ulx[x]];
        const int64_t d = h - static_cast<int64_t>(g);  // in (-T, T)
        const int64_t t = d < 0 ? d + T : d;
        cell_of[x] = static_cast<int32_t>(t * G + g);
        cstart[cell_of[x] + 1]++;
      }
      for (int64_t c = 0; c < GG; ++c) cstart[c + 1] += cstart[c];
      std::vector<int64_t> cur(cstart.begin(), cstart.end() - 1);
      for (int64_t x = 0; x < len; ++x)
        E[cur[cell_of[x]]++] = PlanEnt{static_cast<uint32_t>(x), ulx[x], vil[x], static_cast<float>(rb.r[s + x])};
      // inside a cell: by item, x order kept (entries arrive in x order).  A cell's items all
      // belong to its item group, so this is a counting sort over the group's items, ranked by id.
      std::vector<int32_t> irank(nv), gsize(G, 0);
      for (int64_t v = 0; v < nv; ++v) irank[v] = gsize[gi[v]]++;
      const int32_t gmax = *std::max_element(gsize.begin(), gsize.end());
      std::vector<int32_t> bucket(gmax + 1);
      std::vector<PlanEnt> tmp;
      for (int64_t c = 0; c < GG; ++c) {
        const int64_t c0 = cstart[c], m = cstart[c + 1] - c0;
        if (m < 2) continue;
        const int32_t g = static_cast<int32_t>(c % G), ng = gsize[g];
        std::fill(bucket.begin(), bucket.begin() + ng + 1, 0);
        for (int64_t y = c0; y < c0 + m; ++y) bucket[irank[E[y].vil] + 1]++;
        for (int32_t r = 0; r < ng; ++r) bucket[r + 1] += bucket[r];
        tmp.assign(E.begin() + c0, E.begin() + c0 + m);
        for (const PlanEnt& e : tmp) E[c0 + bucket[irank[e.vil]]++] = e;
      }
    }
    tick.lap(1);
    // Repeated (user, item) ratings (frequent in Zipf-distributed data: a heavy user rates a hot
    // item dozens of times) would sit next to each other and force no-op halves into the pair
    // steps (a pair cannot hold one user twice).  Spread them: inside an item run, the m
    // ratings of one user go to the fractional positions (o + h_u) / m, o = 0..m-1, h_u a
    // per-user hash in [0, 1) -- evenly over the whole run, interleaved with everyone else;
    // ties by a second per-user hash, then x.
    {
      struct K2 { uint64_t pos; PlanEnt e; };
      std::vector<K2> k2;
      std::vector<uint32_t> ucnt(nu, 0), unext(nu, 0);  // per local user in the current run
      for (int64_t c = 0; c < GG; ++c)
        for (int64_t y0 = cstart[c], ye = cstart[c + 1]; y0 < ye;) {
          const uint32_t v0 = E[y0].vil;
          int64_t y1 = y0;
          while (y1 < ye && E[y1].vil == v0) ucnt[E[y1].ul]++, ++y1;
          if (y1 - y0 > 1) {
            k2.resize(y1 - y0);
            for (int64_t y = y0; y < y1; ++y) {
              const uint32_t ul = E[y].ul;
              const uint32_t urow = ul + static_cast<uint32_t>(ub);
              const double h = static_cast<double>(mix32(order_seed * 0x2545F4914F6CDD1DULL ^ urow)) * (1.0 / 4294967296.0);
              const double frac = (unext[ul]++ + h) / ucnt[ul];
              const uint64_t tie = mix32(order_seed ^ (static_cast<uint64_t>(urow) << 20)) & 0xFFFFu;
              k2[y - y0] = K2{(static_cast<uint64_t>(frac * 16777216.0) << 16) | tie, E[y]};
            }
            std::sort(k2.begin(), k2.end(), [](const K2& a2, const K2& b2) { return a2.pos != b2.pos ? a2.pos < b2.pos : a2.e.x < b2.e.x; });
            for (int64_t y = y0; y < y1; ++y) E[y] = k2[y - y0].e;
          }
          for (int64_t y = y0; y < y1; ++y) ucnt[E[y].ul] = unext[E[y].ul] = 0;
          y0 = y1;
        }
    }
    W.regu.resize(nu);
    W.regi.resize(nv);
    for (int64_t ul = 0; ul < nu; ++ul) W.regu[ul] = static_cast<float>(lambda / static_cast<double>(U.omega[ub + ul]));
    for (int64_t il = 0; il < nv; ++il) W.regi[il] = static_cast<float>(lambda / static_cast<double>(I.omega[vreal[il]]));
    W.vrow = std::move(vrow);
    W.b = b; W.len = len; W.nu = nu; W.nv = nv; W.ub = ub; W.GG = GG; W.T = T;
    tick.lap(2);
  });
  const double wall_p1 = wall();
  if (entries_out) {  // the caller emits (kernels_plan.hip); fp keeps the groups and the splits
    if (std::getenv("MFHIP_TIMING"))
      std::fprintf(stderr, "[mfhip]   fast plan wall: blocks %.3f s (emission on the device)\n", wall_p1);
    *entries_out = std::move(work);
    return;
  }
  // Phase 2: emit.  Cells are independent, so a block's cells are cut into chunks of whole cells
  // of about kChunk entries, emitted in parallel and concatenated in cell order.
  struct Chunk2 { int64_t bx, c0, c1; std::vector<FastRec> out; std::vector<int64_t> src; std::vector<int32_t> off; int64_t pads = 0; };
  std::vector<Chunk2> chunks;
  {
    constexpr int64_t kChunk = 1 << 17;
    for (int64_t bx = 0; bx < nblk; ++bx) {
      const BlockWork& W = work[bx];
      int64_t c0 = 0;
      for (int64_t c = 1; c <= W.GG; ++c)
        if (c == W.GG || W.cstart[c] - W.cstart[c0] >= kChunk) {
          chunks.push_back(Chunk2{bx, c0, c, {}, {}, {}, 0});
          c0 = c;
        }
    }
  }
  // largest first, so the tail of the task list is short
  std::vector<int64_t> corder(chunks.size());
  std::iota(corder.begin(), corder.end(), 0);
  std::stable_sort(corder.begin(), corder.end(), [&](int64_t a2, int64_t b2) {
    const BlockWork &A = work[chunks[a2].bx], &B = work[chunks[b2].bx];
    return A.cstart[chunks[a2].c1] - A.cstart[chunks[a2].c0] > B.cstart[chunks[b2].c1] - B.cstart[chunks[b2].c0];
  });
  parallel_tasks(static_cast<int64_t>(chunks.size()), [&](int64_t cx) {
    PhaseTick tick;
    Chunk2& ck = chunks[corder[cx]];
    const BlockWork& W = work[ck.bx];
    const int64_t b = blocks[ck.bx];
    const int64_t s = rb.start[b];
    const uint32_t ub = static_cast<uint32_t>(W.ub);
    // Emit each cell as a sequence the kernel can run with a D-deep prefetch ring: every user
    // and every item row recurs either at the next position (the kernel forwards it in
    // registers: item runs and user runs) or at least kHazardWindow positions later (its
    // store has been issued before the prefetch).  Greedy per position: continue the current
    // item run, or the current user run when that user has more pending ratings than the
    // item; otherwise start from the item with the most pending ratings whose row and some
    // pending user row are both free; only when nothing qualifies emit a no-op record (zero
    // user row, current item).  last_*[x] = (stream, position) of the row's latest emission.
    // Groups are flat: an item group is a contiguous range of the cell's entries, a user group a
    // range of a per-cell CSR list (entries in cell order).
    std::vector<FastRec>& out = ck.out;
    std::vector<int64_t>& src = ck.src;
    std::vector<int32_t>& off = ck.off;
    const int64_t n_in = W.cstart[ck.c1] - W.cstart[ck.c0];
    out.reserve(n_in + n_in / 8 + 16);
    if (rec_src) src.reserve(n_in + n_in / 8 + 16);
    off.assign(ck.c1 - ck.c0, 0);  // end of each cell, relative to the chunk
    struct Last { int32_t sid, pos; };
    // the emission state is kept per cell-local user / item slot (small, hot arrays)
    std::vector<Last> last_u, last_i;
    std::vector<std::pair<int32_t, int32_t>> uslot(W.nu, {-1, 0});
    struct Ent { uint32_t ul, il; int32_t ug, ig; int64_t y; };
    struct Grp { int32_t beg = 0, end = 0, head = 0, left = 0; uint32_t row = 0; };  // [beg, end) of its list
    std::vector<Ent> ents;
    std::vector<Grp> igs, ugs;
    std::vector<int32_t> ulist, ufill;  // user groups' entry lists (CSR over ugs)
    std::vector<uint8_t> taken;
    std::vector<int32_t> iorder;
    // positions and the window count from the start of the cell (sid = the cell)
    for (int64_t c = ck.c0; c < ck.c1; ++c) {
      const int32_t sid = static_cast<int32_t>(c);
      const int64_t stream_begin = static_cast<int64_t>(out.size());
      uint32_t prev_irow = 0;
      ents.clear();
      igs.clear();
      ugs.clear();
      for (int64_t y = W.cstart[c]; y < W.cstart[c + 1]; ++y) {
        const uint32_t il = W.e[y].vil, ul = W.e[y].ul;
        const int32_t e = static_cast<int32_t>(ents.size());
        if (igs.empty() || ents.back().il != il) {
          igs.emplace_back();
          igs.back().row = il;
          igs.back().beg = igs.back().head = e;
        }
        auto& us = uslot[ul];
        if (us.first != c) { us = {static_cast<int32_t>(c), static_cast<int32_t>(ugs.size())}; ugs.emplace_back(); }
        ents.push_back(Ent{ul, il, us.second, static_cast<int32_t>(igs.size()) - 1, y});
        igs.back().end = e + 1;
        ugs[us.second].end++;  // count for now
      }
      const int32_t m = static_cast<int32_t>(ents.size());
      last_u.assign(ugs.size(), Last{-1, 0});  // slots of this cell start free
      last_i.assign(igs.size(), Last{-1, 0});
      {  // user groups: counts -> CSR ranges, entries in cell order
        int32_t acc = 0;
        for (auto& g2 : ugs) { const int32_t n2 = g2.end; g2.beg = g2.head = acc; acc += n2; g2.end = acc; }
        ulist.resize(m);
        ufill.resize(ugs.size());
        for (size_t g2 = 0; g2 < ugs.size(); ++g2) ufill[g2] = ugs[g2].beg;
        for (int32_t e = 0; e < m; ++e) ulist[ufill[ents[e].ug]++] = e;
      }
      taken.assign(m, 0);
      for (auto& g2 : igs) g2.left = g2.end - g2.beg;
      for (auto& g2 : ugs) g2.left = g2.end - g2.beg;
      iorder.resize(igs.size());
      std::iota(iorder.begin(), iorder.end(), 0);
      std::stable_sort(iorder.begin(), iorder.end(), [&](int32_t a2, int32_t b2) {
        return igs[a2].end - igs[a2].beg > igs[b2].end - igs[b2].beg;
      });
      size_t iorder_head = 0;
      int32_t prev_ug = -1, prev_ig = -1;
      int32_t left = m;
      // a single-item cell with a run window: no user within win records, not even the next one
      const bool run_cell = strict_runs && igs.size() == 1;
      const int64_t win = igs.size() == 1 ? kRunWindow : kHazardWindow;
      while (left > 0) {
        const int32_t pos = static_cast<int32_t>(static_cast<int64_t>(out.size()) - stream_begin);
        auto free_at = [&](const Last& L) { return L.sid != sid || pos - L.pos >= win; };
        auto ufree = [&](const Ent& en) { return free_at(last_u[en.ug]); };
        auto ifree = [&](int32_t ig) { return free_at(last_i[ig]); };
        // the first untaken entries of a group's list (at most 4 * window of them) that pass ok
        auto scan = [&](Grp& g2, const int32_t* list, auto ok) -> int32_t {
          while (g2.head < g2.end && taken[list ? list[g2.head] : g2.head]) ++g2.head;
          int seen = 0;
          for (int32_t y = g2.head; y < g2.end && seen < 4 * win; ++y) {
            const int32_t e = list ? list[y] : y;
            if (taken[e]) continue;
            ++seen;
            if (ok(ents[e])) return e;
          }
          return -1;
        };
        auto try_item = [&]() -> int32_t {  // continue the item run
          if (prev_ig < 0 || igs[prev_ig].left == 0) return -1;
          return scan(igs[prev_ig], nullptr, [&](const Ent& en) { return (!run_cell && en.ug == prev_ug) || ufree(en); });
        };
        auto try_user = [&]() -> int32_t {  // continue the user run
          if (run_cell || prev_ug < 0 || ugs[prev_ug].left == 0) return -1;
          return scan(ugs[prev_ug], ulist.data(), [&](const Ent& en) { return en.ig == prev_ig || ifree(en.ig); });
        };
        const bool user_first = prev_ug >= 0 && prev_ig >= 0 && ugs[prev_ug].left > igs[prev_ig].left;
        int32_t pick = user_first ? try_user() : try_item();
        if (pick < 0) pick = user_first ? try_item() : try_user();
        if (pick < 0) {  // fresh start: both rows free
          while (iorder_head < iorder.size() && igs[iorder[iorder_head]].left == 0) ++iorder_head;
          int tried = 0;
          for (size_t z = iorder_head; z < iorder.size() && tried < 64; ++z) {
            Grp& g2 = igs[iorder[z]];
            if (g2.left == 0) continue;
            ++tried;
            if (!ifree(iorder[z])) continue;
            pick = scan(g2, nullptr, [&](const Ent& en) { return ufree(en); });
            if (pick >= 0) break;
          }
        }
        if (pick < 0) {  // no-op record: zero user row, the current item (forwarded)
          out.push_back(FastRec{dummy_row * row_bytes, prev_irow * row_bytes, 0.f, 0.f, 0.f, dummy_row,
                                prev_irow | kPadBit, 0});
          if (rec_src) src.push_back(-1);
          ck.pads++;
          if (prev_ig >= 0) last_i[prev_ig] = Last{sid, pos};
          prev_ug = -1;
          continue;
        }
        const Ent& en = ents[pick];
        taken[pick] = 1;
        --left;
        igs[en.ig].left--;
        ugs[en.ug].left--;
        last_u[en.ug] = Last{sid, pos};
        last_i[en.ig] = Last{sid, pos};
        prev_ug = en.ug;
        prev_ig = en.ig;
        const uint32_t urow = en.ul + ub;
        prev_irow = W.vrow[en.il];
        out.push_back(FastRec{urow * row_bytes, prev_irow * row_bytes, W.e[en.y].r, W.regu[en.ul], W.regi[en.il], urow,
                              prev_irow, 0});
        if (rec_src) src.push_back(s + W.e[en.y].x);
      }
      off[c - ck.c0] = static_cast<int32_t>(out.size());
    }
    tick.lap(3);
  });
  const double wall_p2 = wall();
  if (std::getenv("MFHIP_TIMING"))
    for (int ph = 0; ph < 4; ++ph)
      std::fprintf(stderr, "[mfhip]   fast plan %-10s %8.3f s (thread time)\n", g_fp_times.names[ph], g_fp_times.ns[ph] * 1e-9);
  // concatenate: chunks are in block order, and in cell order inside a block
  std::vector<int64_t> blk_total(nblk, 0), ck_base(chunks.size());
  for (size_t x = 0; x < chunks.size(); ++x) {
    ck_base[x] = blk_total[chunks[x].bx];
    blk_total[chunks[x].bx] += static_cast<int64_t>(chunks[x].out.size());
    pads[chunks[x].bx] += chunks[x].pads;
  }
  int64_t total = 0, cells = 0;
  for (int64_t bx = 0; bx < nblk; ++bx) {
    fp.rec_base[blocks[bx]] = total;
    fp.cell_base[blocks[bx]] = cells;
    total += blk_total[bx];
    cells += static_cast<int64_t>(fp.Gb[blocks[bx]]) * fp.Gb[blocks[bx]] + 1;
    fp.pads += pads[bx];
  }
  resize_huge(fp.recs, total);
  fp.cell_off.assign(cells, 0);
  if (rec_src) rec_src->resize(total);
  parallel_tasks(static_cast<int64_t>(chunks.size()), [&](int64_t x) {
    Chunk2& ck = chunks[x];
    const int64_t b = blocks[ck.bx];
    std::copy(ck.out.begin(), ck.out.end(), fp.recs.begin() + fp.rec_base[b] + ck_base[x]);
    if (rec_src) std::copy(ck.src.begin(), ck.src.end(), rec_src->begin() + fp.rec_base[b] + ck_base[x]);
    for (int64_t c = ck.c0; c < ck.c1; ++c)
      fp.cell_off[fp.cell_base[b] + c + 1] = static_cast<int32_t>(ck_base[x] + ck.off[c - ck.c0]);
    std::vector<FastRec>().swap(ck.out);
    std::vector<int64_t>().swap(ck.src);
  });
  using Works = std::vector<BlockWork>;
  fp.scratch = std::shared_ptr<void>(new Works(std::move(work)), [](void* p) { delete static_cast<Works*>(p); });
  if (std::getenv("MFHIP_TIMING"))
    std::fprintf(stderr, "[mfhip]   fast plan wall: blocks %.3f s, emit %.3f s, gather %.3f s (%zu emit chunks)\n", wall_p1,
                 wall_p2 - wall_p1, wall() - wall_p2, chunks.size());
}

namespace {
// MFHIP_DEBUG_PLAN: why cells were not given the single-run path (stderr, per build).
const bool g_plan_debug = std::getenv("MFHIP_DEBUG_PLAN") != nullptr;
std::atomic<int64_t> g_not_single[8];
struct SubCell { int32_t len; int64_t beg; int32_t j, g, t; };
// The non-empty cells of every sub-step (sm, t) of this shard's rating blocks, longest first.
std::vector<std::vector<SubCell>> collect_subs(const FastPlan& fp, int32_t nb, int32_t c, int32_t shard) {
  using Cell = SubCell;
  const int32_t G = fp.G;
  const int64_t nsub = static_cast<int64_t>(nb) * G;
  std::vector<std::vector<Cell>> subs(nsub);
  parallel_tasks(nsub, [&](int64_t x) {
    const int32_t sm = static_cast<int32_t>(x / G), t = static_cast<int32_t>(x % G);
    auto& cells = subs[x];
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j, q = (p + sm) % nb;
      const int64_t b = static_cast<int64_t>(p) * nb + q;
      if (fp.cell_base[b] < 0) continue;
      const int32_t* off = fp.cell_off.data() + fp.cell_base[b];
      for (int32_t g = 0; g < G; ++g) {
        const int64_t cb = static_cast<int64_t>(t) * G + g;
        const int32_t len = off[cb + 1] - off[cb];
        if (len > 0) cells.push_back(Cell{len, fp.rec_base[b] + off[cb], j, g, t});
      }
    }
    std::stable_sort(cells.begin(), cells.end(), [](const Cell& a, const Cell& b2) { return a.len > b2.len; });
  });
  return subs;
}

// The non-empty cells of every superstep sm of this shard's rating blocks (per-block G), in
// (j, g, t) order.
std::vector<std::vector<SubCell>> collect_supersteps(const FastPlan& fp, int32_t nb, int32_t c, int32_t shard) {
  std::vector<std::vector<SubCell>> subs(nb);
  parallel_tasks(nb, [&](int64_t sm) {
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j, q = static_cast<int32_t>((p + sm) % nb);
      const int64_t b = static_cast<int64_t>(p) * nb + q;
      if (fp.cell_base[b] < 0) continue;
      const int32_t G = fp.Gb[b];
      const int32_t* off = fp.cell_off.data() + fp.cell_base[b];
      for (int32_t g = 0; g < G; ++g)
        for (int32_t t = 0; t < G; ++t) {
          const int64_t cb = static_cast<int64_t>(t) * G + g;
          const int32_t len = off[cb + 1] - off[cb];
          if (len > 0) subs[sm].push_back(SubCell{len, fp.rec_base[b] + off[cb], j, g, t});
        }
    }
  });
  return subs;
}
}  // namespace

// Pair schedule (kernels_pair.hip): each cell's record sequence, in order, cut into steps of
// two consecutive records A, B with distinct users (a no-op B where the next record repeats
// A's user).  Per step the record names the rows to load (kOffOOB where a row is forwarded in
// registers or the record is a no-op) and to store (an item row only where its run ends),
// and how A's user row is forwarded: from the previous step's A or B when that was the
// record just before A.
void build_pair_plan(PairPlan& pp, const FastPlan& fp, int32_t nb, int32_t c, int32_t shard, int32_t k,
                     bool substep_waves, const std::vector<int32_t>* cell_pairs) {
  using Cell = SubCell;
  pp = PairPlan();
  const auto subs = substep_waves ? collect_subs(fp, nb, c, shard) : collect_supersteps(fp, nb, c, shard);
  const int64_t nsub = static_cast<int64_t>(subs.size());
  auto item_of = [](const FastRec& f) { return f.i & ~kPadBit; };
  auto is_pad = [](const FastRec& f) { return (f.i & kPadBit) != 0; };
  auto pairs_of = [](const FastRec* f, int64_t len) {
    int32_t n = 0;
    for (int64_t x = 0; x < len; ++n) x += (x + 1 < len && f[x + 1].u != f[x].u) ? 2 : 1;
    return n;
  };
  // cells in wave order (sub-step / superstep major) and their sub-step; the work below runs
  // over chunks of cells
  pp.sub_off.assign(nsub + 1, 0);
  for (int64_t x = 0; x < nsub; ++x) pp.sub_off[x + 1] = pp.sub_off[x] + static_cast<int64_t>(subs[x].size());
  const int64_t ncells = pp.sub_off[nsub];
  std::vector<const Cell*> cellv(ncells);
  std::vector<int32_t> cell_sx(ncells);
  for (int64_t x = 0; x < nsub; ++x)
    for (size_t y = 0; y < subs[x].size(); ++y) {
      cellv[pp.sub_off[x] + y] = &subs[x][y];
      cell_sx[pp.sub_off[x] + y] = static_cast<int32_t>(x);
    }
  constexpr int64_t kCellChunk = 2048;
  const int64_t nchunks = (ncells + kCellChunk - 1) / kCellChunk;
  // each wave's cell, indexed like fp.cell_off
  pp.wave_cell.resize(ncells);
  for (int64_t y = 0; y < ncells; ++y) {
    const Cell& cl = *cellv[y];
    const int64_t sm = substep_waves ? cell_sx[y] / fp.G : cell_sx[y];
    const int32_t p = shard * c + cl.j;
    const int64_t b = static_cast<int64_t>(p) * nb + (p + sm) % nb;
    pp.wave_cell[y] = fp.cell_base[b] + static_cast<int64_t>(cl.t) * fp.Gb[b] + cl.g;
  }
  std::vector<int32_t> npair(ncells);
  if (cell_pairs)
    for (int64_t y = 0; y < ncells; ++y) npair[y] = (*cell_pairs)[pp.wave_cell[y]];
  else
    parallel_tasks(nchunks, [&](int64_t ch) {
      for (int64_t y = ch * kCellChunk; y < std::min(ncells, (ch + 1) * kCellChunk); ++y)
        npair[y] = pairs_of(fp.recs.data() + cellv[y]->beg, cellv[y]->len);
    });
  pp.waves.resize(ncells);
  int64_t total = 0;
  for (int64_t y = 0; y < ncells; ++y) {
    pp.waves[y] = WaveDesc{total, npair[y], kWaveGeneric};
    total += npair[y];
  }
  if (!cell_pairs) resize_huge(pp.recs, total);
  std::vector<int64_t> cell_noops(ncells, 0);
  std::vector<double> cell_bytes(ncells, 0.0);  // bytes the kernel requests for each cell
  const double row_bytes = 4.0 * k;
  parallel_tasks(cell_pairs ? 0 : nchunks, [&](int64_t ch) {
    for (int64_t w_this = ch * kCellChunk; w_this < std::min(ncells, (ch + 1) * kCellChunk); ++w_this) {
      const Cell& cl = *cellv[w_this];
      int64_t& noop = cell_noops[w_this];
      PairRec* const first = pp.recs.data() + pp.waves[w_this].base;
      PairRec* out = first;
      const FastRec* f = fp.recs.data() + cl.beg;
      const int64_t len = cl.len;
      uint32_t last_u = kOffOOB;  // user offset of the record just before A (real records only)
      uint32_t last_half = 0;     // kPairFwdA / kPairFwdB: the half that record was in
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
        // the item row whose run may end after this step: B's if B exists, else A's
        const FastRec* tail = &a;
        if (has_b) {
          const FastRec& b = f[x + 1];
          tail = &b;
          if (item_of(b) != item_of(a)) {  // split: A's run ends at A, B starts a run
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
      // one item run (no split, every later pair keeps the item): the kernel's lean path
      bool single = first[0].ia != kOffOOB && !(first[0].flags & (kPairKeepQ | kPairSplit));
      int why = single ? 0 : 1;
      for (const PairRec* r = first; single && r < out; ++r) {
        single = !(r->flags & kPairSplit) && (r == first || (r->flags & kPairKeepQ)) && r->ub == r->sb &&
                 (r + 1 < out ? r->si == kOffOOB : r->si == first[0].ia);
        if (!single) why = (r->flags & kPairSplit) ? 2 : !(r == first || (r->flags & kPairKeepQ)) ? 3 : r->ub != r->sb ? 4 : 5;
      }
      // the lean path prefetches pair_ring pairs ahead: a user row it loads must have been
      // stored by an earlier pair at least that far back
      if (single) {  // the stores of the previous pair_ring - 1 pairs, as a ring
        const int kR = pair_ring(pair_kpl(k)) - 1;
        uint32_t ring[kPairPlanRing][2];
        for (auto& rr : ring) rr[0] = rr[1] = kOffOOB;
        for (const PairRec* r = first; single && r < out; ++r) {
          const int64_t j = r - first;
          for (uint32_t off : {r->ua, r->ub}) {
            if (off == kOffOOB) continue;
            for (int y = 0; y < kR; ++y)
              if (ring[y][0] == off || ring[y][1] == off) { single = false; why = 6; }
          }
          if (kR > 0) {
            ring[j % kR][0] = r->sa;
            ring[j % kR][1] = r->sb;
          }
        }
      }
      bool fwd = false;  // A rows forwarded from the previous pair: the lean path's FWD instance
      for (const PairRec* r = first; single && r < out; ++r) fwd = fwd || (r->flags & (kPairFwdA | kPairFwdB));
      if (single) pp.waves[w_this].cells = fwd ? kWaveSingleRunFwd : kWaveSingleRun;
      else if (g_plan_debug) g_not_single[why]++;
      // what the kernel requests: the 64-B record of every pair and every row access with an
      // in-range offset (the lean path: the item row once in, once out, B's row stored where
      // it was loaded from)
      int64_t rows = 0;
      for (const PairRec* r = first; r < out; ++r) {
        if (single) {
          rows += (r->ua != kOffOOB) + 2 * (r->ub != kOffOOB) + (r->sa != kOffOOB);
        } else {
          for (uint32_t off : {r->ua, r->ub, r->ia, r->ib, r->sa, r->sb, r->sia, r->si}) rows += off != kOffOOB;
        }
      }
      if (single && out > first) rows += 2;
      cell_bytes[w_this] = 64.0 * static_cast<double>(out - first) + row_bytes * static_cast<double>(rows);
    }
  });
  std::vector<double> sub_bytes(nsub, 0.0);  // per sub-step, summed in cell order
  for (int64_t y = 0; y < ncells; ++y) {
    pp.noop_halves += cell_noops[y];
    sub_bytes[cell_sx[y]] += cell_bytes[y];
  }
  pp.sm_bytes.assign(nb, 0.0);
  for (int64_t x = 0; x < nsub; ++x) pp.sm_bytes[substep_waves ? x / fp.G : x] += sub_bytes[x];
  if (g_plan_debug) {
    std::fprintf(stderr, "[mfhip] pair plan: cells not single-run: first %lld split %lld item-change %lld "
                 "B-store %lld item-store %lld hazard %lld\n", (long long)g_not_single[1].load(),
                 (long long)g_not_single[2].load(), (long long)g_not_single[3].load(), (long long)g_not_single[4].load(),
                 (long long)g_not_single[5].load(), (long long)g_not_single[6].load());
    for (auto& x : g_not_single) x = 0;
  }
  // systolic tables: superstep sm's waves are (j, g), j-major; wave (j, g) owns G_j cells
  pp.sys_off.assign(nb + 1, 0);
  pp.sys_block_off.assign(static_cast<size_t>(nb) * (c + 1), 0);
  std::vector<std::vector<int64_t>> wave0(nb, std::vector<int64_t>(c, 0));  // sys_waves index of (sm, j, g=0)
  for (int32_t sm = 0; sm < nb; ++sm) {
    pp.sys_off[sm] = static_cast<int64_t>(pp.sys_waves.size());
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j, q = (p + sm) % nb;
      const int64_t b = static_cast<int64_t>(p) * nb + q;
      const int32_t G = fp.cell_base[b] < 0 ? 0 : fp.Gb[b];
      const int64_t w0 = static_cast<int64_t>(pp.sys_waves.size());
      wave0[sm][j] = w0;
      pp.sys_block_off[static_cast<size_t>(sm) * (c + 1) + j] = w0 - pp.sys_off[sm];
      for (int32_t g = 0; g < G; ++g) {
        const int32_t nbr = static_cast<int32_t>(w0 - pp.sys_off[sm]) + (g + 1 == G ? 0 : g + 1);
        pp.sys_waves.push_back(SysWave{static_cast<int64_t>(pp.sys.size()), G, nbr});
        pp.sys.resize(pp.sys.size() + G, WaveDesc{0, 0, kWaveGeneric});
      }
    }
  }
  pp.sys_off[nb] = static_cast<int64_t>(pp.sys_waves.size());
  for (int32_t sm = 0; sm < nb; ++sm)
    pp.sys_block_off[static_cast<size_t>(sm) * (c + 1) + c] = pp.sys_off[sm + 1] - pp.sys_off[sm];
  pp.wave_sys.assign(ncells, -1);
  for (int64_t x = 0; x < nsub; ++x) {
    const int64_t sm = substep_waves ? x / fp.G : x;
    int64_t w = pp.sub_off[x];
    for (const Cell& cl : subs[x]) {
      const SysWave& sw = pp.sys_waves[wave0[sm][cl.j] + cl.g];
      pp.wave_sys[w] = sw.cell0 + cl.t;
      pp.sys[sw.cell0 + cl.t] = pp.waves[w++];
    }
  }
}

void lpt_assign(const std::vector<int64_t>& load, int32_t G, std::vector<int32_t>& group) { lpt_groups(load, G, group); }

std::vector<int32_t> choose_block_groups(const RatingBlocks& rb, const SideLayout& I, int32_t c, int32_t shard,
                                         int32_t waves, int32_t split_run, double cell_ns, double run_ns) {
  const int32_t nb = rb.n_blocks;
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  std::vector<int64_t> size(nb2, 0), top(nb2, 0);  // ratings, ratings of the most rated item
  parallel_tasks(nb2, [&](int64_t b) {
    const int32_t p = static_cast<int32_t>(b / nb), q = static_cast<int32_t>(b % nb);
    if (p < shard * c || p >= (shard + 1) * c || rb.size(b) == 0) return;
    const int64_t ib = I.block_start[q], ni = I.block_start[q + 1] - ib;
    std::vector<int32_t> cnt(ni, 0);
    int32_t mx = 0;
    for (int64_t x = rb.start[b]; x < rb.start[b + 1]; ++x) mx = std::max(mx, ++cnt[rb.irow[x] - ib]);
    size[b] = rb.size(b);
    top[b] = split_run > 0 ? std::min(mx, split_run) : mx;
  });
  return choose_block_groups(size, top, nb, c, shard, waves, cell_ns, run_ns);
}

std::vector<int32_t> choose_block_groups(const std::vector<int64_t>& size, const std::vector<int64_t>& top, int32_t nb,
                                         int32_t c, int32_t shard, int32_t waves, double cell_ns, double run_ns) {
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  std::vector<int32_t> Gb(nb2, 0);
  double pair_ns = kSysPairNs;
  if (const char* v = exp_knob("MFHIP_SYS_MODEL"))  // tuning knob: "cell_ns,pair_ns,run_pair_ns"
    std::sscanf(v, "%lf,%lf,%lf", &cell_ns, &pair_ns, &run_ns);
  auto wave_ns = [&](int64_t b, int32_t G) {
    const double per_group = static_cast<double>(size[b]) / G;
    return G * cell_ns + std::max(per_group / 2 * pair_ns, static_cast<double>(top[b]) / 2 * run_ns);
  };
  constexpr int32_t kStep = 8, kMaxG = 1024;  // G = 4 or 2 measured the same (profiles/r03_placement_NFLX.txt)
  for (int32_t sm = 0; sm < nb; ++sm) {
    std::vector<int64_t> bs;
    for (int32_t j = 0; j < c; ++j) {
      const int32_t p = shard * c + j;
      const int64_t b = static_cast<int64_t>(p) * nb + (p + sm) % nb;
      if (size[b] > 0) bs.push_back(b);
    }
    if (bs.empty()) continue;
    // smallest G (multiple of kStep) whose modelled wave time is <= T, or 0 if none
    auto gmin = [&](int64_t b, double T) {
      for (int32_t G = kStep; G <= kMaxG; G += kStep)
        if (wave_ns(b, G) <= T) return G;
      return 0;
    };
    double lo = 0, hi = 0;
    for (int64_t b : bs) hi = std::max(hi, wave_ns(b, kStep));
    for (int it = 0; it < 60; ++it) {
      const double T = 0.5 * (lo + hi);
      int64_t sum = 0;
      bool ok = true;
      for (int64_t b : bs) {
        const int32_t G = gmin(b, T);
        ok = ok && G > 0;
        sum += G;
      }
      if (ok && sum <= waves) hi = T;
      else lo = T;
    }
    for (int64_t b : bs) Gb[b] = std::max(gmin(b, hi), kStep);
  }
  return Gb;
}

}  // namespace mfhip
