// Host-only probe of the fast pair plan (no GPU): reads ratings written by tools/probe/dump_ratings.py,
// builds the systolic plan exactly as mf_dsgd_prepare does on one device, and prints per-superstep
// wave statistics.  Build: make -C tools/probe
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "plan.hpp"

using namespace mfhip;

static double lap() {
  static auto t = std::chrono::steady_clock::now();
  const auto now = std::chrono::steady_clock::now();
  const double d = std::chrono::duration<double>(now - t).count();
  t = now;
  return d;
}

template <class T>
std::vector<T> load(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) { std::perror(path); std::exit(1); }
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f) / sizeof(T);
  std::fseek(f, 0, SEEK_SET);
  std::vector<T> v(n);
  if (std::fread(v.data(), sizeof(T), n, f) != static_cast<size_t>(n)) std::exit(1);
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  const int nb = argc > 2 ? std::atoi(argv[2]) : 8, k = argc > 3 ? std::atoi(argv[3]) : 128;
  const int waves = argc > 4 ? std::atoi(argv[4]) : 1024;
  char p[512];
  std::snprintf(p, sizeof p, "%s/probe_u.bin", dir); auto u = load<int32_t>(p);
  std::snprintf(p, sizeof p, "%s/probe_i.bin", dir); auto i = load<int32_t>(p);
  std::snprintf(p, sizeof p, "%s/probe_r.bin", dir); auto r = load<double>(p);
  const int64_t n = static_cast<int64_t>(u.size());
  lap();
  SideLayout U, I;
  const int64_t pseed = std::getenv("PROBE_SEED") ? std::atoll(std::getenv("PROBE_SEED")) : 0;
  build_side(U, u.data(), n, nb, pseed, true);
  build_side(I, i.data(), n, nb, pseed, true);
  std::printf("build_side x2 %.3f s\n", lap());
  RatingBlocks rb;
  build_rating_blocks(rb, U, I, u.data(), i.data(), r.data(), n, 0, nb, false);
  std::printf("rating blocks %.3f s\n", lap());
  if (argc > 5 && std::string(argv[5]) == "scale") {
    // Strong-scaling model of the systolic sweep on G GPUs (rank mode, n = nb blocks, c = nb / G
    // user blocks per rank, `waves` resident waves per GPU): per rank and superstep the busiest
    // wave's single-run / mixed pairs and cells, from the plan mf_dsgd_prepare builds for that
    // rank.  Printed per G; tools/scaling_model.py turns it into times.
    for (int G = 1; G <= nb; G *= 2) {
      if (nb % G) continue;
      const int c = nb / G;
      std::vector<int32_t> Gall(static_cast<size_t>(nb) * nb, 0);
      for (int g = 0; g < G; ++g) {
        const auto gb = choose_block_groups(rb, I, c, g, waves, 0, sys_cell_ns(k), sys_run_pair_ns(k));
        for (size_t b = 0; b < gb.size(); ++b) if (gb[b] > 0) Gall[b] = gb[b];
      }
      FastPlan fp;
      build_fast_plan(fp, rb, U, I, 128, k, 1.0, 0 * 0x9E3779B97F4A7C15ULL + 1, static_cast<uint32_t>(U.rows()),
                      nullptr, pair_window(k), &Gall);
      for (int g = 0; g < G; ++g) {
        PairPlan pp;
        build_pair_plan(pp, fp, nb, c, g, k, false);
        for (int sm = 0; sm < nb; ++sm) {
          // every wave of this rank's superstep: cells, single-run pairs, mixed pairs
          for (int64_t w = pp.sys_off[sm]; w < pp.sys_off[sm + 1]; ++w) {
            const SysWave& sw = pp.sys_waves[w];
            int64_t runp = 0, mixp = 0, cells = 0;
            for (int t = 0; t < sw.G; ++t) {
              const WaveDesc& d = pp.sys[sw.cell0 + t];
              if (d.steps == 0) continue;
              ++cells;
              ((d.cells == kWaveSingleRun || d.cells == kWaveSingleRunFwd) ? runp : mixp) += d.steps;
            }
            std::printf("SCALE G %d rank %d sm %d wave %lld cells %lld run %lld mix %lld\n", G, g, sm,
                        (long long)(w - pp.sys_off[sm]), (long long)cells, (long long)runp, (long long)mixp);
          }
        }
      }
      std::fflush(stdout);
    }
    return 0;
  }
  const auto Gb = choose_block_groups(rb, I, nb, 0, waves, 0, sys_cell_ns(k), sys_run_pair_ns(k));
  std::printf("block groups %.3f s\n", lap());
  FastPlan fp;
  build_fast_plan(fp, rb, U, I, 128, k, 1.0, 0 * 0x9E3779B97F4A7C15ULL + 1, static_cast<uint32_t>(U.rows()), nullptr,
                  pair_window(k), &Gb);
  std::printf("fast plan %.3f s\n", lap());
  PairPlan pp;
  build_pair_plan(pp, fp, nb, nb, 0, k, false);
  std::printf("pair plan %.3f s\n", lap());
  std::printf("pads %lld noop halves %lld pairs %zu\n", (long long)fp.pads, (long long)pp.noop_halves, pp.recs.size());
  {  // out-of-range operations per pair step, generic vs single-run waves
    int64_t gen_pairs = 0, gen_oob[8] = {0}, run_pairs = 0, run_oob = 0;
    for (const WaveDesc& w : pp.waves)
      for (int64_t x = w.base; x < w.base + w.steps; ++x) {
        const PairRec& r = pp.recs[x];
        if (w.cells == kWaveSingleRun || w.cells == kWaveSingleRunFwd) {
          ++run_pairs;
          run_oob += (r.ua == kOffOOB) + (r.ub == kOffOOB) + (r.sa == kOffOOB) + (r.sb == kOffOOB);
        } else {
          ++gen_pairs;
          const uint32_t o[8] = {r.ua, r.ub, r.ia, r.ib, r.sa, r.sb, r.sia, r.si};
          for (int y = 0; y < 8; ++y) gen_oob[y] += o[y] == kOffOOB;
        }
      }
    std::printf("generic pairs %lld: out-of-range ua %.2f ub %.2f ia %.2f ib %.2f sa %.2f sb %.2f sia %.2f si %.2f\n",
                (long long)gen_pairs, gen_oob[0] / double(gen_pairs), gen_oob[1] / double(gen_pairs),
                gen_oob[2] / double(gen_pairs), gen_oob[3] / double(gen_pairs), gen_oob[4] / double(gen_pairs),
                gen_oob[5] / double(gen_pairs), gen_oob[6] / double(gen_pairs), gen_oob[7] / double(gen_pairs));
    std::printf("single-run pairs %lld: out-of-range per pair %.2f of 4\n", (long long)run_pairs,
                run_oob / double(std::max<int64_t>(run_pairs, 1)));
    int64_t fwd_pairs = 0, fwd_cells = 0, run_cells = 0, pad_b = 0;
    for (const WaveDesc& w : pp.waves) {
      if (w.cells != kWaveSingleRun && w.cells != kWaveSingleRunFwd) continue;
      ++run_cells;
      bool any = false;
      for (int64_t x = w.base; x < w.base + w.steps; ++x) {
        const PairRec& r = pp.recs[x];
        if (r.flags & (kPairFwdA | kPairFwdB)) { ++fwd_pairs; any = true; }
        pad_b += r.ub == kOffOOB;
      }
      fwd_cells += any;
    }
    std::printf("single-run cells %lld: with forwarding %lld; pairs with forwarding %lld, with a no-op B %lld\n",
                (long long)run_cells, (long long)fwd_cells, (long long)fwd_pairs, (long long)pad_b);
    // blocks of BP pairs of single-run cells: forwarding inside a block, at its first pair, and
    // users shared with the previous block (a row prefetched one block ahead would be stale)
    for (int BP : {4, 7, 8}) {
      int64_t blocks = 0, fwd_in = 0, fwd_first = 0, shared_prev = 0, shared_rows = 0, clean = 0;
      for (const WaveDesc& w : pp.waves) {
        if (w.cells != kWaveSingleRun && w.cells != kWaveSingleRunFwd) continue;
        std::vector<uint32_t> prev;
        for (int64_t x0 = w.base; x0 < w.base + w.steps; x0 += BP) {
          ++blocks;
          std::vector<uint32_t> cur;
          bool fi = false, ff = false;
          for (int64_t x = x0; x < std::min<int64_t>(x0 + BP, w.base + w.steps); ++x) {
            const PairRec& r = pp.recs[x];
            if (r.flags & (kPairFwdA | kPairFwdB)) (x == x0 ? ff : fi) = true;
            if (r.sa != kOffOOB) cur.push_back(r.sa);
            if (r.sb != kOffOOB) cur.push_back(r.sb);
          }
          int sh = 0;
          for (uint32_t o : cur)
            for (uint32_t q : prev) sh += o == q;
          fwd_in += fi;
          fwd_first += ff;
          shared_prev += sh > 0;
          shared_rows += sh;
          clean += !fi && !ff && sh == 0;
          prev = cur;
        }
      }
      std::printf("single-run blocks of %d pairs: %lld, forwarding inside %lld, at the first pair %lld, sharing a user "
                  "with the previous block %lld (%lld rows), clean %lld (%.1f%%)\n", BP, (long long)blocks,
                  (long long)fwd_in, (long long)fwd_first, (long long)shared_prev, (long long)shared_rows,
                  (long long)clean, 100.0 * clean / std::max<int64_t>(blocks, 1));
    }
  }
  {  // fingerprint of the plans (FNV-1a over the records, cell offsets and pair records)
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
      const unsigned char* c = static_cast<const unsigned char*>(p);
      for (size_t x = 0; x < n; ++x) { h ^= c[x]; h *= 1099511628211ull; }
    };
    mix(fp.recs.data(), fp.recs.size() * sizeof(FastRec));
    mix(fp.cell_off.data(), fp.cell_off.size() * 4);
    mix(pp.recs.data(), pp.recs.size() * sizeof(PairRec));
    mix(pp.sys.data(), pp.sys.size() * sizeof(WaveDesc));
    std::printf("plan fingerprint %016llx\n", (unsigned long long)h);
  }
  for (int sm = 0; sm < nb; ++sm) {
    int64_t maxp = 0, maxw = -1, singles = 0, waves_sm = pp.sys_off[sm + 1] - pp.sys_off[sm];
    for (int64_t w = pp.sys_off[sm]; w < pp.sys_off[sm + 1]; ++w) {
      const SysWave& sw = pp.sys_waves[w];
      int64_t pairs = 0;
      for (int t = 0; t < sw.G; ++t) { pairs += pp.sys[sw.cell0 + t].steps; singles += pp.sys[sw.cell0 + t].cells >= kWaveSingleRun; }
      if (pairs > maxp) { maxp = pairs; maxw = w; }
    }
    int64_t ms = 0;
    const SysWave& sw = pp.sys_waves[maxw];
    for (int t = 0; t < sw.G; ++t) ms += pp.sys[sw.cell0 + t].cells >= kWaveSingleRun;
    std::printf("sm %d waves %lld single cells %lld busiest wave %lld: G %d pairs %lld single cells %lld\n", sm,
                (long long)waves_sm, (long long)singles, (long long)(maxw - pp.sys_off[sm]), sw.G, (long long)maxp,
                (long long)ms);
  }
  return 0;
}
