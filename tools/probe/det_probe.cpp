// Host-only probe of the deterministic sweep's per-superstep host build (build_det_step, no GPU):
// reads ratings written by tools/probe/dump_ratings.py, builds the blocking and the det layout as
// mf_dsgd_prepare does on one device, and times build_det_step for a few supersteps (prints an
// FNV digest of the output so that variants of the build can be checked for equality).
// Build: make -C tools/probe det_probe
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "plan.hpp"

using namespace mfhip;

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
  const int nb = argc > 2 ? std::atoi(argv[2]) : 8, waves = argc > 3 ? std::atoi(argv[3]) : 2048;
  const int steps = argc > 4 ? std::atoi(argv[4]) : 3;
  char p[512];
  std::snprintf(p, sizeof p, "%s/probe_u.bin", dir); auto u = load<int32_t>(p);
  std::snprintf(p, sizeof p, "%s/probe_i.bin", dir); auto i = load<int32_t>(p);
  std::snprintf(p, sizeof p, "%s/probe_r.bin", dir); auto r = load<double>(p);
  const int64_t n = static_cast<int64_t>(u.size());
  SideLayout U, I;
  build_side(U, u.data(), n, nb, 0, true);
  build_side(I, i.data(), n, nb, 0, true);
  RatingBlocks rb;
  build_rating_blocks(rb, U, I, u.data(), i.data(), r.data(), n, 0, nb, true);
  rb.det_aos.resize(rb.start.back());  // as prepare_det_sweep
  for (int64_t x = 0; x < rb.start.back(); ++x) rb.det_aos[x] = DetEntry{rb.urow[x], rb.irow[x], rb.r[x]};
  DetSweepLayout L;
  build_det_layout(L, rb, U, I, nb, 0, waves);
  for (int s = 1; s <= steps; ++s) {
    std::vector<int64_t> blocks, seeds;
    int64_t ne = 0, nw = 0;
    for (int32_t pq = 0; pq < nb; ++pq) {
      const int64_t b = static_cast<int64_t>(pq) * nb + (pq + s - 1) % nb;
      if (rb.size(b) == 0) continue;
      blocks.push_back(b);
      seeds.push_back(static_cast<int64_t>(0 ^ static_cast<int32_t>(b)) ^ 42);
      ne += rb.size(b);
      nw += L.block_waves[b];
    }
    static std::vector<DetWave> w;
    static std::vector<uint32_t> ou, oi, oq;
    static std::vector<double> orr;  // kept across supersteps, as the pinned staging buffers are
    w.resize(nw); ou.resize(ne); oi.resize(ne); oq.resize(ne); orr.resize(ne);
    DetStepOut out{w.data(), ou.data(), oi.data(), oq.data(), orr.data()};
    const auto t0 = std::chrono::steady_clock::now();
    static DetStepScratch scratch;
    build_det_step(rb, U, I, L, blocks, seeds, true, out, &scratch);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* d, size_t bytes) {
      const unsigned char* c = static_cast<const unsigned char*>(d);
      for (size_t x = 0; x < bytes; ++x) h = (h ^ c[x]) * 1099511628211ull;
    };
    mix(w.data(), w.size() * sizeof(DetWave));
    mix(ou.data(), ne * 4); mix(oi.data(), ne * 4); mix(oq.data(), ne * 4); mix(orr.data(), ne * 8);
    static int64_t prev[5] = {0, 0, 0, 0, 0};
    double ph[5];
    for (int x = 0; x < 5; ++x) ph[x] = (det_build_phase_ns(x) - prev[x]) / 1e6, prev[x] = det_build_phase_ns(x);
    std::printf("superstep %d: %lld entries %lld waves  build %.1f ms (shuffle %.1f gather %.1f prefix %.1f scatter %.1f "
                "flags %.1f)  digest %016llx\n", s, (long long)ne, (long long)nw, dt * 1e3, ph[0], ph[1], ph[2], ph[3],
                ph[4], (unsigned long long)h);
  }
  return 0;
}
