// Host side of one online micro-batch upload (mfhip.cpp online_update): the batch's three arrays
// (user ids, item ids, ratings: 16 B per rating) copied into the pinned upload buffer by host
// threads, then one H2D copy.  Measures, on the box's CPU: thread spawn per call (parallel_for as
// of round 6) against a persistent worker pool (common.hpp WorkerPool), the copy itself at 4-16
// workers, and the 16-MB DMA.
//
//   hipcc -O3 -std=c++17 -pthread -o host_stage host_stage.cpp && ./host_stage
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t) { return std::chrono::duration<double, std::micro>(clk::now() - t).count(); }

// the pool under test: workers park on a condition variable; the caller runs share 0
struct Pool {
  explicit Pool(int n) {
    for (int t = 1; t < n; ++t) th.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
      ++gen;
    }
    cv.notify_all();
    for (auto& x : th) x.join();
  }
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return gen != seen; });
      if (stop) return;
      seen = gen;
      const std::function<void(int)>* f = job;
      const int w = width;
      lk.unlock();
      if (t < w) (*f)(t);
      if (left.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(m);
        done.notify_one();
      }
    }
  }
  void run(int w, const std::function<void(int)>& f) {
    {
      std::lock_guard<std::mutex> g(m);
      job = &f;
      width = w;
      left.store(static_cast<int>(th.size()));
      ++gen;
    }
    cv.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return left.load() == 0; });
  }
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv, done;
  uint64_t gen = 0;
  const std::function<void(int)>* job = nullptr;
  int width = 0;
  std::atomic<int> left{0};
  bool stop = false;
};

static void spawn_run(int w, const std::function<void(int)>& f) {
  std::vector<std::thread> th;
  for (int t = 1; t < w; ++t) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

int main() {
  const int64_t n = 1000000;
  std::vector<int32_t> u(n), i(n);
  std::vector<double> r(n);
  for (int64_t x = 0; x < n; ++x) { u[x] = static_cast<int32_t>(x * 7); i[x] = static_cast<int32_t>(x * 3); r[x] = 1.0 + x % 5; }
  void* pin = nullptr;
  CK(hipHostMalloc(&pin, n * 16, hipHostMallocDefault));
  void* dev = nullptr;
  CK(hipMalloc(&dev, n * 16));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::setvbuf(stdout, nullptr, _IOLBF, 0);
  std::printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
  auto copy = [&](int w) {
    return [&, w](int t) {
      const int64_t c = (n + w - 1) / w, lo = t * c, hi = std::min(n, lo + c);
      if (lo >= hi) return;
      uint32_t* ur = static_cast<uint32_t*>(pin);
      std::memcpy(ur + lo, u.data() + lo, (hi - lo) * 4);
      std::memcpy(ur + n + lo, i.data() + lo, (hi - lo) * 4);
      std::memcpy(reinterpret_cast<double*>(ur + 2 * n) + lo, r.data() + lo, (hi - lo) * 8);
    };
  };
  for (int w : {1, 4, 8, 16}) {
    Pool pool(w);
    const auto job = copy(w);
    const std::function<void(int)> empty = [](int) {};
    for (int mode = 0; mode < 4; ++mode) {
      std::vector<double> ts;
      for (int rep = 0; rep < 40; ++rep) {
        const auto t0 = clk::now();
        if (mode == 0) spawn_run(w, empty);
        else if (mode == 1) pool.run(w, empty);
        else if (mode == 2) spawn_run(w, job);
        else pool.run(w, job);
        ts.push_back(us_since(t0));
      }
      std::sort(ts.begin(), ts.end());
      static const char* names[] = {"spawn, empty", "pool,  empty", "spawn, 16-MB copy", "pool,  16-MB copy"};
      std::printf("%2d workers  %-18s median %8.1f us  min %8.1f us\n", w, names[mode], ts[ts.size() / 2], ts[0]);
    }
  }
  for (int rep = 0; rep < 5; ++rep) {
    const auto t0 = clk::now();
    CK(hipMemcpyAsync(dev, pin, n * 16, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    std::printf("H2D 16 MB pinned: %.1f us\n", us_since(t0));
  }
  return 0;
}
