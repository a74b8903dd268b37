// CPU check of the host worker pool behind parallel_for / parallel_tasks (csrc/common.hpp
// WorkerPool), built and run by tests/test_pool.py: every index exactly once, nested calls,
// two threads calling at once, an exception from a share (the caller's and a worker's), and a
// forked child (the pool's threads do not exist there).  Prints "ok" and exits 0 on success.
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <vector>

#include "common.hpp"

using namespace mfhip;

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      std::_Exit(1);                                              \
    }                                                             \
  } while (0)

static void cover(int64_t n, int workers) {
  std::vector<std::atomic<int>> hit(static_cast<size_t>(n));
  for (auto& h : hit) h = 0;
  parallel_for(n, [&](int64_t b, int64_t e, int) { for (int64_t x = b; x < e; ++x) hit[x]++; }, workers, 1);
  for (auto& h : hit) CHECK(h.load() == 1);
  for (auto& h : hit) h = 0;
  parallel_tasks(n, [&](int64_t x) { hit[x]++; }, workers);
  for (auto& h : hit) CHECK(h.load() == 1);
}

int main() {
  for (int w : {1, 2, 3, 8, 16}) cover(1000, w);
  cover(7, 16);  // fewer items than workers
  for (int rep = 0; rep < 200; ++rep) cover(64, 8);  // back-to-back jobs

  // nested: a parallel_for inside a share (from the caller's share and from the workers')
  {
    std::atomic<int64_t> sum{0};
    parallel_for(64, [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x)
        parallel_for(100, [&](int64_t b2, int64_t e2, int) { sum += e2 - b2; }, 4, 1);
    }, 8, 1);
    CHECK(sum.load() == 6400);
  }

  // two threads calling at once: one gets the pool, the other starts threads of its own
  {
    std::atomic<int64_t> a{0}, b{0};
    std::thread t1([&] { for (int r = 0; r < 100; ++r) parallel_for(1000, [&](int64_t x, int64_t y, int) { a += y - x; }, 8, 1); });
    std::thread t2([&] { for (int r = 0; r < 100; ++r) parallel_for(1000, [&](int64_t x, int64_t y, int) { b += y - x; }, 8, 1); });
    t1.join();
    t2.join();
    CHECK(a.load() == 100000 && b.load() == 100000);
  }

  // an exception from the caller's share reaches the caller after the workers are done
  {
    std::atomic<int> done{0};
    bool caught = false;
    try {
      parallel_for(8, [&](int64_t b, int64_t, int t) {
        if (t == 0) throw std::runtime_error("share 0");
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        done += static_cast<int>(b >= 0);
      }, 8, 1);
    } catch (const std::runtime_error&) {
      caught = true;
    }
    CHECK(caught);
    CHECK(done.load() == 7);  // every worker's share finished before the call returned
    cover(100, 8);            // and the pool still works
  }

  // a forked child: the pool's threads are not there, the child starts its own
  {
    cover(100, 8);  // the pool exists in the parent
    const pid_t pid = fork();
    if (pid == 0) {
      std::atomic<int64_t> s{0};
      parallel_for(1000, [&](int64_t x, int64_t y, int) { s += y - x; }, 8, 1);
      std::_Exit(s.load() == 1000 ? 0 : 2);
    }
    int st = 0;
    CHECK(waitpid(pid, &st, 0) == pid);
    CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
  std::printf("ok\n");
  return 0;
}
