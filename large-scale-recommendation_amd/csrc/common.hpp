// common.hpp -- status/error plumbing, device buffers and a small host thread pool.
#pragma once
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "mfhip.h"
#include "mfhip_testing.h"

namespace mfhip {

// Every API entry point catches this and converts it to a status + mf_last_error().
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] inline void fail(int code, const std::string& msg) { throw Error(code, msg); }

// The C ABI's error convention: run f, map exceptions to an MF_ERR_* status and keep the
// message for mf_last_error() (thread-local, defined in mfhip.cpp).
extern thread_local std::string g_last_error;
template <typename F>
int guarded(F&& f) {
  try {
    f();
    return MF_OK;
  } catch (const Error& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host allocation failed";
    return MF_ERR_CAPACITY;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return MF_ERR_INVALID;
  }
}

#define MF_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t _e = (call);                                                                 \
    if (_e != hipSuccess)                                                                   \
      ::mfhip::fail(MF_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e) + " at " + \
                                    __FILE__ + ":" + std::to_string(__LINE__));             \
  } while (0)

#define MF_REQUIRE(cond, msg) \
  do {                        \
    if (!(cond)) ::mfhip::fail(MF_ERR_INVALID, (msg)); \
  } while (0)

// Owning device allocation on the current device.
// Device bytes this process holds in DevBufs (live, high-water mark): mf_debug_device_bytes.
inline std::atomic<int64_t>& dev_bytes_live() { static std::atomic<int64_t> v{0}; return v; }
inline std::atomic<int64_t>& dev_bytes_peak() { static std::atomic<int64_t> v{0}; return v; }

class DevBuf {
 public:
  DevBuf() = default;
  ~DevBuf() { release(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p_(o.p_), bytes_(o.bytes_) { o.p_ = nullptr; o.bytes_ = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p_ = o.p_; bytes_ = o.bytes_; o.p_ = nullptr; o.bytes_ = 0; }
    return *this;
  }
  void alloc(size_t bytes) {
    if (bytes <= bytes_ && p_) return;
    release();
    if (bytes == 0) return;
    MF_HIP(hipMalloc(&p_, bytes));
    bytes_ = bytes;
    const int64_t now = dev_bytes_live() += static_cast<int64_t>(bytes);
    int64_t pk = dev_bytes_peak().load();
    while (now > pk && !dev_bytes_peak().compare_exchange_weak(pk, now)) {}
  }
  void release() {
    if (p_) {
      (void)hipFree(p_);
      dev_bytes_live() -= static_cast<int64_t>(bytes_);
    }
    p_ = nullptr;
    bytes_ = 0;
  }
  template <typename T> T* as() const { return static_cast<T*>(p_); }
  void* get() const { return p_; }
  size_t bytes() const { return bytes_; }

 private:
  void* p_ = nullptr;
  size_t bytes_ = 0;
};

// Rating blocks on the device (kernels_block.hip device_blocking's output, rb order).
struct DevRatingBlocks {
  DevBuf urow, irow, r;  // u32, u32, f64
  int64_t total = 0;
};

// Device scratch of online_sweep_plan (kernels_online.hip), kept across micro-batches.
struct OnlineSweepScratch {
  DevBuf ukey, wkey, wkey2, iota, ux, wx, head, start, ticket, tmp;
  DevBuf in, wbeg, uticket, err, touched;  // the batch as uploaded; wave starts, tickets, error flag, counts
  DevBuf dummy;                            // k_online_f32: a scratch ticket line per wave
  DevBuf icnt, iwave;                      // per item row: sampled update counts, own wave (-1: none)
  DevBuf soa, multi, waves;                // the f64 sweep's entry arrays, multi-item flags, wave table
  DevBuf miss;                             // the device id lookup's miss count
  // the plan's independent parts run side by side: the tickets' user sort on s2, the touched-item
  // flags on s3 (each with its own scratch), joined back into the caller's stream
  DevBuf tmp2, tmp3, iota2, iflag;
  hipStream_t s2 = nullptr, s3 = nullptr;
  hipEvent_t ev_in = nullptr, ev2 = nullptr, ev3 = nullptr;
  OnlineSweepScratch() = default;
  OnlineSweepScratch(const OnlineSweepScratch&) = delete;
  OnlineSweepScratch& operator=(const OnlineSweepScratch&) = delete;
  ~OnlineSweepScratch() {
    for (hipEvent_t e : {ev_in, ev2, ev3})
      if (e) (void)hipEventDestroy(e);
    for (hipStream_t q : {s2, s3})
      if (q) (void)hipStreamDestroy(q);
  }
  void side_streams() {  // on the current device (the caller's DeviceGuard)
    if (s2) return;
    MF_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    MF_HIP(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    for (hipEvent_t* e : {&ev_in, &ev2, &ev3}) MF_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
};

// Device scratch of det_device_build (kernels_online.hip), sized once for a shard's largest superstep.
struct DetBuildScratch {
  DevBuf ent, wkey, wkey2, ukey, ukey2, iota, wx, ux, head, start, ticket, tmp, tmp2, blocks;
  int64_t n_max = 0;
  size_t tmp_bytes = 0, tmp2_bytes = 0;
};

// Pinned host staging buffer.
class PinnedBuf {
 public:
  PinnedBuf() = default;
  ~PinnedBuf() { if (p_) (void)hipHostFree(p_); }
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  void alloc(size_t bytes) {
    if (bytes <= bytes_ && p_) return;
    if (p_) (void)hipHostFree(p_);
    p_ = nullptr;
    bytes_ = 0;
    if (bytes == 0) return;
    MF_HIP(hipHostMalloc(&p_, bytes, hipHostMallocDefault));
    bytes_ = bytes;
  }
  template <typename T> T* as() const { return static_cast<T*>(p_); }
  size_t bytes() const { return bytes_; }

 private:
  void* p_ = nullptr;
  size_t bytes_ = 0;
};

// Runtime switches.  The library reads five environment variables:
//   MFHIP_THREADS / OMP_NUM_THREADS  host workers (below);
//   MFHIP_TIMING                     prepare's phase timings on stderr;
//   MFHIP_DEBUG_PLAN                 planner diagnostics and the sweeps' error words on stderr;
//   MFHIP_DEVICE_SHARERS             rank mode: ranks sharing one device (the one-GPU ring rehearsal);
//   MFHIP_TEST                       "key=value,..." overrides the test suite uses to force the
//                                    alternative paths it compares bit for bit (test_knob); four of
//                                    them (pair_sys=0, fast_kernel=cell, det_kernel=level,
//                                    online_kernel=level) are also the supported production fallback
//                                    from the persistent sweeps.
// Experiment switches (hot-item replicas, group-model constants, wave traces, ...) exist only in a
// build with -DMFHIP_EXPERIMENTS (make EXPERIMENTS=1); the default build never reads them.
inline std::string test_knob(const char* key) {
  const char* s = std::getenv("MFHIP_TEST");  // read where it is used (never cached): one process may switch
  if (!s) return "";
  const size_t kl = std::strlen(key);
  for (const char* p = s;;) {
    const char* e = std::strchr(p, ',');
    const size_t len = e ? static_cast<size_t>(e - p) : std::strlen(p);
    if (len > kl && std::strncmp(p, key, kl) == 0 && p[kl] == '=') return std::string(p + kl + 1, len - kl - 1);
    if (!e) return "";
    p = e + 1;
  }
}
#ifdef MFHIP_EXPERIMENTS
inline const char* exp_knob(const char* name) { return std::getenv(name); }
constexpr bool kExperiments = true;
#else
inline const char* exp_knob(const char*) { return nullptr; }
constexpr bool kExperiments = false;
#endif

// Host worker count: OMP_NUM_THREADS / MFHIP_THREADS if set (the GPU box exports 16),
// else hardware_concurrency, capped at 32.
inline int host_threads() {
  for (const char* v : {"MFHIP_THREADS", "OMP_NUM_THREADS"}) {
    if (const char* s = std::getenv(v)) {
      int t = std::atoi(s);
      if (t > 0) return std::min(t, 64);
    }
  }
  unsigned hc = std::thread::hardware_concurrency();
  return static_cast<int>(std::max(1u, std::min(hc, 32u)));
}

// The host workers behind parallel_for / parallel_tasks: host_threads() - 1 threads made once per
// process and parked on a condition variable; the calling thread runs share 0.  Starting 16
// threads per call cost more than the work of an online micro-batch's staging copy
// (tools/micro/host_stage.cpp).  A call from a worker (nested), a call while another thread's
// job runs, or a call in a forked child (the pool's threads are not there) starts its own
// threads instead, as before.  The pool is never destroyed: its parked threads end with the
// process.
class WorkerPool {
 public:
  static WorkerPool* instance() {
    static WorkerPool* p = new WorkerPool(host_threads());
    return p->pid_ == ::getpid() ? p : nullptr;
  }
  // f(0..w-1) on the caller and w-1 workers; false (nothing run) when the pool cannot take it
  bool try_run(int w, const std::function<void(int)>& f) {
    if (in_worker() || w - 1 > static_cast<int>(th_.size())) return false;
    std::unique_lock<std::mutex> busy(run_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      width_ = w;
      left_ = w - 1;
      ++gen_;
    }
    wake_.notify_all();
    std::exception_ptr err;
    in_worker() = true;  // a parallel_for inside f(0) starts threads of its own (run_ is held)
    try {
      f(0);
    } catch (...) {
      err = std::current_exception();  // the workers still hold f: wait for them first
    }
    in_worker() = false;
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return left_ == 0; });
    job_ = nullptr;
    lk.unlock();
    if (err) std::rethrow_exception(err);
    return true;
  }

 private:
  explicit WorkerPool(int n) : pid_(::getpid()) {
    for (int t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
    for (auto& x : th_) x.detach();
  }
  static bool& in_worker() {
    static thread_local bool w = false;
    return w;
  }
  void loop(int t) {
    in_worker() = true;
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      wake_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (t >= width_) continue;  // not part of this job
      const std::function<void(int)>* f = job_;
      lk.unlock();
      (*f)(t);  // an exception here ends the process, as it did in a std::thread of its own
      lk.lock();
      if (--left_ == 0) done_.notify_one();
    }
  }
  const pid_t pid_;
  std::vector<std::thread> th_;
  std::mutex run_, m_;
  std::condition_variable wake_, done_;
  uint64_t gen_ = 0;
  const std::function<void(int)>* job_ = nullptr;
  int width_ = 0, left_ = 0;
};

// f(0..w-1), one share per host worker
inline void run_workers(int w, const std::function<void(int)>& f) {
  if (w <= 1) {
    f(0);
    return;
  }
  if (WorkerPool* p = WorkerPool::instance(); p && p->try_run(w, f)) return;
  std::vector<std::thread> th;
  th.reserve(w);
  for (int t = 0; t < w; ++t) th.emplace_back(f, t);
  for (auto& x : th) x.join();
}

// parallel_for over [0, n) in contiguous chunks; fn(begin, end, worker).
inline void parallel_for(int64_t n, const std::function<void(int64_t, int64_t, int)>& fn,
                         int max_workers = 0, int64_t min_chunk = 1 << 14) {
  if (n <= 0) return;
  int w = max_workers > 0 ? max_workers : host_threads();
  w = static_cast<int>(std::min<int64_t>(w, (n + min_chunk - 1) / min_chunk));
  if (w <= 1) { fn(0, n, 0); return; }
  const int64_t chunk = (n + w - 1) / w;
  run_workers(w, [&](int t) {
    const int64_t b = t * chunk, e = std::min(n, b + chunk);
    if (b < e) fn(b, e, t);
  });
}

// parallel over independent tasks 0..n-1, dynamically: each worker takes the next task index
// (tasks of very different sizes -- rating blocks -- then balance).
inline void parallel_tasks(int64_t n, const std::function<void(int64_t)>& fn, int max_workers = 0) {
  if (n <= 0) return;
  int w = max_workers > 0 ? max_workers : host_threads();
  w = static_cast<int>(std::min<int64_t>(w, n));
  if (w <= 1) { for (int64_t t = 0; t < n; ++t) fn(t); return; }
  std::atomic<int64_t> next{0};
  run_workers(w, [&](int) { for (int64_t x; (x = next.fetch_add(1)) < n;) fn(x); });
}

// Releases large host buffers on a background thread: returning a touched multi-GB allocation
// to the OS costs seconds (page freeing), which would otherwise sit inside mf_dsgd_prepare.
// drop() only takes the buffer over; release() hands everything taken to ONE thread (the unmaps
// hold the process's mmap lock, so a second thread's stack mmap would wait behind the first).
// Joined when the owner is destroyed (mf_destroy) or before the next prepare.
struct Reaper {
  std::vector<std::shared_ptr<void>> held;
  std::thread th;
  template <class V>
  void drop(V& v) {
    using T = std::decay_t<V>;
    held.emplace_back(new T(std::move(v)), [](void* p) { delete static_cast<T*>(p); });
    v = T();
  }
  void release() {
    join();
    if (held.empty()) return;
    th = std::thread([h = std::move(held)]() mutable { h.clear(); });
    held.clear();
  }
  void join() {
    if (th.joinable()) th.join();
  }
  ~Reaper() { join(); }
};

}  // namespace mfhip
