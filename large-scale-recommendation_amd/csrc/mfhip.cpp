// mfhip.cpp -- C ABI of libmfhip.so (include/mfhip.h): context, shards, DSGD driver,
// online micro-batches, evaluation and the item-block ring between GPUs.
//
// Execution model:
//  * A context owns G shards.  Shard g owns user blocks [g*c, (g+1)*c), c = numBlocks / G, and
//    the rating blocks of those rows, resident in HBM for the whole fit.
//  * Superstep s (1-based, DSGDforMF.scala:341-344, :476) runs rating blocks (p, (p+s-1) mod n)
//    for the shard's p on the shard's stream; afterwards the shard hands item block
//    (g*c + s - 1) mod n to shard g-1 and receives ((g+1)*c + s - 1) mod n from shard g+1 --
//    the nextRatingBlock rotation (:611-619).  In-process shards use peer copies; one process
//    per GPU (mf_create_rank) uses RCCL send/recv over xGMI.
//  * Every shard keeps full-size factor slabs with the global row numbering, so a block moves
//    by copying its row range; only the rows a shard currently owns are current.
#include <array>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <future>
#include <memory>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "common.hpp"
#include "jvm_random.hpp"
#include "kernels.hpp"
#include "plan.hpp"

namespace mfhip {

thread_local std::string g_last_error;

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    MF_HIP(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

#define MF_NCCL(call)                                                                     \
  do {                                                                                    \
    ncclResult_t _r = (call);                                                             \
    if (_r != ncclSuccess) ::mfhip::fail(MF_ERR_COMM, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

// Deterministic persistent sweep: one superstep's entries, staged in pinned memory by a host
// thread while earlier supersteps run, then copied to the device (fixed SoA offsets).  A ring of
// kDetSlots buffers: the host builds supersteps s+1 and s+2 (two builders at once) while the device
// runs s.  On the GPU box (16 host threads) one NFLX build takes ~28 ms alone and about as long
// with another beside it, i.e. ~14 ms per superstep -- the split sweep's ~14.4 ms launch; a third
// builder does not raise that rate (three at once: ~44 ms each, the host threads are saturated).
constexpr int kDetSlots = 3;
struct DetBuf {
  PinnedBuf pin;
  DevBuf dev;
  hipEvent_t copied = nullptr;  // the H2D from `pin` finished (pin may be rewritten)
  hipEvent_t swept = nullptr;   // the sweep that read `dev` finished (dev may be rewritten)
  bool pending = false;         // `copied` was recorded and not yet waited for
  bool dev_built = false;       // det_build left only the shuffle here: the device builds the entries
  int64_t n = 0, nw = 0;
  DetStepScratch scratch;  // build_det_step's gathers for this slot (kept: no page faults per superstep)
};

// A device mirror of one side's IdIndex (same slots), for the online batch's id lookup.
struct DevIndex {
  DevBuf slots, upd_pos, upd_val;
  uint64_t gen = 0, cap = 0;
  size_t applied = 0;  // entries of the table's write log already in the mirror
};

struct Shard {
  int device = 0;
  int index = 0;  // global shard index (== rank in rank mode)
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // host-to-device staging beside the sweeps (deterministic mode)
  // ring overlap (c >= 2 user blocks per shard, systolic fast sweep): the shard's last local block
  // runs on `aux` behind the arriving item block; the leaving block moves on `comm` as soon as
  // the launch holding the other blocks has finished
  hipStream_t aux = nullptr, comm = nullptr;
  hipEvent_t ev_front = nullptr;  // launch A (local blocks 0..c-2) of the latest superstep done
  hipEvent_t ev_last = nullptr;   // launch B (local block c-1) of the latest superstep done
  hipEvent_t ev_moved = nullptr;  // the item block this shard sent / received in the latest ring step
  std::vector<int64_t> st_sys_block_off;  // PairPlan::sys_block_off
  hipEvent_t done = nullptr;  // ring hand-off ordering between in-process shards
  DevBuf uf, itf, regu, regi;
  int64_t cap_u = 0, cap_i = 0;
  // deterministic mode staging
  DevBuf det_dev;
  PinnedBuf det_pin;
  OnlineSweepScratch online_sc;  // online micro-batches (k_online_sweep)
  DevIndex didx[2];              // device mirrors of the user [0] / item [1] IdIndex (online id lookup)
  PinnedBuf small_pin;           // online batch: {lookup misses, sweep error, touched users, items}, read back async
  PinnedBuf slots_pin;           // online f64 batch: the wave table read back for det_slot_table
  DevBuf blk_u, blk_i, blk_ru, blk_ri;  // mf_block_update: the block's factor rows and lambda / omega
  // fast mode
  DevBuf fast_recs, fast_cells, fast_blks;
  DevBuf fast_prog, fast_err;  // persistent sweep: progress words + timeout flag
  DevBuf st_recs, st_waves;    // pair schedule: records and per-cell wave table
  int64_t st_nrecs = 0;        // pair records in st_recs
  std::vector<int64_t> st_sub_off;
  std::vector<WaveDesc> st_waves_host;  // kept only when tracing
  DevBuf st_sys, st_sysw;               // systolic pair tables (PairPlan::sys, sys_waves)
  DevBuf st_place;                      // per systolic wave slot: block -> wave of its launch (sys_placement)
  std::vector<int64_t> st_place_off;     // per superstep: its first slot in st_place (nb + 1)
  std::vector<int32_t> st_place_pad;     // per superstep: empty blocks per XCD in its launch (sys_placement)
  std::vector<int64_t> st_sys_off;      // PairPlan::sys_off
  std::vector<WaveDesc> st_sys_host;    // kept only when tracing
  std::vector<SysWave> st_sysw_host;    // kept only when tracing
  uint32_t sys_base = 0;                // progress-word base of the next systolic launch
  uint32_t sys_step = 1;                // base advance per launch (> the largest G_j)
  DevBuf st_trace;                      // MFHIP_WAVE_TRACE: {start, end} per wave
  DevBuf st_split;                      // hot-item replicas (SplitItem), superstep-major
  std::vector<int64_t> st_split_off;    // per superstep (n + 1)
  std::vector<double> sm_bytes;         // per superstep index (s-1) mod n: bytes the sweep requests
  // deterministic persistent sweep (kernels_detsweep.hip)
  DetSweepLayout det_layout;
  DetBuf det_buf[kDetSlots];
  DevBuf det_ticket, det_err, det_scratch;
  int64_t det_n_max = 0, det_nw_max = 0;
  // the superstep's input built on the device (det_device_build; MFHIP_TEST det_build=host: on the
  // host): the rating blocks' 16-B records, the blocks' item -> wave maps, per superstep index
  // (s-1) mod n its block table and its wave / slot table (both fixed: a wave's count is the sum
  // of its items' counts), the uploaded shuffle permutation, and the build's scratch
  DevBuf det_aos_dev, det_iw, det_bt, det_ord;
  DetBuildScratch det_bs;
  std::vector<std::vector<DetWave>> det_sm_slots;
  std::vector<int64_t> det_sm_n;
  std::vector<int32_t> det_sm_nblk;
  uint32_t det_wave_bound = 1;
  // evaluation scratch
  DevBuf ev_u, ev_i, ev_r, ev_mult, ev_out, ev_part;
  // profiling
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  int64_t ev_launches = 0;
};

}  // namespace mfhip

struct mf_ctx {
  mfhip::Reaper reaper;  // host plan buffers being released in the background (first member: joined last)
  mf_params P{};
  std::vector<uint32_t> on_ur, on_ir;  // online batches: factor rows per rating (kept: no page faults per batch)
  bool f64 = true;
  size_t es = 8;  // bytes per factor element
  int G = 1;      // global shard count
  bool rank_mode = false;
  ncclComm_t comm = nullptr;
  std::vector<mfhip::Shard> shards;  // local shards
  mfhip::SideLayout U, I;
  bool have_model = false;
  bool prepared = false;
  int32_t nb = 1;
  int32_t c = 1;  // user blocks per shard
  int64_t superstep_done = 0;
  std::vector<int> item_loc;  // item block -> shard holding it
  mfhip::RatingBlocks rb;     // deterministic mode keeps the rating blocks on the host
  int32_t G_fast = 0;
  uint32_t fast_dummy_u = 0, fast_dummy_i = 0;  // zeroed rows past the real ones (padding / idle prefetch)
  int32_t fast_prio_len = 1 << 30;  // cells at least this long run at raised priority
  bool fast_persistent = false;  // MFHIP_TEST fast_kernel=persistent selects the systolic single launch
  bool fast_pair = false;         // two updates per step (kernels_pair.hip), k in {64, 128, 256}
  bool fast_sys = false;          // pair cells as one systolic launch per superstep (k_sweep_pair_sys)
  bool det_sweep = false;         // deterministic mode: one persistent k_det_sweep launch per superstep
  bool det_split = false;         // ... with single-item chains split over two waves (k_det_sweep_split)
  bool det_dev_build = false;     // ... its input built on the device from the host's shuffle (det_device_build)
  bool det_dev_ready = false;     // ... the device build prepared (the switch below may turn it on)
  bool det_mixed = false;         // ... MFHIP_TEST det_build=mixed: switch from the third superstep on
  std::atomic<bool> det_switch{false};  // ... the host builds fell behind the device: device builds from now on
  int det_idle = 0;               // ... consecutive supersteps whose build the device had to wait for
  bool det_alone = true;          // ... the longest chains on CUs of their own (det_slot_table)
  int64_t det_split_blocks = 0;   // resident blocks of k_det_sweep_split (per device share)
  int64_t det_cu_period = 256;    // CUs of the device: blocks b and b + period share a CU
  bool ring_overlap = false;      // fast systolic sweep, >1 shard, c >= 2: the ring step overlaps the sweep
  // fast-mode hot-item replicas (plan.hpp SplitItem), an experiment outside the product surface:
  // MFHIP_ITEM_SPLIT=m sweeps an item with more than m ratings in one rating block as ceil(r / m)
  // chains averaged when the superstep ends (read at prepare; 0 / unset = off)
  int32_t item_split = 0;
  std::vector<int64_t> fast_rb_size;  // per rating block (fast mode)
  mf_stats stats{};
  bool profiling = false;
  std::vector<int32_t> rows_by_id_u, rows_by_id_i;  // ascending-id row permutations
  bool order_dirty = true;
  int64_t init_seed = 0;      // seed of the initial factors (P.seed, or a random one when unseeded)
  std::string failed;         // non-empty: a device-side bound tripped; the fit must be prepared again
  // deterministic sweep: the next run's first supersteps, built on worker threads when a run ends
  // (a superstep's schedule depends only on its number and the training data): det_spec_s[slot] =
  // the superstep built into det_buf[slot], -1 = none (det_run takes them over; det_spec_wait
  // joins them where the data, layouts or superstep change)
  std::future<void> det_spec[mfhip::kDetSlots];
  int64_t det_spec_s[mfhip::kDetSlots] = {-1, -1, -1};
};

namespace mfhip {
namespace {

constexpr int kSideU = MF_SIDE_USER;

enum class FastKernel { kPair, kCell, kPersistent };

// Fast sweep kernel: pair (default where k is 64, 128 or 256; kernels_pair.hip) | cell (one
// update per step, any k; kernels_fast.hip) | persistent (kernels_fast.hip, one launch per
// superstep); MFHIP_TEST fast_kernel= overrides.
// Pair cells as one systolic launch per superstep (default; MFHIP_TEST pair_sys=0: one launch per
// sub-step).  Falls back to per-sub-step launches when a superstep's waves cannot all be resident.
bool want_pair_sys() { return test_knob("pair_sys") != "0"; }

FastKernel choose_fast_kernel(int k) {
  const std::string want = test_knob("fast_kernel");
  if (want == "persistent") return FastKernel::kPersistent;
  if (want == "cell") return FastKernel::kCell;
  if (pair_kernel_supports(k)) return FastKernel::kPair;
  return FastKernel::kCell;
}



double bytes_per_update(const mf_ctx* ctx) {
  const double k = ctx->P.num_factors;
  return ctx->f64 ? 32.0 * k + 24.0 : 16.0 * k + 20.0;
}

SideLayout& side_of(mf_ctx* ctx, int side) { return side == kSideU ? ctx->U : ctx->I; }

void validate_params(const mf_params* p) {
  MF_REQUIRE(p, "params is null");
  MF_REQUIRE(p->num_factors >= 1 && p->num_factors <= 512, "num_factors must be in [1, 512]");
  MF_REQUIRE(p->iterations >= 0, "iterations must be >= 0");
  MF_REQUIRE(p->num_blocks >= 1, "num_blocks must be >= 1");
  MF_REQUIRE(p->mode == MF_MODE_DETERMINISTIC_F64 || p->mode == MF_MODE_FAST_F32, "unknown mode");
  MF_REQUIRE(p->lr_method >= MF_LR_DEFAULT && p->lr_method <= MF_LR_XU, "unknown lr_method");
  MF_REQUIRE(p->fast_blocking == MF_BLOCKING_BALANCED || p->fast_blocking == MF_BLOCKING_REFERENCE,
             "unknown fast_blocking");
}

void init_shard(Shard& s, int device, int index) {
  s.device = device;
  s.index = index;
  DeviceGuard g(device);
  MF_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  MF_HIP(hipStreamCreateWithFlags(&s.copy_stream, hipStreamNonBlocking));
  MF_HIP(hipStreamCreateWithFlags(&s.aux, hipStreamNonBlocking));
  MF_HIP(hipStreamCreateWithFlags(&s.comm, hipStreamNonBlocking));
  MF_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  for (hipEvent_t* e : {&s.ev_front, &s.ev_last, &s.ev_moved}) MF_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  for (auto& b : s.det_buf) {
    MF_HIP(hipEventCreateWithFlags(&b.copied, hipEventDisableTiming));
    MF_HIP(hipEventCreateWithFlags(&b.swept, hipEventDisableTiming));
  }
}

void destroy_shard(Shard& s) {
  if (!s.stream) return;
  (void)hipSetDevice(s.device);
  (void)hipStreamSynchronize(s.stream);
  (void)hipStreamSynchronize(s.copy_stream);
  (void)hipStreamSynchronize(s.aux);
  (void)hipStreamSynchronize(s.comm);
  for (hipEvent_t e : {s.ev_front, s.ev_last, s.ev_moved})
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(s.aux);
  (void)hipStreamDestroy(s.comm);
  for (auto e : s.ev) (void)hipEventDestroy(e);
  s.ev.clear();
  for (auto& b : s.det_buf) {
    if (b.copied) (void)hipEventDestroy(b.copied);
    if (b.swept) (void)hipEventDestroy(b.swept);
  }
  (void)hipEventDestroy(s.done);
  (void)hipStreamDestroy(s.copy_stream);
  (void)hipStreamDestroy(s.stream);
  s.stream = nullptr;
}

// Grow a factor slab (and its regularisation column) to hold `rows`, keeping the contents.
void ensure_rows(mf_ctx* ctx, Shard& s, int side, int64_t rows) {
  int64_t& cap = side == kSideU ? s.cap_u : s.cap_i;
  if (rows <= cap) return;
  DeviceGuard g(s.device);
  const int64_t ncap = std::max<int64_t>({rows, cap * 2, 1024});
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  DevBuf f, rg;
  f.alloc(static_cast<size_t>(ncap) * k * ctx->es);
  rg.alloc(static_cast<size_t>(ncap) * ctx->es);
  MF_HIP(hipMemsetAsync(rg.get(), 0, static_cast<size_t>(ncap) * ctx->es, s.stream));
  DevBuf& of = side == kSideU ? s.uf : s.itf;
  DevBuf& og = side == kSideU ? s.regu : s.regi;
  if (cap > 0) {
    MF_HIP(hipMemcpyAsync(f.get(), of.get(), static_cast<size_t>(cap) * k * ctx->es, hipMemcpyDeviceToDevice, s.stream));
    MF_HIP(hipMemcpyAsync(rg.get(), og.get(), static_cast<size_t>(cap) * ctx->es, hipMemcpyDeviceToDevice, s.stream));
  }
  MF_HIP(hipStreamSynchronize(s.stream));
  of = std::move(f);
  og = std::move(rg);
  cap = ncap;
}

// Host f64 rows -> device slab rows [row0, row0+n) in the context's precision.
void upload_rows(mf_ctx* ctx, Shard& s, int side, int64_t row0, const double* src, int64_t n) {
  if (n <= 0) return;
  DeviceGuard g(s.device);
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  DevBuf& slab = side == kSideU ? s.uf : s.itf;
  char* dst = slab.as<char>() + static_cast<size_t>(row0) * k * ctx->es;
  if (ctx->f64) {
    MF_HIP(hipMemcpy(dst, src, static_cast<size_t>(n) * k * 8, hipMemcpyHostToDevice));
  } else {
    std::vector<float> tmp(static_cast<size_t>(n) * k);
    parallel_for(static_cast<int64_t>(tmp.size()), [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x) tmp[x] = static_cast<float>(src[x]);
    });
    MF_HIP(hipMemcpy(dst, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice));
  }
}

void upload_regs(mf_ctx* ctx, Shard& s, int side, int64_t row0, const double* src, int64_t n) {
  if (n <= 0) return;
  DeviceGuard g(s.device);
  DevBuf& reg = side == kSideU ? s.regu : s.regi;
  char* dst = reg.as<char>() + static_cast<size_t>(row0) * ctx->es;
  if (ctx->f64) {
    MF_HIP(hipMemcpy(dst, src, static_cast<size_t>(n) * 8, hipMemcpyHostToDevice));
  } else {
    std::vector<float> tmp(n);
    for (int64_t x = 0; x < n; ++x) tmp[x] = static_cast<float>(src[x]);
    MF_HIP(hipMemcpy(dst, tmp.data(), static_cast<size_t>(n) * 4, hipMemcpyHostToDevice));
  }
}

// Device slab rows [row0, row0+n) -> host f64.
void download_rows(mf_ctx* ctx, Shard& s, int side, int64_t row0, int64_t n, double* out) {
  if (n <= 0) return;
  DeviceGuard g(s.device);
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  DevBuf& slab = side == kSideU ? s.uf : s.itf;
  const char* src = slab.as<char>() + static_cast<size_t>(row0) * k * ctx->es;
  MF_HIP(hipStreamSynchronize(s.stream));
  if (ctx->f64) {
    MF_HIP(hipMemcpy(out, src, static_cast<size_t>(n) * k * 8, hipMemcpyDeviceToHost));
  } else {
    std::vector<float> tmp(static_cast<size_t>(n) * k);
    MF_HIP(hipMemcpy(tmp.data(), src, tmp.size() * 4, hipMemcpyDeviceToHost));
    for (size_t x = 0; x < tmp.size(); ++x) out[x] = static_cast<double>(tmp[x]);
  }
}

// Initial factors: k x nextDouble of new Random(id ^ seed) (DSGDforMF.scala:548-549), or of
// new Random(id) for PseudoRandomFactorInitializer (core/FactorInitializer.scala:23-27).
void init_vectors(const int32_t* ids, int64_t n, int k, bool xor_seed, int64_t seed, std::vector<double>& out) {
  out.resize(static_cast<size_t>(n) * k);
  parallel_for(n, [&](int64_t b, int64_t e, int) {
    for (int64_t x = b; x < e; ++x) {
      JavaRandom rng(xor_seed ? (static_cast<int64_t>(ids[x]) ^ seed) : static_cast<int64_t>(ids[x]));
      double* v = out.data() + static_cast<size_t>(x) * k;
      for (int f = 0; f < k; ++f) v[f] = rng.nextDouble();
    }
  }, 0, 1024);
}

// ---------------------------------------------------------------------------------------
// profiling: a pair of HIP events around every sweep-kernel launch on the shard's stream.
// ext = true: the launch records the pair itself (hipExtLaunchKernel start/stop events, part
// of the dispatch packet, so timing adds no commands between kernels); start() / stop() give
// the events, or null when profiling is off.
struct LaunchTimer {
  Shard& s;
  bool on, ext;
  size_t slot = 0;
  LaunchTimer(Shard& sh, bool enabled, bool ext_events = false) : s(sh), on(enabled), ext(ext_events) {
    if (!on) return;
    if (s.ev_used + 2 > s.ev.size()) {
      for (int x = 0; x < 512; ++x) {
        hipEvent_t e;
        MF_HIP(hipEventCreate(&e));
        s.ev.push_back(e);
      }
    }
    slot = s.ev_used;
    s.ev_used += 2;
    if (!ext) MF_HIP(hipEventRecord(s.ev[slot], s.stream));
  }
  hipEvent_t start() const { return on ? s.ev[slot] : nullptr; }
  hipEvent_t stop() const { return on ? s.ev[slot + 1] : nullptr; }
  ~LaunchTimer() {
    if (on) {
      if (!ext) (void)hipEventRecord(s.ev[slot + 1], s.stream);
      s.ev_launches++;
    }
  }
};

void collect_profile(mf_ctx* ctx) {
  for (auto& s : ctx->shards) {
    if (s.ev_used == 0) continue;
    DeviceGuard g(s.device);
    MF_HIP(hipStreamSynchronize(s.stream));
    double ms = 0.0;
    for (size_t x = 0; x + 1 < s.ev_used; x += 2) {
      float t = 0.f;
      MF_HIP(hipEventElapsedTime(&t, s.ev[x], s.ev[x + 1]));
      ms += t;
    }
    ctx->stats.kernel_ms += ms;
    s.ev_used = 0;
  }
}

// MFHIP_WAVE_TRACE=<file>: per wave of the per-cell schedules "shard sm t wave steps cells start
// end" (100 MHz clock) of the last time every sub-step ran; written when the context is destroyed.
// The systolic sweep adds a 9th column: the cell's shader-clock cycles (s_memtime), so the clock
// the wave actually ran at is cycles / ((end - start) x 10 ns), and a 10th: where the wave ran,
// XCC_ID << 32 | HW_ID (SIMD bits 5:4, CU 11:8, SH 12, SE 15:13).
void dump_wave_trace(mf_ctx* ctx) {
  const char* path = exp_knob("MFHIP_WAVE_TRACE");
  if (!path) return;
  FILE* f = nullptr;
  for (auto& s : ctx->shards) {
    if (s.st_trace.get() && !s.st_sys_host.empty()) {  // systolic: one row per cell, wave = index in superstep
      DeviceGuard g(s.device);
      std::vector<uint64_t> tr(s.st_sys_host.size() * 4);
      MF_HIP(hipMemcpy(tr.data(), s.st_trace.get(), tr.size() * 8, hipMemcpyDeviceToHost));
      if (!f) f = std::fopen(path, "w");
      if (!f) return;
      for (int32_t sm = 0; sm < ctx->nb; ++sm)
        for (int64_t w = s.st_sys_off[sm]; w < s.st_sys_off[sm + 1]; ++w) {
          const SysWave& sw = s.st_sysw_host[w];
          for (int32_t t = 0; t < sw.G; ++t) {
            const int64_t x = sw.cell0 + t;
            std::fprintf(f, "%d %d %d %lld %d %d %llu %llu %llu %llu\n", s.index, sm, t, (long long)(w - s.st_sys_off[sm]),
                         s.st_sys_host[x].steps, s.st_sys_host[x].cells, (unsigned long long)tr[4 * x],
                         (unsigned long long)tr[4 * x + 1], (unsigned long long)tr[4 * x + 2],
                         (unsigned long long)tr[4 * x + 3]);
          }
        }
      continue;
    }
    if (!s.st_trace.get() || s.st_waves_host.empty()) continue;
    DeviceGuard g(s.device);
    std::vector<uint64_t> tr(s.st_waves_host.size() * 2);
    MF_HIP(hipMemcpy(tr.data(), s.st_trace.get(), tr.size() * 8, hipMemcpyDeviceToHost));
    if (!f) f = std::fopen(path, "w");
    if (!f) return;
    const int64_t G = ctx->G_fast;
    for (size_t x = 0; x + 1 < s.st_sub_off.size(); ++x)
      for (int64_t w = s.st_sub_off[x]; w < s.st_sub_off[x + 1]; ++w)
        std::fprintf(f, "%d %lld %lld %lld %d %d %llu %llu\n", s.index, (long long)(x / G), (long long)(x % G),
                     (long long)(w - s.st_sub_off[x]), s.st_waves_host[w].steps, s.st_waves_host[w].cells,
                     (unsigned long long)tr[2 * w], (unsigned long long)tr[2 * w + 1]);
  }
  if (f) std::fclose(f);
}

// Joins the speculative builds of det_run.  invalidate: the training data, the layouts or the
// superstep changes, so the builds are dropped (otherwise a later run may still use them).
// A failed build is never used: its slot is marked empty before the error can surface, and when the
// builds are being dropped (invalidate) their errors are dropped with them (MFHIP_DEBUG_PLAN logs
// them) -- only a run that would take a build over reports its failure (det_run).
void det_spec_wait(mf_ctx* ctx, bool invalidate) {
  std::exception_ptr first;
  for (int slot = 0; slot < kDetSlots; ++slot) {
    if (ctx->det_spec[slot].valid()) {
      try {
        ctx->det_spec[slot].get();
      } catch (const std::exception& e) {
        ctx->det_spec_s[slot] = -1;
        if (invalidate) {
          if (std::getenv("MFHIP_DEBUG_PLAN")) std::fprintf(stderr, "[mfhip] dropped speculative build: %s\n", e.what());
        } else if (!first) {
          first = std::current_exception();
        }
      } catch (...) {
        ctx->det_spec_s[slot] = -1;
        if (!invalidate && !first) first = std::current_exception();
      }
    }
    if (invalidate) ctx->det_spec_s[slot] = -1;
  }
  if (first) std::rethrow_exception(first);
}

// (does not wait for det_run's speculative builds: they touch no device state, and a caller's
// sync must not pay for the next run's host work)
void sync_all(mf_ctx* ctx) {
  for (auto& s : ctx->shards) {
    DeviceGuard g(s.device);
    MF_HIP(hipStreamSynchronize(s.stream));
    MF_HIP(hipStreamSynchronize(s.aux));
    MF_HIP(hipStreamSynchronize(s.comm));
    for (DevBuf* eb : {&s.fast_err, &s.det_err}) {
      if (!eb->get()) continue;
      int32_t err4[4] = {0, 0, 0, 0};
      MF_HIP(hipMemcpy(err4, eb->get(), std::min<size_t>(sizeof(err4), eb->bytes()), hipMemcpyDeviceToHost));
      const int32_t err = err4[0];
      if (err) {
        MF_HIP(hipMemsetAsync(eb->get(), 0, std::min<size_t>(sizeof(err4), eb->bytes()), s.stream));
        MF_HIP(hipStreamSynchronize(s.stream));
        if (std::getenv("MFHIP_DEBUG_PLAN") && eb->bytes() > 16) {
          std::vector<uint32_t> dg(eb->bytes() / 4);
          MF_HIP(hipMemcpy(dg.data(), eb->get(), eb->bytes(), hipMemcpyDeviceToHost));
          for (size_t w = 0; 4 + 4 * w + 3 < dg.size(); ++w)
            if (dg[4 + 4 * w + 3])
              std::fprintf(stderr, "[mfhip] sweep timeout: wave slot %zu seen %u want %u published %u\n", w,
                           dg[4 + 4 * w], dg[4 + 4 * w + 1], dg[4 + 4 * w + 2]);
          MF_HIP(hipMemsetAsync(eb->get(), 0, eb->bytes(), s.stream));
          MF_HIP(hipStreamSynchronize(s.stream));
        }
        // waves that gave up skipped the rest of their work: the model is partly updated, so
        // the context refuses further supersteps and reads until the fit is prepared again
        ctx->failed = eb == &s.fast_err
                          ? "fast sweep: a wave waited > 1 s for its neighbour (workgroups not co-resident?); "
                            "set MFHIP_TEST=pair_sys=0 (or fast_kernel=cell; INTEGRATION.md section 5)"
                          : "deterministic sweep: a wave waited > 1 s for a user ticket (waves not co-resident?); "
                            "set MFHIP_TEST=det_kernel=level (INTEGRATION.md section 5)";
        fail(MF_ERR_TIMEOUT, ctx->failed);
      }
    }
  }
  collect_profile(ctx);
}

void require_healthy(const mf_ctx* ctx) {
  if (!ctx->failed.empty())
    fail(MF_ERR_STATE, "the context failed earlier (" + ctx->failed + "); prepare the fit again");
}

// ---------------------------------------------------------------------------------------
// Model construction for a fit.
// Slab rows [0, n) := initial factors of ids[0..n) generated on the device (launch_jvm_init_rows):
// only the ids cross PCIe (4 B per row instead of k doubles), bit-exact with init_vectors.
void init_rows_on_device(mf_ctx* ctx, Shard& s, int side, const int32_t* ids, int64_t n, bool xor_seed, int64_t seed) {
  if (n <= 0) return;
  DeviceGuard g(s.device);
  const int k = ctx->P.num_factors;
  std::vector<uint64_t> jump(4 * static_cast<size_t>(k));  // (mult, add) after m = 1..2k LCG steps
  constexpr uint64_t kMult = 0x5DEECE66DULL, kMask = (1ULL << 48) - 1;
  uint64_t m = 1, a = 0;
  for (int step = 0; step < 2 * k; ++step) {
    m = (m * kMult) & kMask;
    a = (a * kMult + 0xBULL) & kMask;
    jump[2 * step] = m;
    jump[2 * step + 1] = a;
  }
  DevBuf dids, djump;
  dids.alloc(static_cast<size_t>(n) * 4);
  djump.alloc(jump.size() * 8);
  MF_HIP(hipMemcpyAsync(dids.get(), ids, static_cast<size_t>(n) * 4, hipMemcpyHostToDevice, s.stream));
  MF_HIP(hipMemcpyAsync(djump.get(), jump.data(), jump.size() * 8, hipMemcpyHostToDevice, s.stream));
  DevBuf& slab = side == kSideU ? s.uf : s.itf;
  launch_jvm_init_rows(s.stream, dids.as<int32_t>(), n, k, xor_seed, seed, djump.as<uint64_t>(), slab.get(), ctx->f64);
  MF_HIP(hipGetLastError());
  MF_HIP(hipStreamSynchronize(s.stream));  // the temporaries die here
}

// Every shard's slabs := the initial factors of every row (fitSGD's starting point).
void init_factors(mf_ctx* ctx) {
  for (int side = 0; side < 2; ++side) {
    SideLayout& S = side == kSideU ? ctx->U : ctx->I;
    for (auto& s : ctx->shards) init_rows_on_device(ctx, s, side, S.row_id.data(), S.rows(), true, ctx->init_seed);
  }
}

// sides_built: ctx->U / ctx->I already hold the blocking (device_blocking).
void build_model(mf_ctx* ctx, const int32_t* u, const int32_t* i, int64_t n, bool sides_built) {
  const bool seeded = ctx->P.has_seed != 0;
  const Blocking bl = !ctx->f64 && ctx->P.fast_blocking == MF_BLOCKING_BALANCED ? Blocking::kBalanced : Blocking::kJvm;
  if (!sides_built) {
    build_side(ctx->U, u, n, ctx->nb, ctx->P.seed, seeded, bl);
    build_side(ctx->I, i, n, ctx->nb, ctx->P.seed, seeded, bl);
  }
  for (int side = 0; side < 2; ++side) {
    SideLayout& S = side == kSideU ? ctx->U : ctx->I;
    std::vector<double> reg(S.rows());
    for (int64_t x = 0; x < S.rows(); ++x) reg[x] = ctx->P.lambda / static_cast<double>(S.omega[x]);
    for (auto& s : ctx->shards) {
      ensure_rows(ctx, s, side, std::max<int64_t>(S.rows(), 1));
      upload_regs(ctx, s, side, 0, reg.data(), S.rows());
    }
  }
  ctx->init_seed = ctx->P.seed;
  if (!seeded) {
    std::random_device rd;
    ctx->init_seed = (static_cast<int64_t>(rd()) << 32) ^ rd();
  }
  init_factors(ctx);
  ctx->have_model = true;
  ctx->order_dirty = true;
}

void ensure_order(mf_ctx* ctx) {
  if (!ctx->order_dirty) return;
  for (int side = 0; side < 2; ++side) {
    SideLayout& S = side_of(ctx, side);
    auto& ord = side == kSideU ? ctx->rows_by_id_u : ctx->rows_by_id_i;
    ord.resize(S.rows());
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return S.row_id[a] < S.row_id[b]; });
  }
  ctx->order_dirty = false;
}

int shard_of_user_block(const mf_ctx* ctx, int32_t p) { return p / ctx->c; }

Shard* local_shard(mf_ctx* ctx, int global) {
  for (auto& s : ctx->shards)
    if (s.index == global) return &s;
  return nullptr;
}

// ---------------------------------------------------------------------------------------
// One superstep on one shard.
void det_superstep(mf_ctx* ctx, Shard& s, int64_t superstep, int32_t iteration, double eta) {
  const int32_t n = ctx->nb;
  std::vector<std::vector<int32_t>> orders;
  std::vector<OrderedSeq> seqs;
  std::vector<int64_t> rbids;
  for (int32_t j = 0; j < ctx->c; ++j) {
    const int32_t p = s.index * ctx->c + j;
    const int32_t q = static_cast<int32_t>((p + superstep - 1) % n);
    const int64_t b = static_cast<int64_t>(p) * n + q;  // toRatingBlockId (:597-601)
    if (ctx->rb.size(b) > 0) rbids.push_back(b);
  }
  orders.resize(rbids.size());
  parallel_tasks(static_cast<int64_t>(rbids.size()), [&](int64_t x) {
    const int64_t b = rbids[x];
    const int64_t len = ctx->rb.size(b);
    orders[x].resize(len);
    if (ctx->P.has_seed) {
      JavaRandom rng(static_cast<int64_t>(iteration ^ static_cast<int32_t>(b)) ^ ctx->P.seed);  // :392
      scala_shuffle(rng, orders[x].data(), len);                                                // :393
    } else {
      std::random_device rd;
      JavaRandom rng((static_cast<int64_t>(rd()) << 32) ^ rd());
      scala_shuffle(rng, orders[x].data(), len);
    }
  });
  for (size_t x = 0; x < rbids.size(); ++x) {
    const int64_t b = rbids[x];
    const int32_t p = static_cast<int32_t>(b / n), q = static_cast<int32_t>(b % n);
    const int64_t st = ctx->rb.start[b];
    OrderedSeq sq;
    sq.u = ctx->rb.urow.data() + st;
    sq.i = ctx->rb.irow.data() + st;
    sq.r = ctx->rb.r.data() + st;
    sq.order = orders[x].data();
    sq.len = ctx->rb.size(b);
    sq.u_lo = static_cast<uint32_t>(ctx->U.block_start[p]);
    sq.u_hi = static_cast<uint32_t>(ctx->U.block_start[p + 1]);
    sq.i_lo = static_cast<uint32_t>(ctx->I.block_start[q]);
    sq.i_hi = static_cast<uint32_t>(ctx->I.block_start[q + 1]);
    seqs.push_back(sq);
  }
  if (seqs.empty()) return;
  LevelPlan lp;
  build_level_plan(seqs, lp);
  DeviceGuard g(s.device);
  const size_t bytes = lp.entries.size() * sizeof(DetEntry);
  MF_HIP(hipStreamSynchronize(s.stream));  // the pinned staging buffer is reused
  s.det_pin.alloc(bytes);
  s.det_dev.alloc(bytes);
  std::memcpy(s.det_pin.as<void>(), lp.entries.data(), bytes);
  MF_HIP(hipMemcpyAsync(s.det_dev.get(), s.det_pin.as<void>(), bytes, hipMemcpyHostToDevice, s.stream));
  const DetEntry* dev = s.det_dev.as<DetEntry>();
  for (int64_t l = 0; l < lp.levels(); ++l) {
    const int64_t b0 = lp.level_start[l], cnt = lp.level_start[l + 1] - b0;
    LaunchTimer t(s, ctx->profiling);
    launch_level(s.stream, dev + b0, cnt, s.uf.get(), s.itf.get(), s.regu.get(), s.regi.get(),
                 ctx->P.num_factors, eta, Arith::kDsgd, true);
  }
  MF_HIP(hipGetLastError());
  ctx->stats.levels += lp.levels();
  ctx->stats.updates += static_cast<int64_t>(lp.entries.size());
  ctx->stats.kernel_launches += lp.levels();
  // per update: two f64 rows read and written, the 16-B entry, the two lambda/omega values
  ctx->stats.moved_bytes += static_cast<double>(lp.entries.size()) * (32.0 * ctx->P.num_factors + 32.0);
}

// Block -> wave map of one systolic launch (waves [a, z) of a superstep whose waves start at w0 in
// pp.sys_waves), written to place[w0 + a + b].  Measured (profiles/r03_placement_NFLX.txt): the
// dispatcher deals a launch's blocks round-robin over the 8 XCDs (b % 8) and, inside an XCD, over
// its 32 CUs in block order, so the XCD's blocks k, k + 32, k + 64 (k = b / 8) share a CU -- every
// one of 4768 block pairs (b, b + 256) in two traced fits did.  And a wave's pair step slows with
// every other busy wave on its CU (NFLX single-run pairs: 127 ns alone, 173 ns with one other
// wave, 206 ns with two; mixed pairs 214 / 248 ns): the CU's shared vector-memory path, not the
// SIMD (no two waves ever shared one).  So each XCD keeps its contiguous wave range (the hand-offs
// stay in one L2), and inside it the heaviest waves (modelled time) take the CUs that hold the
// fewest waves, with the lightest waves as their partners.  Placement only: results are
// identical (tests compare with the per-sub-step launches bit for bit).  MFHIP_SYS_PLACE=0: the
// plain XCD-contiguous map.  Measured and dropped: per-CU wave counts chosen against a crowding
// factor (1 / 1.3 / 1.52 / 1.8 per waves on the CU), spare slots padded with empty blocks -- NFLX
// 21.6 vs 21.3 ms, ML20M equal (profiles/r03_placement_NFLX.txt).  Kept since round 6: one empty
// block per XCD as the heaviest wave's partner, so each rating block's hot-item wave has a CU to
// itself (NFLX 19.88 -> 19.74 ms, profiles/r06_sys_isolation_ab.txt; single-run pairs now weigh
// 185 ns: at 171 the hot wave sometimes ranked 16th-54th of its XCD).
// pad (>= 0): empty blocks per XCD (place = -1, they exit at once), dealt as the lightest partners:
// the heaviest wave of each XCD then shares its CU with empty blocks only -- alone on it when pad
// covers its CU's other slots (sys_iso_pad).  place gets nw + 8 pad entries from out on.
void sys_placement(const PairPlan& pp, int64_t w0, int64_t a, int64_t z, std::vector<int32_t>& place, int64_t out,
                   int32_t pad = 0) {
  const int64_t nw = z - a;
  if (nw <= 0) return;
  std::vector<double> load(nw, 0.0);
  for (int64_t L = 0; L < nw; ++L) {
    const SysWave& sw = pp.sys_waves[w0 + a + L];
    for (int32_t t = 0; t < sw.G; ++t) {
      const WaveDesc& d = pp.sys[sw.cell0 + t];
      if (d.steps > 0) load[L] += 2000.0 + d.steps * (d.cells == kWaveSingleRun || d.cells == kWaveSingleRunFwd ? 185.0 : 218.0);
    }
  }
  const int64_t per = nw / 8, extra = nw % 8;
  for (int64_t x = 0; x < 8; ++x) {
    const int64_t nx = per + (x < extra ? 1 : 0), base = x * per + std::min(x, extra);
    if (nx == 0) continue;
    const int64_t n = nx + pad;  // this XCD's blocks
    std::vector<int64_t> byload(n);  // this XCD's waves, heaviest first, then the empty blocks (-1)
    std::iota(byload.begin(), byload.begin() + nx, base);
    std::fill(byload.begin() + nx, byload.end(), -1);
    std::stable_sort(byload.begin(), byload.begin() + nx, [&](int64_t u, int64_t v) { return load[u] > load[v]; });
    std::vector<int64_t> cus(std::min<int64_t>(n, 32));  // CU slots, fewest waves first
    std::iota(cus.begin(), cus.end(), 0);
    auto members = [&](int64_t c) { return (n - c + 31) / 32; };
    std::stable_sort(cus.begin(), cus.end(), [&](int64_t u, int64_t v) { return members(u) < members(v); });
    int64_t hi = 0, lo = n - 1;
    for (int64_t c : cus)
      for (int64_t kk = c, m = 0; kk < n; kk += 32, ++m)
        place[out + x + 8 * kk] = static_cast<int32_t>(m == 0 ? byload[hi++] : byload[lo--]);
  }
}

// Empty blocks per XCD that leave the `iso` heaviest waves of every XCD alone on their CUs: iso x
// (the fewest blocks a CU slot holds - 1) once the XCD holds nw / 8 + pad blocks.  0 when the
// launch could not hold them all at once (cap), or when the padding would put one more wave on the
// fullest CUs (YAHOO, 126 waves per XCD: pad 3 makes a five-wave CU, 236.6 -> 270 ms per epoch).
int32_t sys_iso_pad(int64_t nw, int64_t cap, int32_t iso) {
  const int64_t n0 = (nw + 7) / 8;  // the fullest XCD's waves (a smaller XCD needs no more)
  for (int32_t pad = 0; pad <= 3 * iso; ++pad) {
    const int64_t n = n0 + pad;
    const int64_t fewest = n <= 32 ? 1 : n / 32;  // blocks of its emptiest CU slot
    if (iso * (fewest - 1) <= pad)
      return nw + 8 * pad <= cap && (n + 31) / 32 == (n0 + 31) / 32 ? pad : 0;
  }
  return 0;
}

void fast_superstep(mf_ctx* ctx, Shard& s, int64_t superstep, double eta) {
  const int32_t n = ctx->nb;
  const int64_t smod = (superstep - 1) % n;
  DeviceGuard g(s.device);
  const FastBlk* blks = s.fast_blks.as<FastBlk>() + smod * ctx->c;
  int64_t ups = 0;
  for (int32_t j = 0; j < ctx->c; ++j) {
    const int32_t p = s.index * ctx->c + j;
    const int32_t q = static_cast<int32_t>((p + superstep - 1) % n);
    ups += ctx->fast_rb_size[static_cast<int64_t>(p) * n + q];
  }
  if (ups == 0) return;
  const int64_t sp0 = s.st_split_off.empty() ? 0 : s.st_split_off[smod];
  const int nsplit = s.st_split_off.empty() ? 0 : static_cast<int>(s.st_split_off[smod + 1] - sp0);
  launch_split_fork(s.stream, s.st_split.as<SplitItem>() + sp0, nsplit, s.itf.as<float>(), ctx->P.num_factors);
  if (ctx->fast_pair && ctx->fast_sys) {
    const int64_t w0 = s.st_sys_off[smod], nw = s.st_sys_off[smod + 1] - w0;
    auto sweep = [&](hipStream_t st, int64_t a, int64_t z) {  // waves [a, z) of the superstep
      if (z <= a) return;
      LaunchTimer tm(s, ctx->profiling, true);
      // with a placement table the launch has its empty blocks too (sys_placement pad)
      const bool placed = s.st_place.get() != nullptr;
      const int64_t blocks = z - a + (placed && a == 0 && z == nw ? 8 * s.st_place_pad[smod] : 0);
      launch_sweep_pair_sys(st, s.st_sysw.as<SysWave>() + w0 + a, s.st_sys.as<WaveDesc>(), static_cast<int>(blocks),
                            static_cast<int>(a), s.st_recs.as<PairRec>(), s.uf.as<float>(), s.itf.as<float>(),
                            s.uf.bytes(), s.itf.bytes(), ctx->P.num_factors, static_cast<float>(eta),
                            s.fast_prog.as<int32_t>(), s.sys_base, s.fast_err.as<int32_t>(),
                            s.st_trace.get() ? s.st_trace.as<uint64_t>() : nullptr, tm.start(), tm.stop(),
                            placed ? s.st_place.as<int32_t>() + s.st_place_off[smod] + a : nullptr);
      ctx->stats.kernel_launches += 1;
    };
    if (ctx->ring_overlap) {
      // A: local blocks 0..c-2 on the compute stream, behind the previous superstep's block c-1
      // (its item block is A's last one now); B: block c-1 on aux, behind the item block the
      // ring step delivered.  Both may run at once (disjoint rows, all waves resident).
      const int64_t split = s.st_sys_block_off[static_cast<size_t>(smod) * (ctx->c + 1) + ctx->c - 1];
      MF_HIP(hipStreamWaitEvent(s.stream, s.ev_last, 0));
      sweep(s.stream, 0, split);
      MF_HIP(hipEventRecord(s.ev_front, s.stream));
      MF_HIP(hipStreamWaitEvent(s.aux, s.ev_moved, 0));
      sweep(s.aux, split, nw);
      MF_HIP(hipEventRecord(s.ev_last, s.aux));
    } else {
      sweep(s.stream, 0, nw);
    }
    if (nw > 0) s.sys_base += s.sys_step;
  } else if (ctx->fast_pair) {
    for (int32_t t = 0; t < ctx->G_fast; ++t) {
      const int64_t x = smod * ctx->G_fast + t;
      const int64_t w0 = s.st_sub_off[x], nw = s.st_sub_off[x + 1] - w0;
      if (nw == 0) continue;
      LaunchTimer tm(s, ctx->profiling, true);
      launch_sweep_pair(s.stream, s.st_waves.as<WaveDesc>() + w0, static_cast<int>(nw), s.st_recs.as<PairRec>(),
                        s.uf.as<float>(), s.itf.as<float>(), s.uf.bytes(), s.itf.bytes(), ctx->P.num_factors,
                        static_cast<float>(eta), s.st_trace.get() ? s.st_trace.as<uint64_t>() + 2 * w0 : nullptr,
                        tm.start(), tm.stop());
      ctx->stats.kernel_launches += 1;
    }
  } else if (ctx->fast_persistent) {
    MF_HIP(hipMemsetAsync(s.fast_prog.get(), 0, s.fast_prog.bytes(), s.stream));
    LaunchTimer tm(s, ctx->profiling);
    launch_fast_superstep(s.stream, blks, ctx->c, ctx->G_fast, s.fast_recs.as<FastRec>(), s.fast_cells.as<int32_t>(),
                          s.uf.as<float>(), s.itf.as<float>(), ctx->P.num_factors, static_cast<float>(eta),
                          s.uf.bytes(), s.itf.bytes(), (ctx->fast_dummy_u + 1) * 4u * ctx->P.num_factors,
                          ctx->fast_dummy_i * 4u * ctx->P.num_factors, s.fast_prog.as<int32_t>(),
                          s.fast_err.as<int32_t>());
    ctx->stats.kernel_launches += 1;
  } else {
    for (int32_t t = 0; t < ctx->G_fast; ++t) {
      LaunchTimer tm(s, ctx->profiling);
      launch_fast_substep(s.stream, blks, ctx->c, ctx->G_fast, t, s.fast_recs.as<FastRec>(),
                          s.fast_cells.as<int32_t>(), s.uf.as<float>(), s.itf.as<float>(), ctx->P.num_factors,
                          static_cast<float>(eta), s.uf.bytes(), s.itf.bytes(),
                          (ctx->fast_dummy_u + 1) * 4u * ctx->P.num_factors,
                          ctx->fast_dummy_i * 4u * ctx->P.num_factors, ctx->fast_prio_len);
    }
    ctx->stats.kernel_launches += ctx->G_fast;
  }
  static const bool keep_join = [] { const char* v = exp_knob("MFHIP_SPLIT_JOIN"); return v && std::string(v) == "keep"; }();
  if (!keep_join)  // MFHIP_SPLIT_JOIN=keep: the item keeps replica 0's chain (the others are dropped)
    launch_split_join(s.stream, s.st_split.as<SplitItem>() + sp0, nsplit, s.itf.as<float>(), ctx->P.num_factors);
  MF_HIP(hipGetLastError());
  ctx->stats.updates += ups;
  if (!s.sm_bytes.empty()) ctx->stats.moved_bytes += s.sm_bytes[smod];
}

// One step of the item-block ring after superstep s (1-based) for shard / rank g of G, n = c*G
// blocks: rating block (p, q) hands its item block to (p-1, q) (nextRatingBlock, :611-619), so
// shard g, which just ran item block (g*c + s-1) mod n in its first user block, sends it to
// shard g-1 and receives ((g+1)*c + s-1) mod n from shard g+1.
struct RingStep {
  int32_t out_blk, in_blk, dst, src;
};
RingStep ring_step(int32_t g, int32_t G, int32_t c, int32_t n, int64_t superstep) {
  RingStep r;
  r.out_blk = static_cast<int32_t>((static_cast<int64_t>(g) * c + superstep - 1) % n);
  r.in_blk = static_cast<int32_t>((static_cast<int64_t>((g + 1) % G) * c + superstep - 1) % n);
  r.dst = (g + G - 1) % G;
  r.src = (g + 1) % G;
  return r;
}

// The ring step with the overlap of fast_superstep's split launches: the block leaving shard g
// is the item block of its local block 0, done when launch A is, so it moves on the comm stream
// behind A while launch B (block c-1) still runs; the arriving block is first needed by the next
// superstep's launch B, which waits for ev_moved.
void ring_shift_overlapped(mf_ctx* ctx, int64_t superstep) {
  const int32_t n = ctx->nb;
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  auto bytes_of = [&](int32_t blk, size_t& off, size_t& bytes) {
    const int64_t r0 = ctx->I.block_start[blk], cnt = ctx->I.block_start[blk + 1] - r0;
    off = static_cast<size_t>(r0) * k * ctx->es;
    bytes = static_cast<size_t>(cnt) * k * ctx->es;
  };
  if (ctx->rank_mode) {
    Shard& s = ctx->shards[0];
    DeviceGuard g(s.device);
    const RingStep rs = ring_step(s.index, ctx->G, ctx->c, n, superstep);
    size_t oo, ob, io, ib;
    bytes_of(rs.out_blk, oo, ob);
    bytes_of(rs.in_blk, io, ib);
    char* base = s.itf.as<char>();
    MF_HIP(hipStreamWaitEvent(s.comm, s.ev_front, 0));
    MF_NCCL(ncclGroupStart());
    if (ob > 0) MF_NCCL(ncclSend(base + oo, ob / ctx->es, ncclFloat32, rs.dst, ctx->comm, s.comm));
    if (ib > 0) MF_NCCL(ncclRecv(base + io, ib / ctx->es, ncclFloat32, rs.src, ctx->comm, s.comm));
    MF_NCCL(ncclGroupEnd());
    MF_HIP(hipEventRecord(s.ev_moved, s.comm));
  } else {
    // the sender copies its leaving block into the receiver's slab on its comm stream once its
    // launch A is done; the receiver's next launch B waits for that copy
    for (auto& src : ctx->shards) {
      const RingStep rs = ring_step(src.index, ctx->G, ctx->c, n, superstep);
      Shard& dst = *local_shard(ctx, rs.dst);
      size_t off, bytes;
      bytes_of(rs.out_blk, off, bytes);
      DeviceGuard g(src.device);
      MF_HIP(hipStreamWaitEvent(src.comm, src.ev_front, 0));
      if (bytes > 0)
        MF_HIP(hipMemcpyPeerAsync(dst.itf.as<char>() + off, dst.device, src.itf.as<char>() + off, src.device, bytes,
                                  src.comm));
      MF_HIP(hipEventRecord(src.done, src.comm));
    }
    for (auto& dst : ctx->shards) {
      Shard& src = *local_shard(ctx, ring_step(dst.index, ctx->G, ctx->c, n, superstep).src);
      DeviceGuard g(dst.device);
      MF_HIP(hipStreamWaitEvent(dst.comm, src.done, 0));
      MF_HIP(hipEventRecord(dst.ev_moved, dst.comm));
    }
  }
  for (int32_t g = 0; g < ctx->G; ++g) {
    const RingStep rs = ring_step(g, ctx->G, ctx->c, n, superstep);
    ctx->item_loc[rs.out_blk] = rs.dst;
  }
}

// nextRatingBlock rotation (:611-619) across shards after superstep s.
void ring_shift(mf_ctx* ctx, int64_t superstep) {
  if (ctx->G <= 1) return;
  if (ctx->ring_overlap) {
    ring_shift_overlapped(ctx, superstep);
    return;
  }
  const int32_t n = ctx->nb;
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  auto rows_of = [&](int32_t blk, int64_t& r0, int64_t& cnt) {
    r0 = ctx->I.block_start[blk];
    cnt = ctx->I.block_start[blk + 1] - r0;
  };
  if (ctx->rank_mode) {
    Shard& s = ctx->shards[0];
    DeviceGuard g(s.device);
    const RingStep rs = ring_step(s.index, ctx->G, ctx->c, n, superstep);
    int64_t o0, oc, i0, ic;
    rows_of(rs.out_blk, o0, oc);
    rows_of(rs.in_blk, i0, ic);
    char* base = s.itf.as<char>();
    MF_NCCL(ncclGroupStart());
    if (oc > 0)
      MF_NCCL(ncclSend(base + o0 * k * ctx->es, oc * k, ctx->f64 ? ncclFloat64 : ncclFloat32, rs.dst, ctx->comm,
                       s.stream));
    if (ic > 0)
      MF_NCCL(ncclRecv(base + i0 * k * ctx->es, ic * k, ctx->f64 ? ncclFloat64 : ncclFloat32, rs.src, ctx->comm,
                       s.stream));
    MF_NCCL(ncclGroupEnd());
  } else {
    // in-process shards: peer copy on the sender's stream, receiver waits on an event
    for (auto& src : ctx->shards) {
      DeviceGuard g(src.device);
      MF_HIP(hipEventRecord(src.done, src.stream));
    }
    for (auto& src : ctx->shards) {
      const RingStep rs = ring_step(src.index, ctx->G, ctx->c, n, superstep);
      Shard& dst = *local_shard(ctx, rs.dst);
      int64_t r0, cnt;
      rows_of(rs.out_blk, r0, cnt);
      if (cnt == 0) continue;
      DeviceGuard g(src.device);
      MF_HIP(hipStreamWaitEvent(src.stream, dst.done, 0));  // dst finished superstep s
      const size_t off = static_cast<size_t>(r0) * k * ctx->es, bytes = static_cast<size_t>(cnt) * k * ctx->es;
      MF_HIP(hipMemcpyPeerAsync(dst.itf.as<char>() + off, dst.device, src.itf.as<char>() + off, src.device,
                                bytes, src.stream));
    }
    for (auto& src : ctx->shards) {
      DeviceGuard g(src.device);
      MF_HIP(hipEventRecord(src.done, src.stream));
    }
    for (auto& dst : ctx->shards) {
      Shard& src = *local_shard(ctx, ring_step(dst.index, ctx->G, ctx->c, n, superstep).src);
      DeviceGuard g(dst.device);
      MF_HIP(hipStreamWaitEvent(dst.stream, src.done, 0));
    }
  }
  for (int32_t g = 0; g < ctx->G; ++g) {
    const RingStep rs = ring_step(g, ctx->G, ctx->c, n, superstep);
    ctx->item_loc[rs.out_blk] = rs.dst;
  }
}

// Fixed SoA layout of a DetBuf for at most n entries and nw waves (256-B aligned regions).
struct DetOffsets {
  size_t waves, u, i, qf, r, total;
};
// The pair sweep's plan window for k (plan.hpp pair_window, plan_window_pack): MFHIP_TEST
// pair_window=N overrides the mixed cells' window for the window sweeps (clamped to the ring's
// minimum 2 * pair_ring), run_window=N the single-item cells' (plan.hpp pair_run_window; 0 = the
// same window, forwarded repeats allowed).
int32_t plan_window(int32_t k) {
  int32_t w = pair_window(k), rw = pair_run_window(k);
  if (const std::string v = test_knob("pair_window"); !v.empty())
    w = std::max<int32_t>(2 * pair_ring(pair_kpl(k)), std::atoi(v.c_str()));
  if (const std::string v = test_knob("run_window"); !v.empty()) rw = std::atoi(v.c_str());
  if (rw != 0) rw = std::clamp<int32_t>(rw, w, 0x7FFF);
  return plan_window_pack(w, rw);
}
int64_t det_slot_room(int64_t nw);
DetOffsets det_offsets(int64_t n, int64_t nw) {
  auto up = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
  DetOffsets o;
  const size_t ne = static_cast<size_t>(n + kDetPad);  // the sweep reads whole chunks past a wave's end
  o.waves = 0;
  o.u = up(static_cast<size_t>(det_slot_room(nw)) * sizeof(DetWave));  // room for the split sweep's slot table
  o.i = o.u + up(ne * 4);
  o.qf = o.i + up(ne * 4);
  o.r = o.qf + up(ne * 4);
  o.total = o.r + up(ne * 8);
  return o;
}

// The rating blocks shard s runs in superstep `superstep` and their shuffle seeds
// (new Random(iteration ^ ratingBlockId ^ seed), DSGDforMF.scala:392).
void det_blocks(const mf_ctx* ctx, const Shard& s, int64_t superstep, std::vector<int64_t>& blocks,
                std::vector<int64_t>& seeds) {
  const int32_t n = ctx->nb;
  const int32_t iteration = static_cast<int32_t>(superstep / n);
  blocks.clear();
  seeds.clear();
  for (int32_t j = 0; j < ctx->c; ++j) {
    const int32_t p = s.index * ctx->c + j;
    const int32_t q = static_cast<int32_t>((p + superstep - 1) % n);
    const int64_t b = static_cast<int64_t>(p) * n + q;  // toRatingBlockId (:597-601)
    if (ctx->rb.size(b) == 0) continue;
    blocks.push_back(b);
    seeds.push_back(static_cast<int64_t>(iteration ^ static_cast<int32_t>(b)) ^ ctx->P.seed);
  }
}

// MFHIP_TIMING=1: where a det_run call's host time goes (build time, waits for builds and for
// staging copies), on stderr at the end of the call
struct DetRunClock {
  std::atomic<int64_t> build_ns{0}, builds{0};
};
DetRunClock g_det_clock;
const bool g_det_timing = std::getenv("MFHIP_TIMING") != nullptr;

// The split sweep's slot table (kernels.hpp launch_det_sweep_split), in place over the nw waves of
// build_det_step (the buffer holds det_slot_room(nw)): each single-item wave with its helper slot,
// longest first (block 0 is the hottest chain), then the other waves two per block; empty waves
// dropped.  The chains within half of the longest (at most kDetAlone) bound the superstep, so they
// get a CU each: the dispatcher deals block b to XCD b % 8 and, inside it, CU (b / 8) % (cus / 8),
// so blocks b + cus m share block b's CU (period = the device's CU count, 256 on MI355X) -- those
// positions stay empty (both waves leave at once) while the table has at most max_blocks blocks
// (the co-resident limit: a block past it would never start and the ticket sweep would hang).
// Returns the slot count (even).
int64_t device_cu_count(int dev) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
  return cus;
}
constexpr int64_t kDetAlone = 64;
// H <= period / 2 chains keep their CU, so at most half of the positions are empty: <= 4 nw slots
int64_t det_slot_room(int64_t nw) { return 4 * nw + 4; }
int64_t det_slot_table(DetWave* waves, int64_t nw, int64_t max_blocks, bool alone, int64_t period) {
  period = std::max<int64_t>(period, 8);
  std::vector<DetWave> single, multi;
  for (int64_t w = 0; w < nw; ++w) {
    if (waves[w].count == 0) continue;
    ((waves[w].flags & kDetWaveSingleItem) ? single : multi).push_back(waves[w]);
  }
  std::stable_sort(single.begin(), single.end(), [](const DetWave& a, const DetWave& b) { return a.count > b.count; });
  std::vector<std::array<DetWave, 2>> blocks;
  for (const DetWave& d : single) blocks.push_back({d, DetWave{d.begin, 0, kDetWaveHelper}});
  for (size_t x = 0; x < multi.size(); x += 2)
    blocks.push_back({multi[x], x + 1 < multi.size() ? multi[x + 1] : DetWave{0, 0, 0}});
  if (blocks.empty()) blocks.push_back({DetWave{0, 0, 0}, DetWave{0, 0, 0}});
  int64_t H = 0;  // chains that get a CU each
  if (alone)
    while (H < std::min<int64_t>(kDetAlone, static_cast<int64_t>(single.size())) && 2 * single[H].count >= single[0].count)
      ++H;
  const int64_t nb = static_cast<int64_t>(blocks.size());
  int64_t empties = 0;
  H = std::min(H, period / 2);
  for (int64_t b = period; b < nb + empties; ++b) empties += (b % period) < H;
  if (nb + empties > max_blocks) empties = 0, H = 0;  // no room: the plain order
  MF_REQUIRE(nb <= max_blocks, "det slot table: more blocks than can be resident at once");
  int64_t n = 0, next = 0;
  for (int64_t b = 0; next < nb; ++b) {
    if (b >= period && (b % period) < H) {
      waves[n++] = DetWave{0, 0, 0};
      waves[n++] = DetWave{0, 0, 0};
    } else {
      waves[n++] = blocks[next][0];
      waves[n++] = blocks[next][1];
      ++next;
    }
  }
  return n;
}

// Host side of one superstep for every local shard, into det_buf[slot] (runs on a worker thread
// while the device runs the previous superstep).
void det_build(mf_ctx* ctx, int64_t superstep, int slot) {
  const auto t_build = std::chrono::steady_clock::now();
  struct Done {
    std::chrono::steady_clock::time_point t;
    ~Done() {
      if (g_det_timing) {
        g_det_clock.build_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
        g_det_clock.builds += 1;
      }
    }
  } done{t_build};
  std::vector<int64_t> blocks, seeds;
  if (ctx->det_dev_build || ctx->det_switch.load(std::memory_order_acquire)) {
    // the device builds the entries (det_run): here only each block's JVM shuffle, written as the
    // uploaded permutation, and the superstep index's fixed slot table
    const int64_t sm = (superstep - 1) % ctx->nb;
    for (auto& s : ctx->shards) {
      DetBuf& db = s.det_buf[slot];
      det_blocks(ctx, s, superstep, blocks, seeds);
      db.dev_built = true;
      db.n = s.det_sm_n[sm];
      db.nw = static_cast<int64_t>(s.det_sm_slots[sm].size());
      if (db.n == 0) continue;
      const DetOffsets o = det_offsets(s.det_n_max, s.det_nw_max);
      char* base = db.pin.as<char>();
      std::memcpy(base + o.waves, s.det_sm_slots[sm].data(), static_cast<size_t>(db.nw) * sizeof(DetWave));
      int32_t* ord = reinterpret_cast<int32_t*>(base + o.u);  // (the host path's u region)
      std::vector<int64_t> e0(blocks.size() + 1, 0);
      for (size_t x = 0; x < blocks.size(); ++x) e0[x + 1] = e0[x] + ctx->rb.size(blocks[x]);
      std::vector<uint64_t> rseeds(blocks.size());
      if (!ctx->P.has_seed) {
        std::random_device rd;
        for (auto& v : rseeds) v = (static_cast<uint64_t>(rd()) << 32) ^ rd();
      }
      parallel_tasks(static_cast<int64_t>(blocks.size()), [&](int64_t x) {
        JavaRandom rng(ctx->P.has_seed ? seeds[x] : static_cast<int64_t>(rseeds[x]));
        scala_shuffle(rng, ord + e0[x], e0[x + 1] - e0[x]);  // DSGDforMF.scala:392-393
      });
    }
    return;
  }
  for (auto& s : ctx->shards) {
    DetBuf& db = s.det_buf[slot];
    det_blocks(ctx, s, superstep, blocks, seeds);
    db.dev_built = false;
    db.n = db.nw = 0;
    for (int64_t b : blocks) {
      db.n += ctx->rb.size(b);
      db.nw += s.det_layout.block_waves[b];
    }
    if (db.n == 0) continue;
    const DetOffsets o = det_offsets(s.det_n_max, s.det_nw_max);
    char* base = db.pin.as<char>();
    DetStepOut out{reinterpret_cast<DetWave*>(base + o.waves), reinterpret_cast<uint32_t*>(base + o.u),
                   reinterpret_cast<uint32_t*>(base + o.i), reinterpret_cast<uint32_t*>(base + o.qf),
                   reinterpret_cast<double*>(base + o.r)};
    build_det_step(ctx->rb, ctx->U, ctx->I, s.det_layout, blocks, seeds, ctx->P.has_seed != 0, out, &db.scratch);
    if (ctx->det_split)
      db.nw = det_slot_table(out.waves, db.nw, ctx->det_split_blocks, ctx->det_alone, ctx->det_cu_period);
  }
}

// Deterministic supersteps with the persistent sweep: the host builds supersteps s+1 and s+2
// while the device runs superstep s.
void det_run(mf_ctx* ctx, int64_t count) {
  const int k = ctx->P.num_factors;
  const int64_t s0 = ctx->superstep_done + 1;
  using clk = std::chrono::steady_clock;
  const auto t_run = clk::now();
  const int64_t b_ns0 = g_det_clock.build_ns, b_n0 = g_det_clock.builds;
  int64_t wait_build_ns = 0, wait_copy_ns = 0;
  auto since = [](clk::time_point t) { return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t).count(); };
  auto reclaim = [&](int slot) {  // the staging copy out of this slot's pinned buffer has finished
    const auto t = clk::now();
    for (auto& sh : ctx->shards) {
      DetBuf& db = sh.det_buf[slot];
      if (!db.pending) continue;
      DeviceGuard g(sh.device);
      MF_HIP(hipEventSynchronize(db.copied));
      db.pending = false;
    }
    wait_copy_ns += since(t);
  };
  std::future<void> builds[kDetSlots];
  constexpr int kAhead = kDetSlots - 1;  // supersteps built ahead of the one launched
  // the previous run's speculative builds of supersteps s0 .. s0+kAhead-1 (slots 0 ..) are taken over;
  // any other is joined and dropped (a taken-over build is waited for like the run's own)
  bool prebuilt[kDetSlots] = {};
  for (int slot = 0; slot < kDetSlots; ++slot) {
    const int64_t built = ctx->det_spec_s[slot];
    ctx->det_spec_s[slot] = -1;  // before anything can throw: a slot is never taken over twice
    if (slot < kAhead && slot < count && built == s0 + slot && ctx->det_spec[slot].valid()) {
      builds[slot] = std::move(ctx->det_spec[slot]);  // joined (and its error raised) below, like a fresh build
      prebuilt[slot] = true;
    } else if (ctx->det_spec[slot].valid()) {
      try {
        ctx->det_spec[slot].get();  // a build this run does not use: its failure does not matter
      } catch (...) {
      }
    }
  }
  for (int slot = 0; slot < kDetSlots; ++slot) reclaim(slot);  // a previous call's last copies
  for (int64_t x = 0; x < std::min<int64_t>(count, kAhead); ++x)
    if (!prebuilt[x % kDetSlots])
      builds[x % kDetSlots] = std::async(std::launch::async, det_build, ctx, s0 + x, static_cast<int>(x % kDetSlots));
  for (int64_t x = 0; x < count; ++x) {
    const int64_t s = s0 + x;
    const int slot = static_cast<int>(x % kDetSlots);
    {
      const auto t = clk::now();
      builds[slot].get();  // every superstep of the run has a build (taken over or started here)
      wait_build_ns += since(t);
    }
    // auto mode: when the device has already finished the previous superstep twice in a row by the
    // time its host build is done, the host is the bottleneck (a busy or small host): from then on
    // the builds leave the gather / sorts / scatter to the device (det_device_build), whose host
    // part is the shuffle alone.  Either build gives the same entries, so the factors do not change.
    if (ctx->det_dev_ready && !ctx->det_dev_build && !ctx->det_switch.load() && x >= 2) {
      bool idle = true;
      for (auto& sh : ctx->shards) {
        const DetBuf& pb = sh.det_buf[(slot + kDetSlots - 1) % kDetSlots];
        if (pb.n == 0) continue;
        DeviceGuard g(sh.device);
        idle = idle && hipEventQuery(pb.swept) == hipSuccess;
      }
      ctx->det_idle = idle || ctx->det_mixed ? ctx->det_idle + 1 : 0;
      if (ctx->det_idle >= 2) {
        ctx->det_switch.store(true, std::memory_order_release);
        if (g_det_timing)
          std::fprintf(stderr, "[mfhip] det_run: host builds fell behind at superstep %lld: device builds from now on\n",
                       static_cast<long long>(s));
      }
    }
    const int32_t iteration = static_cast<int32_t>(s / ctx->nb);  // :476
    const double eta = learning_rate(ctx->P.lr_method, ctx->P.learning_rate, iteration + 1, ctx->P.lambda,
                                     ctx->P.lr_arg);  // :383-386
    for (auto& sh : ctx->shards) {
      DetBuf& db = sh.det_buf[slot];
      if (db.n == 0) continue;
      DeviceGuard g(sh.device);
      const DetOffsets o = det_offsets(sh.det_n_max, sh.det_nw_max);
      const char* hp = db.pin.as<char>();
      char* dp = db.dev.as<char>();
      // staging copy on the copy stream, after the sweep that last read this buffer (s-3), so it
      // overlaps the sweeps still running on the compute stream
      MF_HIP(hipStreamWaitEvent(sh.copy_stream, db.swept, 0));
      if (db.dev_built) {
        // the slot table and the shuffle permutation go up; the entries are built on the device
        // (det_device_build), on the same stream
        const int64_t sm = (s - 1) % ctx->nb;
        MF_HIP(hipMemcpyAsync(dp + o.waves, hp + o.waves, static_cast<size_t>(db.nw) * sizeof(DetWave),
                              hipMemcpyHostToDevice, sh.copy_stream));
        MF_HIP(hipMemcpyAsync(sh.det_ord.get(), hp + o.u, static_cast<size_t>(db.n) * 4, hipMemcpyHostToDevice,
                              sh.copy_stream));
        det_device_build(sh.copy_stream, sh.det_bs, sh.det_ord.as<int32_t>(), db.n,
                         sh.det_bt.as<DetBuildBlock>() + static_cast<size_t>(sm) * ctx->c, sh.det_sm_nblk[sm],
                         sh.det_aos_dev.as<DetEntry>(), sh.det_iw.as<int32_t>(), sh.det_wave_bound,
                         static_cast<uint32_t>(ctx->U.rows()), reinterpret_cast<uint32_t*>(dp + o.u),
                         reinterpret_cast<uint32_t*>(dp + o.i), reinterpret_cast<uint32_t*>(dp + o.qf),
                         reinterpret_cast<double*>(dp + o.r));
      } else {
        const std::pair<size_t, size_t> regions[] = {{o.waves, static_cast<size_t>(db.nw) * sizeof(DetWave)},
                                                     {o.u, static_cast<size_t>(db.n) * 4},
                                                     {o.i, static_cast<size_t>(db.n) * 4},
                                                     {o.qf, static_cast<size_t>(db.n) * 4},
                                                     {o.r, static_cast<size_t>(db.n) * 8}};
        for (const auto& rg : regions)
          MF_HIP(hipMemcpyAsync(dp + rg.first, hp + rg.first, rg.second, hipMemcpyHostToDevice, sh.copy_stream));
      }
      MF_HIP(hipEventRecord(db.copied, sh.copy_stream));
      db.pending = true;
      MF_HIP(hipStreamWaitEvent(sh.stream, db.copied, 0));
      MF_HIP(hipMemsetAsync(sh.det_ticket.get(), 0, sh.det_ticket.bytes(), sh.stream));
      LaunchTimer tm(sh, ctx->profiling, true);
      if (ctx->det_split)
        launch_det_sweep_split(sh.stream, reinterpret_cast<const DetWave*>(dp + o.waves), static_cast<int>(db.nw),
                               reinterpret_cast<const uint32_t*>(dp + o.u), reinterpret_cast<const uint32_t*>(dp + o.i),
                               reinterpret_cast<const uint32_t*>(dp + o.qf), reinterpret_cast<const double*>(dp + o.r),
                               sh.uf.as<double>(), sh.itf.as<double>(), sh.uf.bytes(), sh.itf.bytes(),
                               sh.regu.as<double>(), sh.regi.as<double>(), k, eta, sh.det_ticket.as<int32_t>(),
                               sh.det_err.as<int32_t>(), tm.start(), tm.stop());
      else
        launch_det_sweep(sh.stream, reinterpret_cast<const DetWave*>(dp + o.waves), static_cast<int>(db.nw),
                         reinterpret_cast<const uint32_t*>(dp + o.u), reinterpret_cast<const uint32_t*>(dp + o.i),
                         reinterpret_cast<const uint32_t*>(dp + o.qf), reinterpret_cast<const double*>(dp + o.r),
                         sh.uf.as<double>(), sh.itf.as<double>(), sh.uf.bytes(), sh.itf.bytes(), sh.regu.as<double>(),
                         sh.regi.as<double>(), k, eta, sh.det_ticket.as<int32_t>(),
                         sh.det_scratch.as<int32_t>(), sh.det_err.as<int32_t>(), tm.start(), tm.stop());
      MF_HIP(hipGetLastError());
      MF_HIP(hipEventRecord(db.swept, sh.stream));
      ctx->stats.updates += db.n;
      ctx->stats.kernel_launches += 1;
      // rows: user in + out and item in + out per update (an upper bound: an item row kept in
      // registers across consecutive entries of its item moves once); per update the 20-B entry,
      // two lambda/omega doubles and the ticket poll + store
      ctx->stats.moved_bytes += 8.0 * k * static_cast<double>(4 * db.n) + 44.0 * db.n;
    }
    ring_shift(ctx, s);
    ctx->superstep_done = s;
    ctx->stats.supersteps++;
    if (x + kAhead < count) {  // superstep s+kAhead goes where s-1 was staged: its copy must be done
      const int other = static_cast<int>((x + kAhead) % kDetSlots);
      reclaim(other);
      builds[other] = std::async(std::launch::async, det_build, ctx, s + kAhead, other);
    }
  }
  ctx->stats.algorithmic_bytes = static_cast<double>(ctx->stats.updates) * bytes_per_update(ctx);
  if (g_det_timing)
    std::fprintf(stderr,
                 "[mfhip] det_run: %lld supersteps enqueued in %.1f ms; waited %.1f ms for host builds, %.1f ms for "
                 "staging copies; %lld builds finished meanwhile, %.2f ms each\n",
                 static_cast<long long>(count), since(t_run) / 1e6, wait_build_ns / 1e6, wait_copy_ns / 1e6,
                 static_cast<long long>(g_det_clock.builds - b_n0),
                 g_det_clock.builds > b_n0 ? (g_det_clock.build_ns - b_ns0) / 1e6 / (g_det_clock.builds - b_n0) : 0.0);
  if (g_det_timing && g_det_clock.builds > 0)
    std::fprintf(stderr, "[mfhip] det builds so far, ms each: shuffle %.2f gather %.2f prefix %.2f scatter %.2f flags %.2f\n",
                 det_build_phase_ns(0) / 1e6 / g_det_clock.builds, det_build_phase_ns(1) / 1e6 / g_det_clock.builds,
                 det_build_phase_ns(2) / 1e6 / g_det_clock.builds, det_build_phase_ns(3) / 1e6 / g_det_clock.builds,
                 det_build_phase_ns(4) / 1e6 / g_det_clock.builds);
  // the next run's first supersteps, built in the background while the caller syncs, evaluates or
  // returns: a run's start no longer waits for its first host build (~36 ms of an NFLX call).  A builder
  // first waits for the staging copy that last read its slot's pinned buffer.
  for (int64_t x = 0; x < kAhead; ++x) {
    const int slot = static_cast<int>(x);
    const int64_t s = s0 + count + x;
    ctx->det_spec[slot] = std::async(std::launch::async, [ctx, slot, s] {
      for (auto& sh : ctx->shards) {
        if (!sh.det_buf[slot].copied) continue;
        DeviceGuard g(sh.device);
        MF_HIP(hipEventSynchronize(sh.det_buf[slot].copied));
      }
      det_build(ctx, s, slot);
    });
    ctx->det_spec_s[slot] = s;
  }
}

void run_supersteps(mf_ctx* ctx, int64_t count) {
  MF_REQUIRE(ctx->prepared, "mf_dsgd_run before mf_dsgd_prepare");
  require_healthy(ctx);
  if (ctx->f64 && ctx->det_sweep) {
    if (count > 0) det_run(ctx, count);
    return;
  }
  for (int64_t x = 0; x < count; ++x) {
    const int64_t s = ctx->superstep_done + 1;
    const int32_t iteration = static_cast<int32_t>(s / ctx->nb);  // getSuperstepNumber / numBlocks (:476)
    const double eta = learning_rate(ctx->P.lr_method, ctx->P.learning_rate, iteration + 1, ctx->P.lambda,
                                     ctx->P.lr_arg);  // :383-386
    for (auto& sh : ctx->shards) {
      if (ctx->f64) det_superstep(ctx, sh, s, iteration, eta);
      else fast_superstep(ctx, sh, s, eta);
    }
    ring_shift(ctx, s);
    ctx->superstep_done = s;
    ctx->stats.supersteps++;
  }
  ctx->stats.algorithmic_bytes = static_cast<double>(ctx->stats.updates) * bytes_per_update(ctx);
}

void reset_item_loc(mf_ctx* ctx) {
  ctx->item_loc.assign(ctx->nb, 0);
  for (int32_t q = 0; q < ctx->nb; ++q) ctx->item_loc[q] = q / ctx->c;
  for (int64_t s = 1; s <= ctx->superstep_done; ++s)
    if (ctx->G > 1)
      for (int32_t g = 0; g < ctx->G; ++g) {
        const RingStep rs = ring_step(g, ctx->G, ctx->c, ctx->nb, s);
        ctx->item_loc[rs.out_blk] = rs.dst;
      }
}

// MFHIP_TIMING=1: host phases of prepare on stderr.
struct PhaseClock {
  bool on = std::getenv("MFHIP_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[mfhip] %-28s %10.3f ms\n", what, 1e3 * std::chrono::duration<double>(now - t).count());
    t = now;
  }
};

// The device build of the det sweep's input (kernels.hpp det_device_build): per shard, the rating
// blocks' records and item -> wave maps on the device, and per superstep index its block table and
// wave / slot table.  A wave's entries are its items' ratings of the block, so its count -- and
// with it the wave table and the slot table -- is the same every time the block comes round; only
// the order inside the waves (the shuffle) changes.
void prepare_det_device_build(mf_ctx* ctx) {
  const int32_t n = ctx->nb;
  const DetEntry* aos = ctx->rb.det_aos.data();
  const int64_t total = static_cast<int64_t>(ctx->rb.det_aos.size());
  for (auto& s : ctx->shards) {
    DeviceGuard g(s.device);
    const DetSweepLayout& L = s.det_layout;
    const int64_t nb2 = static_cast<int64_t>(n) * n;
    // per rating block of this shard: its wave counts and its item -> wave map's offset
    std::vector<std::vector<int64_t>> wcnt(nb2);
    std::vector<int64_t> iwoff(nb2, -1);
    std::vector<int32_t> iw;
    for (int64_t b = 0; b < nb2; ++b)
      if (L.block_waves[b] > 0 && !L.item_wave[b].empty()) {
        iwoff[b] = static_cast<int64_t>(iw.size());
        iw.insert(iw.end(), L.item_wave[b].begin(), L.item_wave[b].end());
      }
    parallel_tasks(nb2, [&](int64_t b) {
      if (L.block_waves[b] <= 0 || ctx->rb.size(b) == 0) return;
      const int64_t i0 = ctx->I.block_start[b % n];
      wcnt[b].assign(L.block_waves[b], 0);
      for (int64_t e = ctx->rb.start[b]; e < ctx->rb.start[b + 1]; ++e) wcnt[b][L.item_wave[b][aos[e].i - i0]]++;
    });
    s.det_sm_slots.assign(n, {});
    s.det_sm_n.assign(n, 0);
    s.det_sm_nblk.assign(n, 0);
    std::vector<DetBuildBlock> bt(static_cast<size_t>(n) * std::max(ctx->c, 1));
    std::vector<int64_t> blocks, seeds;
    for (int32_t sm = 0; sm < n; ++sm) {
      det_blocks(ctx, s, sm + 1, blocks, seeds);  // the blocks of superstep s depend on (s-1) mod n
      std::vector<DetWave> waves;
      int64_t e0 = 0;
      for (size_t x = 0; x < blocks.size(); ++x) {
        const int64_t b = blocks[x];
        MF_REQUIRE(iwoff[b] >= 0 && static_cast<int64_t>(wcnt[b].size()) == L.block_waves[b],
                   "det device build: a block without its wave layout");
        bt[static_cast<size_t>(sm) * ctx->c + x] =
            DetBuildBlock{e0, ctx->rb.start[b], iwoff[b], static_cast<uint32_t>(ctx->I.block_start[b % n]),
                          static_cast<uint32_t>(waves.size())};
        int64_t at = e0;
        for (int32_t w = 0; w < L.block_waves[b]; ++w) {
          waves.push_back(DetWave{at, static_cast<int32_t>(wcnt[b][w]), L.wave_single[b][w] ? kDetWaveSingleItem : 0});
          at += wcnt[b][w];
        }
        e0 = at;
      }
      const int64_t nw = static_cast<int64_t>(waves.size());
      waves.resize(static_cast<size_t>(det_slot_room(nw)));
      const int64_t nslots =
          ctx->det_split ? det_slot_table(waves.data(), nw, ctx->det_split_blocks, ctx->det_alone, ctx->det_cu_period)
                         : nw;
      waves.resize(static_cast<size_t>(nslots));
      s.det_sm_slots[sm] = std::move(waves);
      s.det_sm_n[sm] = e0;
      s.det_sm_nblk[sm] = static_cast<int32_t>(blocks.size());
    }
    s.det_aos_dev.alloc(static_cast<size_t>(std::max<int64_t>(total, 1)) * sizeof(DetEntry));
    if (total > 0)
      MF_HIP(hipMemcpy(s.det_aos_dev.get(), aos, static_cast<size_t>(total) * sizeof(DetEntry), hipMemcpyHostToDevice));
    s.det_iw.alloc(std::max<size_t>(iw.size(), 1) * 4);
    if (!iw.empty()) MF_HIP(hipMemcpy(s.det_iw.get(), iw.data(), iw.size() * 4, hipMemcpyHostToDevice));
    s.det_bt.alloc(bt.size() * sizeof(DetBuildBlock));
    MF_HIP(hipMemcpy(s.det_bt.get(), bt.data(), bt.size() * sizeof(DetBuildBlock), hipMemcpyHostToDevice));
    s.det_ord.alloc(static_cast<size_t>(std::max<int64_t>(s.det_n_max, 1)) * 4);
    s.det_wave_bound = static_cast<uint32_t>(std::max<int64_t>(s.det_nw_max, 1));
    det_device_build_reserve(s.det_bs, s.det_n_max, s.det_wave_bound, static_cast<uint32_t>(ctx->U.rows()));
  }
}

// Deterministic mode: the persistent sweep's item -> wave layout and staging buffers, unless
// MFHIP_TEST det_kernel=level (one launch per dependency level, det_superstep) or the device
// cannot hold a superstep's waves.  Waves per superstep and shard: half the device's resident
// capacity (shared by the shards on that device; MFHIP_TEST det_waves= overrides).
void prepare_det_sweep(mf_ctx* ctx) {
  if (test_knob("det_kernel") == "level") return;
  // single-item chains split over two waves where k allows (MFHIP_TEST det_split=0: one wave each)
  const bool split = test_knob("det_split") != "0" && det_split_capacity(ctx->P.num_factors) > 0;
  int cap = 1 << 30;
  for (auto& s : ctx->shards) {
    DeviceGuard g(s.device);
    int sharers = 0;
    for (auto& o : ctx->shards) sharers += o.device == s.device;
    if (const char* v = std::getenv("MFHIP_DEVICE_SHARERS"))
      if (ctx->rank_mode) sharers = std::max(sharers, std::atoi(v));
    // in wave slots; the split sweep's helpers take one each, at most one per wave of the layout
    // (waves = cap / 2 below), so the slot table stays within the resident capacity
    cap = std::min(cap, (split ? det_split_capacity(ctx->P.num_factors) : det_sweep_capacity(ctx->P.num_factors)) /
                            std::max(1, sharers));
  }
  if (cap < 1) return;
  const uint64_t k8 = static_cast<uint64_t>(ctx->P.num_factors) * 8;
  if (static_cast<uint64_t>(ctx->U.rows()) * k8 >= 0xFFFFF000ull || static_cast<uint64_t>(ctx->I.rows()) * k8 >= 0xFFFFF000ull)
    return;  // the sweep addresses each f64 slab with 32-bit offsets
  // k not a multiple of 64: lanes past k use voffset 0x80000000, and with the out-of-range row
  // offset kOOB in soffset the 32-bit sum wraps to 0x7FFFF000 -- inside a slab of 2 GiB or more
  if (ctx->P.num_factors % 64 != 0 &&
      (static_cast<uint64_t>(ctx->U.rows()) * k8 >= 0x7FFFF000ull || static_cast<uint64_t>(ctx->I.rows()) * k8 >= 0x7FFFF000ull))
    return;
  int32_t waves = std::max(1, cap / 2);
  // the split sweep's slot table holds at most one block (two slots) per wave of the layout, and
  // at most cap / 2 blocks are resident: so at most cap / 2 waves there
  if (const std::string v = test_knob("det_waves"); !v.empty())
    waves = std::clamp(std::atoi(v.c_str()), 1, split ? std::max(1, cap / 2) : cap);
  const int32_t n = ctx->nb;
  {  // the build's shuffle-order gather reads one 16-B record per rating
    const int64_t total = ctx->rb.start.empty() ? 0 : ctx->rb.start.back();
    resize_huge(ctx->rb.det_aos, static_cast<size_t>(total));  // random reads: fewer TLB misses
    DetEntry* a = ctx->rb.det_aos.data();
    parallel_for(total, [&](int64_t b, int64_t e, int) {
      for (int64_t x = b; x < e; ++x) a[x] = DetEntry{ctx->rb.urow[x], ctx->rb.irow[x], ctx->rb.r[x]};
    });
  }
  for (auto& s : ctx->shards) {
    build_det_layout(s.det_layout, ctx->rb, ctx->U, ctx->I, ctx->c, s.index, waves);
    s.det_n_max = s.det_nw_max = 0;
    for (int32_t sm = 0; sm < n; ++sm) {
      int64_t cnt = 0, nw = 0;
      for (int32_t j = 0; j < ctx->c; ++j) {
        const int32_t p = s.index * ctx->c + j;
        const int64_t b = static_cast<int64_t>(p) * n + (p + sm) % n;
        cnt += ctx->rb.size(b);
        nw += s.det_layout.block_waves[b];
      }
      s.det_n_max = std::max(s.det_n_max, cnt);
      s.det_nw_max = std::max(s.det_nw_max, nw);
    }
    DeviceGuard g(s.device);
    const size_t bytes = std::max<size_t>(det_offsets(s.det_n_max, s.det_nw_max).total, 256);
    for (auto& db : s.det_buf) {
      if (db.pending) { MF_HIP(hipEventSynchronize(db.copied)); db.pending = false; }
      db.pin.alloc(bytes);
      db.dev.alloc(bytes);
    }
    s.det_ticket.alloc(static_cast<size_t>(std::max<int64_t>(ctx->U.rows(), 1)) * 4);
    s.det_scratch.alloc(static_cast<size_t>(s.det_nw_max) * 64);  // one scratch line per wave
    s.det_err.alloc(16);
    MF_HIP(hipMemsetAsync(s.det_err.get(), 0, 16, s.stream));
  }
  // the sweep's host build reads only det_aos from here on: release the (user row, item row,
  // rating) arrays it was made from (16 B per rating; ~11.5 GB at full YAHOO)
  ctx->reaper.drop(ctx->rb.urow);
  ctx->reaper.drop(ctx->rb.irow);
  ctx->reaper.drop(ctx->rb.r);
  ctx->reaper.release();
  ctx->det_sweep = true;
  ctx->det_split = split;
  ctx->det_split_blocks = cap / 2;
  ctx->det_alone = test_knob("det_alone") != "0";
  ctx->det_cu_period = device_cu_count(ctx->shards[0].device);
  // The sweep's input is built on the host while the device keeps up with it; the device build
  // (4% slower on a free host: its traffic slows the running chain, profiles/r06_det_device_build_ab.txt)
  // takes over when the host falls behind (det_run).  MFHIP_TEST det_build=device / host: always
  // that one; mixed: the switch from the third superstep on (tests).
  const std::string dbk = test_knob("det_build");
  ctx->det_dev_build = dbk == "device";
  ctx->det_dev_ready = dbk != "host";
  ctx->det_mixed = dbk == "mixed";
  ctx->det_switch = false;
  ctx->det_idle = 0;
  if (ctx->det_dev_ready) prepare_det_device_build(ctx);
}

void prepare(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n) {
  MF_REQUIRE(n >= 0, "negative rating count");
  MF_REQUIRE(n == 0 || (u && i && r), "null rating arrays");
  det_spec_wait(ctx, true);
  ctx->failed.clear();
  sync_all(ctx);
  PhaseClock clk;
  ctx->item_split = 0;
  if (const char* v = exp_knob("MFHIP_ITEM_SPLIT")) ctx->item_split = std::max(0, std::atoi(v));  // replicas
  ctx->reaper.join();
  DevRatingBlocks dev_rb;  // the device copy of the rating blocks (full device schedule only)
  ctx->nb = std::max(1, ctx->P.num_blocks);
  MF_REQUIRE(ctx->nb % ctx->G == 0, "num_blocks must be a multiple of the device count");
  ctx->c = ctx->nb / ctx->G;
  int32_t lo = 0, hi = ctx->nb;
  if (ctx->rank_mode) { lo = ctx->shards[0].index * ctx->c; hi = lo + ctx->c; }
  // the reference's seeded blocking runs on the device (MFHIP_TEST host_blocking=1: on the host)
  const std::string hb = test_knob("host_blocking");
  const bool on_device = ctx->P.has_seed && (ctx->f64 || ctx->P.fast_blocking == MF_BLOCKING_REFERENCE) &&
                         !(!hb.empty() && hb != "0") && n < (int64_t{1} << 31);
  if (on_device) {
    Shard& s0 = ctx->shards[0];
    DeviceGuard g(s0.device);
    const std::string dpv0 = test_knob("device_plan");
    const bool keep = !ctx->f64 && ctx->shards.size() == 1 && ctx->item_split == 0 &&
                      choose_fast_kernel(ctx->P.num_factors) == FastKernel::kPair && dpv0 != "0" && dpv0 != "1";
    device_blocking(s0.stream, u, i, r, n, ctx->nb, ctx->P.seed, lo, hi, ctx->f64, ctx->U, ctx->I, ctx->rb,
                    keep ? &dev_rb : nullptr, !keep);
    clk.lap("blocking + rating blocks (device)");
  }
  build_model(ctx, u, i, n, on_device);
  clk.lap("factor init + H2D");
  if (!on_device) {
    build_rating_blocks(ctx->rb, ctx->U, ctx->I, u, i, r, n, lo, hi, ctx->f64 && ctx->P.has_seed);
    clk.lap("rating blocks");
  }
  const int64_t nb2 = static_cast<int64_t>(ctx->nb) * ctx->nb;
  ctx->det_sweep = false;
  ctx->ring_overlap = false;
  if (ctx->f64) prepare_det_sweep(ctx);
  clk.lap("deterministic sweep layout");
  if (!ctx->f64) {
    const int64_t local = ctx->rb.start[nb2];
    const int64_t blocks_local = static_cast<int64_t>(hi - lo) * ctx->nb;
    const FastKernel fk = choose_fast_kernel(ctx->P.num_factors);
    ctx->G_fast = choose_groups(local / std::max<int64_t>(blocks_local, 1), ctx->c, ctx->P.fast_waves,
                                fk == FastKernel::kPair ? 40.0 : 150.0, fk == FastKernel::kPair ? 1024 : 2048);
    FastPlan fp;
    const uint32_t dummy = static_cast<uint32_t>(ctx->U.rows());  // zeroed row used by padding records
    MF_REQUIRE(static_cast<uint64_t>(ctx->U.rows() + 2) * ctx->P.num_factors * 4 < (1ull << 32) &&
                   static_cast<uint64_t>(ctx->I.rows() + 1) * ctx->P.num_factors * 4 < (1ull << 32),
               "fast mode addresses each factor slab with 32-bit offsets (< 4 GiB)");
    const int k = ctx->P.num_factors;
    ctx->fast_pair = fk == FastKernel::kPair;
    ctx->fast_sys = false;
    std::vector<int32_t> block_groups;  // systolic sweep, automatic G: one G_j per rating block
    int64_t sys_cap = 0;                // blocks of one systolic launch that can be resident at once
    if (ctx->fast_pair && want_pair_sys()) {
      int cap = 1 << 30, simds = 1 << 30;
      for (auto& s : ctx->shards) {
        DeviceGuard g(s.device);
        int cus = 0;
        MF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.device));
        cap = std::min(cap, sweep_pair_sys_capacity(k));
        simds = std::min(simds, 4 * cus);
      }
      // the group model's wave budget: one wave per SIMD.  (With the round-4 ring of 7 pairs a budget
      // of two waves per CU at k <= 128 and three at k = 256 was faster -- a pair step slowed sharply
      // with the waves sharing its CU; with the per-width rings of round 5 (plan.hpp pair_ring) the
      // model's own choice is best again: NFLX 20.0 ms with 656 waves vs 20.24 with 512, YAHOO 223.7
      // vs 232.0 ms with 1004 vs 768; profiles/r05_wave_budget.txt.)
      if (const std::string v = test_knob("sys_waves"); !v.empty()) simds = std::max(8, std::atoi(v.c_str()));
      if (ctx->P.fast_waves == 0 && test_knob("block_groups") != "0") {
        block_groups.assign(nb2, 0);
        for (auto& s : ctx->shards) {
          std::vector<int32_t> gb;
          if (ctx->rb.urow.empty() && dev_rb.urow.get()) {  // rating blocks on the device only
            DeviceGuard g(s.device);
            std::vector<int64_t> size(nb2, 0);
            for (int64_t b = 0; b < nb2; ++b) size[b] = ctx->rb.size(b);
            gb = choose_block_groups(size, device_block_tops(s.stream, dev_rb, ctx->rb, ctx->I), ctx->nb, ctx->c,
                                     s.index, simds, sys_cell_ns(k), sys_run_pair_ns(k));
          } else {
            gb = choose_block_groups(ctx->rb, ctx->I, ctx->c, s.index, simds, ctx->item_split, sys_cell_ns(k),
                                     sys_run_pair_ns(k));
          }
          for (int64_t b = 0; b < nb2; ++b)
            if (gb[b] > 0) block_groups[b] = gb[b];
        }
      }
      // every wave of a superstep must be resident at once -- on a device shared by several
      // shards (their streams run concurrently) or, in rank mode, by MFHIP_DEVICE_SHARERS ranks
      // (the one-GPU rehearsal of the ring), all of theirs together
      if (const char* v = std::getenv("MFHIP_DEVICE_SHARERS"))
        if (ctx->rank_mode && std::atoi(v) > 1) cap /= std::atoi(v);
      sys_cap = cap;
      bool fits = cap > 0;
      for (int32_t sm = 0; sm < ctx->nb && fits; ++sm) {
        std::vector<std::pair<int, int64_t>> per_dev;  // (device, waves of superstep sm)
        for (auto& s : ctx->shards) {
          int64_t waves = 0;
          for (int32_t j = 0; j < ctx->c; ++j) {
            const int32_t p = s.index * ctx->c + j;
            const int64_t b = static_cast<int64_t>(p) * ctx->nb + (p + sm) % ctx->nb;
            waves += block_groups.empty() || block_groups[b] == 0 ? ctx->G_fast : block_groups[b];
          }
          auto it = std::find_if(per_dev.begin(), per_dev.end(), [&](const auto& e) { return e.first == s.device; });
          if (it == per_dev.end()) per_dev.emplace_back(s.device, waves);
          else it->second += waves;
        }
        for (const auto& e : per_dev) fits = fits && e.second <= cap;
      }
      ctx->fast_sys = fits;
      if (!fits) block_groups.clear();
    }
    clk.lap("schedule model (groups)");
    // the per-cell emission and the pair records on the device (kernels_plan.hip) for the default
    // systolic pair sweep of one shard; MFHIP_TEST device_plan=0 keeps them on the host
    const std::string dpv = test_knob("device_plan");
    // (a rank whose user blocks hold no rating -- the reference's blocking can leave a block
    // empty -- plans on the host: its schedule is empty)
    const bool dev_plan = ctx->fast_pair && ctx->fast_sys && ctx->item_split == 0 &&
                          ctx->shards.size() == 1 && ctx->rb.start[nb2] > 0 && dpv != "0";
    std::vector<FastBlockWork> entries;
    PairPlan dev_pp;
    DevBuf dev_pairs;
    // MFHIP_TEST device_plan: unset / 2 = the whole schedule on the device, 1 = host phase 1 + device
    // emission, 0 = host
    const bool dev_full = dev_plan && dev_rb.total == ctx->rb.start[nb2] && dev_rb.urow.get();
    if (dev_full) {
      std::vector<int32_t> Gb(nb2, ctx->G_fast);
      if (!block_groups.empty())
        for (int64_t b = 0; b < nb2; ++b) Gb[b] = block_groups[b] > 0 ? block_groups[b] : ctx->G_fast;
      Shard& s0 = ctx->shards[0];
      DeviceGuard g(s0.device);
      device_fast_schedule(s0.stream, dev_rb, ctx->rb, ctx->U, ctx->I, Gb, ctx->P.lambda,
                           static_cast<uint64_t>(ctx->P.seed) * 0x9E3779B97F4A7C15ULL + 1, fp, ctx->c, s0.index, k,
                           dummy, plan_window(k), dev_pp, dev_pairs);
      dev_rb = DevRatingBlocks();
    } else {
      if (ctx->rb.urow.empty() && dev_rb.urow.get()) {  // a host-built plan after all
        Shard& s0 = ctx->shards[0];
        DeviceGuard g(s0.device);
        fetch_rating_blocks(s0.stream, dev_rb, ctx->rb);
      }
      build_fast_plan(fp, ctx->rb, ctx->U, ctx->I, ctx->G_fast, k, ctx->P.lambda,
                      static_cast<uint64_t>(ctx->P.seed) * 0x9E3779B97F4A7C15ULL + 1, dummy, nullptr,
                      ctx->fast_pair ? plan_window(k) : kHazardWindow, block_groups.empty() ? nullptr : &block_groups,
                      ctx->item_split, static_cast<uint32_t>(ctx->I.rows() + 1), dev_plan ? &entries : nullptr);
    }
    MF_REQUIRE(static_cast<uint64_t>(ctx->I.rows() + 1 + fp.scratch_rows) * k * 4 < (1ull << 32),
               "hot-item replica rows exceed the 32-bit item slab offsets");
    if (dev_plan && !dev_full) {
      Shard& s0 = ctx->shards[0];
      DeviceGuard g(s0.device);
      clk.lap("cell order (host)");
      device_pair_schedule(s0.stream, entries, fp, ctx->nb, ctx->c, s0.index, k, dummy, plan_window(k), false, dev_pp,
                           dev_pairs);
      ctx->reaper.drop(entries);
    }
    ctx->stats.pads = fp.pads;
    ctx->reaper.drop(fp.scratch);
    clk.lap(dev_full ? "schedule (device)" : dev_plan ? "cell emission + pairs (device)" : "cell plan");
    {  // priority threshold: 3x the mean non-empty cell length
      int64_t cells = 0, recs = 0;
      for (int64_t b = 0; b < nb2; ++b)
        if (fp.cell_base[b] >= 0) {
          const int32_t* o = fp.cell_off.data() + fp.cell_base[b];
          const int64_t gg = static_cast<int64_t>(fp.Gb[b]) * fp.Gb[b];
          for (int64_t c2 = 0; c2 < gg; ++c2) cells += o[c2 + 1] > o[c2];
          recs += o[gg];
        }
      ctx->fast_prio_len = cells ? static_cast<int32_t>(std::max<int64_t>(16, 3 * recs / cells)) : (1 << 30);
      if (const char* v = exp_knob("MFHIP_PRIO_LEN")) ctx->fast_prio_len = std::atoi(v);
    }
    ctx->fast_rb_size.assign(nb2, 0);
    for (int64_t b = 0; b < nb2; ++b) ctx->fast_rb_size[b] = ctx->rb.size(b);
    ctx->stats.groups = ctx->G_fast;
    if (!block_groups.empty()) {  // report the mean G_j of the non-empty rating blocks
      int64_t sum = 0, cnt = 0;
      for (int64_t b = 0; b < nb2; ++b)
        if (fp.cell_base[b] >= 0) { sum += fp.Gb[b]; ++cnt; }
      ctx->stats.groups = cnt ? static_cast<int32_t>((sum + cnt / 2) / cnt) : ctx->G_fast;
    }
    ctx->fast_dummy_u = dummy;
    ctx->fast_dummy_i = static_cast<uint32_t>(ctx->I.rows());
    {
      ctx->ring_overlap = ctx->fast_pair && ctx->fast_sys && ctx->G > 1 && ctx->c >= 2 &&
                          ctx->item_split == 0 && test_knob("ring_overlap") != "0";
    }
    for (auto& s : ctx->shards) {
      ensure_rows(ctx, s, kSideU, ctx->U.rows() + 2);
      ensure_rows(ctx, s, MF_SIDE_ITEM, ctx->I.rows() + 1 + fp.scratch_rows);
      DeviceGuard g(s.device);
      {  // hot-item replicas of this shard's rating blocks, per superstep
        std::vector<SplitItem> tab;
        s.st_split_off.assign(ctx->nb + 1, 0);
        for (int32_t sm = 0; sm < ctx->nb; ++sm) {
          for (int32_t j = 0; j < ctx->c; ++j) {
            const int32_t p = s.index * ctx->c + j;
            const int64_t b = static_cast<int64_t>(p) * ctx->nb + (p + sm) % ctx->nb;
            tab.insert(tab.end(), fp.splits.begin() + fp.split_off[b], fp.splits.begin() + fp.split_off[b + 1]);
          }
          s.st_split_off[sm + 1] = static_cast<int64_t>(tab.size());
        }
        s.st_split.alloc(std::max<size_t>(tab.size(), 1) * sizeof(SplitItem));
        if (!tab.empty())
          MF_HIP(hipMemcpy(s.st_split.get(), tab.data(), tab.size() * sizeof(SplitItem), hipMemcpyHostToDevice));
      }
      const size_t row_bytes = static_cast<size_t>(ctx->P.num_factors) * ctx->es;
      MF_HIP(hipMemsetAsync(s.uf.as<char>() + static_cast<size_t>(dummy) * row_bytes, 0, 2 * row_bytes, s.stream));
      MF_HIP(hipMemsetAsync(s.itf.as<char>() + static_cast<size_t>(ctx->fast_dummy_i) * row_bytes, 0, row_bytes,
                            s.stream));
      if (ctx->fast_pair) {
        PairPlan pp;
        if (dev_plan) {
          pp = std::move(dev_pp);
          s.st_recs = std::move(dev_pairs);
        } else {
          build_pair_plan(pp, fp, ctx->nb, ctx->c, s.index, k, !ctx->fast_sys);
        }
        ctx->stats.pads += pp.noop_halves - fp.pads;  // run padding on top of the planner's
        s.sm_bytes = pp.sm_bytes;
        s.st_nrecs = 0;
        for (const WaveDesc& wd : pp.waves) s.st_nrecs = std::max<int64_t>(s.st_nrecs, wd.base + wd.steps);
        if (!dev_plan) s.st_recs.alloc(std::max<size_t>(pp.recs.size(), 1) * sizeof(PairRec));
        s.st_waves.alloc(std::max<size_t>(pp.waves.size(), 1) * sizeof(WaveDesc));
        if (!pp.recs.empty())
          MF_HIP(hipMemcpy(s.st_recs.get(), pp.recs.data(), pp.recs.size() * sizeof(PairRec), hipMemcpyHostToDevice));
        if (!pp.waves.empty())
          MF_HIP(hipMemcpy(s.st_waves.get(), pp.waves.data(), pp.waves.size() * sizeof(WaveDesc), hipMemcpyHostToDevice));
        s.st_sub_off = std::move(pp.sub_off);
        s.st_sys_host.clear();
        s.sys_base = 0;
        if (ctx->fast_sys) {
          s.st_sys.alloc(std::max<size_t>(pp.sys.size(), 1) * sizeof(WaveDesc));
          if (!pp.sys.empty())
            MF_HIP(hipMemcpy(s.st_sys.get(), pp.sys.data(), pp.sys.size() * sizeof(WaveDesc), hipMemcpyHostToDevice));
          s.st_sysw.alloc(std::max<size_t>(pp.sys_waves.size(), 1) * sizeof(SysWave));
          if (!pp.sys_waves.empty())
            MF_HIP(hipMemcpy(s.st_sysw.get(), pp.sys_waves.data(), pp.sys_waves.size() * sizeof(SysWave),
                             hipMemcpyHostToDevice));
          s.st_sys_off = pp.sys_off;
          s.st_sys_block_off = pp.sys_block_off;
          s.st_place.release();
          s.st_place_off.assign(ctx->nb + 1, 0);
          s.st_place_pad.assign(ctx->nb, 0);
          if (test_knob("sys_place") != "0" && !pp.sys_waves.empty()) {
            // empty blocks isolate each XCD's heaviest wave (one launch per superstep, one shard:
            // the co-residency check above counted this shard's waves alone); MFHIP_TEST sys_iso=N:
            // its N heaviest (0: none).  Default: k <= 128 (NFLX -0.7%, ML20M even; YAHOO's four-wave
            // CUs lose 0.3% to the slots the empty blocks take, profiles/r06_sys_isolation_ab.txt)
            int32_t iso = !ctx->ring_overlap && ctx->shards.size() == 1 && k <= 128 ? 1 : 0;
            if (const std::string v = test_knob("sys_iso"); !v.empty() && iso) iso = std::clamp(std::atoi(v.c_str()), 0, 8);
            for (int32_t sm = 0; sm < ctx->nb; ++sm) {
              const int64_t nw = pp.sys_off[sm + 1] - pp.sys_off[sm];
              s.st_place_pad[sm] = iso ? sys_iso_pad(nw, sys_cap, iso) : 0;
              s.st_place_off[sm + 1] = s.st_place_off[sm] + nw + 8 * s.st_place_pad[sm];
            }
            std::vector<int32_t> place(static_cast<size_t>(s.st_place_off[ctx->nb]), 0);
            for (int32_t sm = 0; sm < ctx->nb; ++sm) {
              const int64_t w0 = pp.sys_off[sm], nw = pp.sys_off[sm + 1] - w0, out = s.st_place_off[sm];
              if (ctx->ring_overlap) {  // the two launches of fast_superstep
                const int64_t split = pp.sys_block_off[static_cast<size_t>(sm) * (ctx->c + 1) + ctx->c - 1];
                sys_placement(pp, w0, 0, split, place, out);
                sys_placement(pp, w0, split, nw, place, out + split);
              } else {
                sys_placement(pp, w0, 0, nw, place, out, s.st_place_pad[sm]);
              }
              // per launch: every wave exactly once, the rest empty (a missing wave would stall its
              // neighbours)
              const int64_t cut = ctx->ring_overlap
                                      ? pp.sys_block_off[static_cast<size_t>(sm) * (ctx->c + 1) + ctx->c - 1]
                                      : nw;
              for (const auto& [b0, len, waves] : {std::tuple<int64_t, int64_t, int64_t>{out, cut + 8 * s.st_place_pad[sm], cut},
                                                   std::tuple<int64_t, int64_t, int64_t>{out + cut, nw - cut, nw - cut}}) {
                std::vector<uint8_t> seen(static_cast<size_t>(waves), 0);
                int64_t empty = 0;
                for (int64_t b = b0; b < b0 + len; ++b) {
                  const int32_t L = place[b];
                  if (L < 0) { ++empty; continue; }
                  MF_REQUIRE(L < waves && !seen[L], "systolic placement is not a permutation");
                  seen[L] = 1;
                }
                MF_REQUIRE(empty == len - waves, "systolic placement: empty blocks miscounted");
              }
            }
            s.st_place.alloc(place.size() * sizeof(int32_t));
            MF_HIP(hipMemcpy(s.st_place.get(), place.data(), place.size() * sizeof(int32_t), hipMemcpyHostToDevice));
          }
          s.sys_step = static_cast<uint32_t>(fp.G) + 1u;
          int64_t max_waves = 1;
          for (int32_t sm = 0; sm < ctx->nb; ++sm) max_waves = std::max(max_waves, pp.sys_off[sm + 1] - pp.sys_off[sm]);
          s.fast_prog.alloc(static_cast<size_t>(max_waves) * kProgStride * sizeof(int32_t));
          MF_HIP(hipMemsetAsync(s.fast_prog.get(), 0, s.fast_prog.bytes(), s.stream));
          s.fast_err.alloc(16);
          MF_HIP(hipMemsetAsync(s.fast_err.get(), 0, 16, s.stream));
        }
        clk.lap("pair plan + H2D");
        ctx->reaper.drop(pp.recs);
        if (exp_knob("MFHIP_WAVE_TRACE")) {
          const size_t n = ctx->fast_sys ? pp.sys.size() : pp.waves.size();
          const size_t per = ctx->fast_sys ? 32 : 16;  // systolic: realtime and shader-clock stamps
          s.st_trace.alloc(std::max<size_t>(n, 1) * per);
          MF_HIP(hipMemsetAsync(s.st_trace.get(), 0, std::max<size_t>(n, 1) * per, s.stream));
          if (ctx->fast_sys) {
            s.st_sys_host = pp.sys;
            s.st_sysw_host = pp.sys_waves;
          }
          else s.st_waves_host = pp.waves;
        }
        continue;
      }
      {  // requested bytes per superstep: 32-B record, user row in + out, item row per run in + out
        s.sm_bytes.assign(ctx->nb, 0.0);
        const double row_bytes = 4.0 * k;
        for (int32_t sm = 0; sm < ctx->nb; ++sm)
          for (int32_t j = 0; j < ctx->c; ++j) {
            const int32_t p = s.index * ctx->c + j;
            const int64_t b = static_cast<int64_t>(p) * ctx->nb + (p + sm) % ctx->nb;
            if (fp.cell_base[b] < 0) continue;
            const int32_t* o = fp.cell_off.data() + fp.cell_base[b];
            const int64_t GG = static_cast<int64_t>(fp.Gb[b]) * fp.Gb[b];
            const FastRec* f = fp.recs.data() + fp.rec_base[b];
            int64_t runs = 0;
            for (int64_t cc = 0; cc < GG; ++cc)
              for (int32_t x = o[cc]; x < o[cc + 1]; ++x)
                runs += x == o[cc] || ((f[x].i ^ f[x - 1].i) & ~kPadBit) != 0;
            s.sm_bytes[sm] += (32.0 + 2.0 * row_bytes) * o[GG] + 2.0 * row_bytes * static_cast<double>(runs);
          }
      }
      s.fast_recs.alloc(std::max<size_t>(fp.recs.size(), 1) * sizeof(FastRec));
      s.fast_cells.alloc(std::max<size_t>(fp.cell_off.size(), 1) * sizeof(int32_t));
      if (!fp.recs.empty())
        MF_HIP(hipMemcpy(s.fast_recs.get(), fp.recs.data(), fp.recs.size() * sizeof(FastRec), hipMemcpyHostToDevice));
      if (!fp.cell_off.empty())
        MF_HIP(hipMemcpy(s.fast_cells.get(), fp.cell_off.data(), fp.cell_off.size() * sizeof(int32_t),
                         hipMemcpyHostToDevice));
      std::vector<FastBlk> blks(static_cast<size_t>(ctx->nb) * ctx->c);
      for (int32_t sm = 0; sm < ctx->nb; ++sm)
        for (int32_t j = 0; j < ctx->c; ++j) {
          const int32_t p = s.index * ctx->c + j;
          const int32_t q = (p + sm) % ctx->nb;
          const int64_t b = static_cast<int64_t>(p) * ctx->nb + q;
          blks[static_cast<size_t>(sm) * ctx->c + j] = FastBlk{fp.rec_base[b], fp.cell_base[b] < 0 ? 0 : fp.cell_base[b]};
        }
      s.fast_prog.alloc(static_cast<size_t>(ctx->c) * ctx->G_fast * kProgStride * sizeof(int32_t));
      s.fast_err.alloc(16);
      MF_HIP(hipMemsetAsync(s.fast_err.get(), 0, 16, s.stream));
      s.fast_blks.alloc(blks.size() * sizeof(FastBlk));
      MF_HIP(hipMemcpy(s.fast_blks.get(), blks.data(), blks.size() * sizeof(FastBlk), hipMemcpyHostToDevice));
    }
    clk.lap("device tables");
    // the device holds the schedule; release the host copies in the background
    ctx->reaper.drop(fp.recs);
    ctx->reaper.drop(ctx->rb.urow);
    ctx->reaper.drop(ctx->rb.irow);
    ctx->reaper.drop(ctx->rb.r);
    ctx->rb = RatingBlocks();
    ctx->rb.n_blocks = ctx->nb;
    ctx->reaper.release();
  }
  clk.lap("release host blocks");
  // hipMemset on device memory returns before the fill is done and the legacy stream does not
  // order the non-blocking sweep streams (tools/micro/memset_order.hip: a 4-GiB memset returns
  // in 3 us and a kernel on another stream still reads the old bytes), so the zeroing above is
  // issued on the shard streams, and the device drains here: the first superstep's launches
  // (aux included, which waits on no event yet) see every table, zeroed row and progress word.
  // A run of 8 ranks sharing one GPU raced here (stale progress words let waves skip a hand-off).
  for (auto& s : ctx->shards) {
    DeviceGuard g(s.device);
    MF_HIP(hipDeviceSynchronize());
  }
  ctx->superstep_done = 0;
  reset_item_loc(ctx);
  ctx->prepared = true;
}

// Make every row current on shard `dst` (users from their owners, items from their holders).
void consolidate(mf_ctx* ctx, Shard& dst) {
  if (ctx->G <= 1 || ctx->rank_mode || !ctx->prepared) return;
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  sync_all(ctx);
  for (int32_t b = 0; b < ctx->nb; ++b) {
    for (int side = 0; side < 2; ++side) {
      const SideLayout& S = side_of(ctx, side);
      const int owner = side == kSideU ? shard_of_user_block(ctx, b) : ctx->item_loc[b];
      if (owner == dst.index) continue;
      Shard& src = *local_shard(ctx, owner);
      const int64_t r0 = S.block_start[b], cnt = S.block_start[b + 1] - r0;
      if (cnt == 0) continue;
      const size_t off = static_cast<size_t>(r0) * k * ctx->es, bytes = static_cast<size_t>(cnt) * k * ctx->es;
      DevBuf& sb = side == kSideU ? src.uf : src.itf;
      DevBuf& db = side == kSideU ? dst.uf : dst.itf;
      DeviceGuard g(dst.device);
      MF_HIP(hipMemcpyPeerAsync(db.as<char>() + off, dst.device, sb.as<char>() + off, src.device, bytes, dst.stream));
    }
  }
  DeviceGuard g(dst.device);
  MF_HIP(hipStreamSynchronize(dst.stream));
}

// Rank mode: broadcast each item block from its holder so every rank has all items.
void allgather_items(mf_ctx* ctx) {
  if (!ctx->rank_mode || ctx->G <= 1) return;
  // The last superstep may still be running: with the ring overlap its second launch is on
  // `aux` and the item block's send/recv on `comm`.  The broadcast below reads and writes item
  // rows on `stream`, and two RCCL operations of one communicator must not run on unordered
  // streams, so every stream of the rank drains first (and a sweep timeout surfaces here).
  sync_all(ctx);
  require_healthy(ctx);
  Shard& s = ctx->shards[0];
  DeviceGuard g(s.device);
  const size_t k = static_cast<size_t>(ctx->P.num_factors);
  MF_NCCL(ncclGroupStart());
  for (int32_t b = 0; b < ctx->nb; ++b) {
    const int64_t r0 = ctx->I.block_start[b], cnt = ctx->I.block_start[b + 1] - r0;
    if (cnt == 0) continue;
    char* p = s.itf.as<char>() + static_cast<size_t>(r0) * k * ctx->es;
    MF_NCCL(ncclBroadcast(p, p, cnt * k, ctx->f64 ? ncclFloat64 : ncclFloat32, ctx->item_loc[b], ctx->comm, s.stream));
  }
  MF_NCCL(ncclGroupEnd());
  MF_HIP(hipStreamSynchronize(s.stream));
  // item_loc keeps tracking the ring (all ranks simulate it identically); copies made here
  // are read-only snapshots for evaluation.
}

// Evaluation: resolve ids on the host, gather-dot on the device.
struct EvalOut {
  double sse = 0, cnt = 0, risk = 0;
};

EvalOut evaluate(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n,
                 const int32_t* mult, double lambda, double* pred_out, uint8_t* found_out) {
  MF_REQUIRE(ctx->have_model, "The MatrixFactorization model has not been fitted to data. "
                              "Prior to predicting values, it has to be trained on data.");
  MF_REQUIRE(n >= 0, "negative count");
  require_healthy(ctx);
  EvalOut res;
  if (n == 0) return res;
  Shard& s = ctx->shards[0];
  if (ctx->rank_mode) allgather_items(ctx);
  else consolidate(ctx, s);
  std::vector<uint32_t> ur, ir;
  lookup_rows(ctx->U, u, n, ur);
  lookup_rows(ctx->I, i, n, ir);
  std::vector<int32_t> urow(n), irow(n);
  const int me = s.index;
  for (int64_t j = 0; j < n; ++j) {
    int32_t a = static_cast<int32_t>(ur[j]), b = static_cast<int32_t>(ir[j]);
    if (ctx->rank_mode && a >= 0 && ctx->U.row_block[a] / ctx->c != me) a = -1;  // not my user
    urow[j] = a;
    irow[j] = b;
  }
  DeviceGuard g(s.device);
  MF_HIP(hipStreamSynchronize(s.stream));
  s.ev_u.alloc(n * 4);
  s.ev_i.alloc(n * 4);
  MF_HIP(hipMemcpy(s.ev_u.get(), urow.data(), n * 4, hipMemcpyHostToDevice));
  MF_HIP(hipMemcpy(s.ev_i.get(), irow.data(), n * 4, hipMemcpyHostToDevice));
  double* dout = nullptr;
  if (pred_out) { s.ev_out.alloc(n * 8); dout = s.ev_out.as<double>(); }
  const double* dr = nullptr;
  const int32_t* dm = nullptr;
  double* dpart = nullptr;
  const int grid = predict_grid(n);
  if (r) {
    s.ev_r.alloc(n * 8);
    MF_HIP(hipMemcpy(s.ev_r.get(), r, n * 8, hipMemcpyHostToDevice));
    dr = s.ev_r.as<double>();
    s.ev_part.alloc(static_cast<size_t>(grid) * 3 * 8);
    dpart = s.ev_part.as<double>();
    if (mult) {
      s.ev_mult.alloc(n * 4);
      MF_HIP(hipMemcpy(s.ev_mult.get(), mult, n * 4, hipMemcpyHostToDevice));
      dm = s.ev_mult.as<int32_t>();
    }
  }
  launch_predict(s.stream, s.ev_u.as<int32_t>(), s.ev_i.as<int32_t>(), n, s.uf.get(), s.itf.get(),
                 ctx->P.num_factors, ctx->f64, dout, dr, dm, lambda, dpart);
  MF_HIP(hipGetLastError());
  MF_HIP(hipStreamSynchronize(s.stream));
  if (pred_out) {
    MF_HIP(hipMemcpy(pred_out, dout, n * 8, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < n; ++j) found_out[j] = (urow[j] >= 0 && irow[j] >= 0) ? 1 : 0;
  }
  if (r) {
    std::vector<double> part(static_cast<size_t>(grid) * 3);
    MF_HIP(hipMemcpy(part.data(), dpart, part.size() * 8, hipMemcpyDeviceToHost));
    for (int w = 0; w < grid; ++w) {
      res.sse += part[3 * w];
      res.cnt += part[3 * w + 1];
      res.risk += part[3 * w + 2];
    }
  }
  if (ctx->rank_mode && ctx->G > 1) {
    // combine per-rank results: predictions (owner rank writes, others contribute 0), sums
    DevBuf red;
    const int64_t m = 3 + (pred_out ? 2 * n : 0);
    std::vector<double> h(m, 0.0);
    h[0] = res.sse; h[1] = res.cnt; h[2] = res.risk;
    if (pred_out)
      for (int64_t j = 0; j < n; ++j) { h[3 + j] = found_out[j] ? pred_out[j] : 0.0; h[3 + n + j] = found_out[j]; }
    red.alloc(m * 8);
    MF_HIP(hipMemcpy(red.get(), h.data(), m * 8, hipMemcpyHostToDevice));
    MF_NCCL(ncclAllReduce(red.get(), red.get(), m, ncclFloat64, ncclSum, ctx->comm, s.stream));
    MF_HIP(hipStreamSynchronize(s.stream));
    MF_HIP(hipMemcpy(h.data(), red.get(), m * 8, hipMemcpyDeviceToHost));
    res.sse = h[0]; res.cnt = h[1]; res.risk = h[2];
    if (pred_out)
      for (int64_t j = 0; j < n; ++j) { pred_out[j] = h[3 + j]; found_out[j] = h[3 + n + j] > 0.5 ? 1 : 0; }
  }
  return res;
}

// ---------------------------------------------------------------------------------------
// Online micro-batches (single shard).
int32_t online_row(mf_ctx* ctx, SideLayout& S, int32_t id, std::vector<int32_t>& fresh) {
  const int32_t row = S.index.find(id);
  if (row >= 0) return row;
  const int32_t nr = static_cast<int32_t>(S.rows());
  S.index.insert(id, nr);
  S.row_id.push_back(id);
  S.omega.push_back(0);
  S.row_block.push_back(-1);
  fresh.push_back(id);
  ctx->order_dirty = true;
  return nr;
}

// Brings the device mirror d up to the host table ix: the whole table after a rehash / clear / a
// table of its own (generation changed), else only the slots written since the last sync.
void sync_dev_index(Shard& s, const IdIndex& ix, DevIndex& d) {
  const uint64_t cap = ix.capacity();
  const auto& log = ix.log();
  if (cap == 0) {
    d.gen = ix.gen();
    d.cap = 0;
    d.applied = log.size();
    return;
  }
  if (d.gen != ix.gen() || d.cap != cap) {
    d.slots.alloc(cap * sizeof(IdIndex::Slot));
    MF_HIP(hipMemcpyAsync(d.slots.get(), ix.slots(), cap * sizeof(IdIndex::Slot), hipMemcpyHostToDevice, s.stream));
    MF_HIP(hipStreamSynchronize(s.stream));  // pageable source
    d.gen = ix.gen();
    d.cap = cap;
    d.applied = log.size();
    return;
  }
  const size_t m = log.size() - d.applied;
  if (m == 0) return;
  std::vector<uint32_t> pos(log.begin() + static_cast<std::ptrdiff_t>(d.applied), log.end());
  std::vector<IdIndex::Slot> val(m);
  for (size_t j = 0; j < m; ++j) val[j] = ix.slots()[pos[j]];
  d.upd_pos.alloc(m * 4);
  d.upd_val.alloc(m * sizeof(IdIndex::Slot));
  MF_HIP(hipMemcpyAsync(d.upd_pos.get(), pos.data(), m * 4, hipMemcpyHostToDevice, s.stream));
  MF_HIP(hipMemcpyAsync(d.upd_val.get(), val.data(), m * sizeof(IdIndex::Slot), hipMemcpyHostToDevice, s.stream));
  launch_id_scatter(s.stream, d.slots.get(), d.upd_pos.as<uint32_t>(), d.upd_val.get(), static_cast<int64_t>(m));
  MF_HIP(hipStreamSynchronize(s.stream));  // pos / val are released on return
  d.applied = log.size();
}

void online_update(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n, int flavour,
                   int num_partitions, int64_t* tu, int64_t* ti, double* uout = nullptr, double* iout = nullptr) {
  MF_REQUIRE(ctx->shards.size() == 1 && !ctx->rank_mode, "online updates run on a single-device context");
  MF_REQUIRE(flavour >= MF_ONLINE_NEXT_FACTORS && flavour <= MF_ONLINE_SPARK_SWEEP, "unknown online flavour");
  MF_REQUIRE(n >= 0 && (n == 0 || (u && i && r)), "bad rating arrays");
  MF_REQUIRE(!(uout || iout) || flavour != MF_ONLINE_SPARK_SWEEP,
             "MF_ONLINE_SPARK_SWEEP emits touched rows only (OfflineSpark.scala:33-67): no per-rating outputs");
  require_healthy(ctx);
  Shard& s = ctx->shards[0];
  if (!ctx->have_model) {
    ctx->U = SideLayout();
    ctx->I = SideLayout();
    ctx->have_model = true;
  }
  const int k = ctx->P.num_factors;
  PhaseClock clk;
  std::vector<int32_t> fu, fi;
  // one persistent launch (the default; MFHIP_TEST online_kernel=level forces the level-by-level
  // replay, which is also the path with per-rating outputs): NFLX 1M-rating batches 1.1e8 vs
  // 0.5e8 ratings/s end to end
  const bool outs = uout || iout;
  int cap = 0;
  // f64 at k = 64 / 128 / 256: the deterministic sweep's kernel with nextFactors' update (split
  // hot-item chains, kernels_detsweep.hip), while every row offset fits its 32-bit buffer offsets
  // (rows after this batch's new ids at most rows + n); MFHIP_TEST online_kernel=ticket keeps
  // k_online_sweep
  // f32 at k <= 256: k_online_f32, whose row offsets are 32-bit as well (u * k * 4 bytes); a slab
  // that would pass 4 GiB with this batch's new rows takes k_online_sweep (size_t addressing).
  // MFHIP_TEST offset_limit=<bytes> lowers the limit so the tests reach that fallback.
  bool det_online = false, f32_online = false;
  if (n > 0 && !outs && test_knob("online_kernel") != "level") {
    DeviceGuard g(s.device);
    double limit = 4294963200.0;  // raw_rsrc's clamp (pair_device.hpp)
    if (const std::string v = test_knob("offset_limit"); !v.empty()) limit = std::stod(v);
    const auto fits = [&](int64_t rows, int eb) { return static_cast<double>(rows + n) * k * eb <= limit; };
    det_online = ctx->f64 && test_knob("online_kernel") != "ticket" && online_det_capacity(k) > 0 &&
                 fits(ctx->U.rows(), 8) && fits(ctx->I.rows(), 8);
    f32_online = !ctx->f64 && online_f32_supports(k) && fits(ctx->U.rows(), 4) && fits(ctx->I.rows(), 4);
    // 0 (occupancy query failed): the level replay
    cap = det_online ? online_det_capacity(k)
          : f32_online ? online_f32_capacity(k) : online_sweep_capacity(k, ctx->f64);
    if (cap == 0) det_online = f32_online = false;
  }
  // the sweep in arrival order takes the rows straight into its pinned upload buffer (user rows,
  // item rows, ratings: 16 B per rating), with no staging pass; otherwise they go to on_ur / on_ir
  const bool direct = cap > 0 && flavour != MF_ONLINE_SPARK_SWEEP;
  // the f32 sweep's upload carries the ratings as floats (12 B per rating instead of 16): the
  // sweep rounds each rating to float first in any case (online_f32.hpp), so the bits are the same
  const bool rf32 = f32_online;
  const size_t in_bytes = static_cast<size_t>(n) * (rf32 ? 12 : 16);
  auto stage_r = [&](void* dst, int64_t lo2, int64_t hi2) {  // ratings [lo2, hi2) into the upload's rating array
    if (rf32) {
      float* f = static_cast<float*>(dst);
      for (int64_t x = lo2; x < hi2; ++x) f[x] = static_cast<float>(r[x]);
    } else {
      std::memcpy(static_cast<double*>(dst) + lo2, r + lo2, static_cast<size_t>(hi2 - lo2) * 8);
    }
  };
  uint32_t* ur = nullptr;
  uint32_t* ir = nullptr;
  if (direct) {
    DeviceGuard g(s.device);
    MF_HIP(hipStreamSynchronize(s.stream));  // det_pin may still feed an earlier copy
    s.det_pin.alloc(static_cast<size_t>(n) * 16);
    ur = s.det_pin.as<uint32_t>();
    ir = ur + n;
  } else {
    if (static_cast<int64_t>(ctx->on_ur.size()) < n) {
      ctx->on_ur.resize(n);
      ctx->on_ir.resize(n);
    }
    ur = ctx->on_ur.data();
    ir = ctx->on_ir.data();
  }
  const int64_t u0 = ctx->U.rows(), i0 = ctx->I.rows();
  std::vector<uint8_t> seen_u, seen_i;
  int64_t cu = 0, ci = 0;
  // rows of known ids in parallel (the index is only read; kMiss marks the others); then, in
  // rating order, the ids first seen in this batch get new rows in order of appearance, exactly
  // as one sequential scan would
  constexpr uint32_t kMiss = 0xFFFFFFFFu;
  std::atomic<int64_t> misses{0};
  // the direct path looks the ids up on the device (a mirror of each side's IdIndex, kept in step
  // by sync_dev_index): the host only copies the batch into the pinned upload, and resolves misses
  // (ids first seen in this batch) itself, in rating order, when there are any.  MFHIP_TEST
  // online_lookup=host keeps the host lookup (the tests compare the two bit for bit).
  const bool dev_lookup = direct && test_knob("online_lookup") != "host";
  bool uploaded = false;
  // the sweep's device plan (online_sweep_plan) of the batch in sc.in.  On the device-lookup path it
  // is queued right behind the lookup, before the host waits for the miss count, so the host's ~100
  // plan launches overlap the upload's DMA; misses (new ids) void it and it runs again after the
  // host has given them rows.
  int64_t W = 1;
  if (cap > 0) {
    int64_t wmax = 4096;
    if (const char* v = exp_knob("MFHIP_ONLINE_WAVES")) wmax = std::max(1, std::atoi(v));
    W = std::max<int64_t>(1, std::min<int64_t>({static_cast<int64_t>(cap / 2), wmax, n}));
  }
  const size_t ebytes = static_cast<size_t>(n) * sizeof(DetEntry), qbytes = static_cast<size_t>(n) * 4;
  bool planned = false;
  uint32_t nsingle = 0;
  auto plan_batch = [&]() {
    OnlineSweepScratch& sc = s.online_sc;
    s.det_dev.alloc(ebytes + qbytes);
    sc.wbeg.alloc(static_cast<size_t>(W + 1) * 8);
    sc.touched.alloc(8);
    const uint32_t* du = sc.in.as<uint32_t>();
    // waves [0, nsingle) hold one item each: k_online_f32's lean single-item path
    nsingle = online_sweep_plan(
        s.stream, sc, du, du + n, reinterpret_cast<const double*>(du + 2 * n), n, static_cast<uint32_t>(W),
        static_cast<uint32_t>(ctx->U.rows()), static_cast<uint32_t>(ctx->I.rows()), s.det_dev.as<DetEntry>(),
        reinterpret_cast<uint32_t*>(s.det_dev.as<char>() + ebytes), sc.wbeg.as<int64_t>(), sc.touched.as<int32_t>(),
        rf32 ? reinterpret_cast<const float*>(du + 2 * n) : nullptr);
    planned = true;
  };
  // the f32 sweep of the planned batch, queued with its error word and touched counts read back into
  // pinned memory (pin4[1..3]); skip: the lookup's miss count (the launch does nothing when non-zero)
  s.small_pin.alloc(16);
  int32_t* pin4 = s.small_pin.as<int32_t>();
  auto queue_f32_sweep = [&](const int32_t* skip) {
    OnlineSweepScratch& sc = s.online_sc;
    const size_t ub = static_cast<size_t>(std::max<int64_t>(ctx->U.rows(), 1)) * 4;
    sc.uticket.alloc(ub);
    MF_HIP(hipMemsetAsync(sc.uticket.get(), 0, ub, s.stream));
    sc.err.alloc(4);
    MF_HIP(hipMemsetAsync(sc.err.get(), 0, 4, s.stream));
    sc.dummy.alloc(static_cast<size_t>(W) * 64);
    {
      LaunchTimer t(s, ctx->profiling, true);
      launch_online_f32(s.stream, static_cast<int>(W), sc.wbeg.as<int64_t>(), s.det_dev.as<DetEntry>(),
                        reinterpret_cast<const uint32_t*>(s.det_dev.as<char>() + ebytes), s.uf.as<float>(),
                        s.itf.as<float>(), s.uf.bytes(), s.itf.bytes(), k, ctx->P.online_learning_rate,
                        sc.uticket.as<int32_t>(), sc.dummy.as<int32_t>(), sc.err.as<int32_t>(),
                        test_knob("online_single") == "0" ? 0 : static_cast<int>(nsingle), skip, t.start(), t.stop());
    }
    MF_HIP(hipGetLastError());
    MF_HIP(hipMemcpyAsync(pin4 + 1, sc.err.get(), 4, hipMemcpyDeviceToHost, s.stream));
    MF_HIP(hipMemcpyAsync(pin4 + 2, sc.touched.get(), 8, hipMemcpyDeviceToHost, s.stream));
  };
  // the f64 sweep's entry arrays and wave table from the plan; the table comes back to the host
  // (pinned) for det_slot_table, read after the next stream sync
  uint32_t *det_eu = nullptr, *det_ei = nullptr, *det_eq = nullptr;
  double* det_er = nullptr;
  bool det_entries = false;
  auto queue_det_entries = [&]() {
    OnlineSweepScratch& sc = s.online_sc;
    sc.waves.alloc(static_cast<size_t>(det_slot_room(W)) * sizeof(DetWave));
    online_det_entries(s.stream, sc, s.det_dev.as<DetEntry>(),
                       reinterpret_cast<const uint32_t*>(s.det_dev.as<char>() + ebytes), sc.wbeg.as<int64_t>(), n,
                       static_cast<uint32_t>(W), det_eu, det_ei, det_eq, det_er, sc.waves.as<DetWave>());
    s.slots_pin.alloc(static_cast<size_t>(det_slot_room(W)) * sizeof(DetWave));
    MF_HIP(hipMemcpyAsync(s.slots_pin.as<DetWave>(), sc.waves.get(), static_cast<size_t>(W) * sizeof(DetWave),
                          hipMemcpyDeviceToHost, s.stream));
    det_entries = true;
  };
  if (dev_lookup) {
    DeviceGuard g(s.device);
    OnlineSweepScratch& sc = s.online_sc;
    sync_dev_index(s, ctx->U.index, s.didx[0]);
    sync_dev_index(s, ctx->I.index, s.didx[1]);
    sc.in.alloc(in_bytes);
    // (staging in pieces with each piece's upload queued behind it was slower: 2-3 ms against ~1 ms
    // per NFLX batch, gpurun_out/r6d)
    parallel_for(n, [&](int64_t lo2, int64_t hi2, int) {
      const size_t c = static_cast<size_t>(hi2 - lo2);
      std::memcpy(ur + lo2, u + lo2, c * 4);
      std::memcpy(ir + lo2, i + lo2, c * 4);
      stage_r(ir + n, lo2, hi2);
    });
    MF_HIP(hipMemcpyAsync(sc.in.get(), ur, in_bytes, hipMemcpyHostToDevice, s.stream));
    clk.lap("online: staging + upload");
    sc.miss.alloc(4);
    MF_HIP(hipMemsetAsync(sc.miss.get(), 0, 4, s.stream));
    const DevIndex &du = s.didx[0], &di = s.didx[1];
    launch_id_lookup(s.stream, sc.in.as<uint32_t>(), n, du.cap ? du.slots.get() : nullptr, du.cap - 1,
                     di.cap ? di.slots.get() : nullptr, di.cap - 1, sc.miss.as<int32_t>());
    MF_HIP(hipMemcpyAsync(pin4, sc.miss.get(), 4, hipMemcpyDeviceToHost, s.stream));
    plan_batch();  // (the plan's kernels skip rows past the tables: the misses)
    // f32: the sweep goes right behind the plan, so the batch runs through without the host in the
    // loop; a batch with misses skips it on the device and takes the path below
    const bool queued = f32_online;
    if (queued) {
      ensure_rows(ctx, s, kSideU, std::max<int64_t>(ctx->U.rows(), 1));
      ensure_rows(ctx, s, MF_SIDE_ITEM, std::max<int64_t>(ctx->I.rows(), 1));
      queue_f32_sweep(sc.miss.as<int32_t>());
    } else if (det_online) {
      queue_det_entries();  // (void with the plan when there are misses)
    }
    clk.lap("online: lookup + plan queued");
    MF_HIP(hipStreamSynchronize(s.stream));
    const int32_t m = pin4[0];
    misses = m;
    if (queued && m == 0) {
      clk.lap("online: sweep (device)");
      if (pin4[1]) {
        ctx->failed = "online sweep: a wave waited > 1 s for a user ticket (waves not co-resident?); "
                      "set MFHIP_TEST=online_kernel=level (INTEGRATION.md section 5)";
        fail(MF_ERR_TIMEOUT, ctx->failed);
      }
      if (tu) *tu = pin4[2];
      if (ti) *ti = pin4[3];
      ctx->stats.kernel_launches += 1;
      ctx->stats.updates += n;
      return;
    }
    if (m > 0) {  // the rows as found (kMiss where absent) back into the pinned buffer
      planned = det_entries = false;
      MF_HIP(hipMemcpyAsync(ur, sc.in.get(), static_cast<size_t>(n) * 8, hipMemcpyDeviceToHost, s.stream));
      MF_HIP(hipStreamSynchronize(s.stream));
    }
    uploaded = m == 0;
  } else {
    parallel_for(n, [&](int64_t lo2, int64_t hi2, int) {
      ctx->U.index.find_many(u + lo2, hi2 - lo2, ur + lo2);
      ctx->I.index.find_many(i + lo2, hi2 - lo2, ir + lo2);
      if (direct) stage_r(ir + n, lo2, hi2);
      int64_t m = 0;
      for (int64_t j = lo2; j < hi2; ++j) m += (ur[j] == kMiss) + (ir[j] == kMiss);
      misses += m;
    });
  }
  if (misses > 0)
    for (int64_t j = 0; j < n; ++j) {
      if (ur[j] == kMiss) ur[j] = static_cast<uint32_t>(online_row(ctx, ctx->U, u[j], fu));
      if (ir[j] == kMiss) ir[j] = static_cast<uint32_t>(online_row(ctx, ctx->I, i[j], fi));
    }
  clk.lap("online: id lookup");
  // touched-row counts (UpdateSeparatedHashMap.updates, OfflineSpark.scala:33-67): counted on the
  // device by the sweep's plan, else here
  if (cap == 0) {
  seen_u.assign(ctx->U.rows(), 0);
  seen_i.assign(ctx->I.rows(), 0);
  // flags set with plain relaxed stores, and only when still clear (a locked exchange per rating
  // kept the flag lines bouncing between cores: 8 ms per 1M ratings), then counted
  parallel_for(n, [&](int64_t lo2, int64_t hi2, int) {
    for (int64_t j = lo2; j < hi2; ++j) {
      if (!__atomic_load_n(&seen_u[ur[j]], __ATOMIC_RELAXED)) __atomic_store_n(&seen_u[ur[j]], 1, __ATOMIC_RELAXED);
      if (!__atomic_load_n(&seen_i[ir[j]], __ATOMIC_RELAXED)) __atomic_store_n(&seen_i[ir[j]], 1, __ATOMIC_RELAXED);
    }
  });
  std::atomic<int64_t> acu{0}, aci{0};
  parallel_for(static_cast<int64_t>(std::max(seen_u.size(), seen_i.size())), [&](int64_t lo2, int64_t hi2, int) {
    int64_t lu = 0, li = 0;
    for (int64_t x = lo2; x < hi2; ++x) {
      if (x < static_cast<int64_t>(seen_u.size())) lu += seen_u[x];
      if (x < static_cast<int64_t>(seen_i.size())) li += seen_i[x];
    }
    acu += lu;
    aci += li;
  });
  cu = acu;
  ci = aci;
  if (tu) *tu = cu;
  if (ti) *ti = ci;
  clk.lap("online: touched rows");
  }
  // new rows take the slab rows the fast DSGD schedule keeps zeroed (padding / idle prefetch
  // rows past the real ones): that schedule is void now, a further fit must prepare again
  if (ctx->prepared && !ctx->f64 && (!fu.empty() || !fi.empty())) ctx->prepared = false;
  // first-touch initialisation of unseen ids
  const bool xor_seed = ctx->P.online_init == MF_INIT_SEEDED;
  for (int side = 0; side < 2; ++side) {
    const std::vector<int32_t>& fresh = side == kSideU ? fu : fi;
    const int64_t row0 = side == kSideU ? u0 : i0;
    const SideLayout& S = side_of(ctx, side);
    ensure_rows(ctx, s, side, std::max<int64_t>(S.rows(), 1));
    if (fresh.empty()) continue;
    std::vector<double> vec;
    init_vectors(fresh.data(), static_cast<int64_t>(fresh.size()), k, xor_seed, ctx->P.seed, vec);
    upload_rows(ctx, s, side, row0, vec.data(), static_cast<int64_t>(fresh.size()));
  }
  if (n == 0) return;
  // sequential order of the flavour
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  if (flavour == MF_ONLINE_SPARK_SWEEP) {
    // OfflineSpark.scala:135-147,163-203: user partition id % P, item rating block abs(i) % P;
    // sub-epoch s (1-based) pairs partition p with item block (p - (s-1)) mod P; each cell in
    // insertion order.  One iteration per micro-batch (OnlineSpark.scala:191-194).
    MF_REQUIRE(num_partitions >= 1, "num_partitions must be >= 1 for MF_ONLINE_SPARK_SWEEP");
    const int P = num_partitions;
    std::vector<std::vector<int32_t>> cells(static_cast<size_t>(P) * P);
    for (int64_t j = 0; j < n; ++j) {
      MF_REQUIRE(u[j] >= 0 && i[j] != INT32_MIN, "Spark sweep needs non-negative user ids");
      const int up = u[j] % P, ib = std::abs(i[j]) % P;
      cells[static_cast<size_t>(up) * P + ib].push_back(static_cast<int32_t>(j));
    }
    order.clear();
    for (int sub = 1; sub <= P; ++sub)
      for (int p = 0; p < P; ++p) {
        const int q = ((p - (sub - 1)) % P + P) % P;
        const auto& c = cells[static_cast<size_t>(p) * P + q];
        order.insert(order.end(), c.begin(), c.end());
      }
  }
  if (cap > 0) {
    // one persistent launch (k_online_sweep): items spread over the waves, each wave's updates in
    // sequence order, and per update the number of earlier updates of its user (its ticket value)
    DeviceGuard g(s.device);
    // the batch in sequence order goes up as is (16 bytes an update); the per-wave lists and the
    // tickets are built on the device (online_sweep_plan, kernels_online.hip)
    OnlineSweepScratch& sc = s.online_sc;
    if (!direct) {  // the Spark-sweep order: staged here
      MF_HIP(hipStreamSynchronize(s.stream));  // det_pin may still feed an earlier copy
      s.det_pin.alloc(in_bytes);
      uint32_t* pu = s.det_pin.as<uint32_t>();
      uint32_t* pi = pu + n;
      double* pr = reinterpret_cast<double*>(pi + n);
      float* prf = reinterpret_cast<float*>(pi + n);
      parallel_for(n, [&](int64_t lo2, int64_t hi2, int) {
        for (int64_t x = lo2; x < hi2; ++x) {
          const int32_t j = order[x];
          pu[x] = ur[j];
          pi[x] = ir[j];
          if (rf32) prf[x] = static_cast<float>(r[j]);
          else pr[x] = r[j];
        }
      });
      clk.lap("online: sweep staging");
    }
    uint32_t* pu = s.det_pin.as<uint32_t>();
    if (!uploaded) {  // (the device lookup left the batch's rows in sc.in already)
      sc.in.alloc(in_bytes);
      MF_HIP(hipMemcpyAsync(sc.in.get(), pu, in_bytes, hipMemcpyHostToDevice, s.stream));
    }
    if (!planned) plan_batch();
    if (f32_online) {
      queue_f32_sweep(nullptr);
    } else if (det_online) {
      const size_t ub = static_cast<size_t>(std::max<int64_t>(ctx->U.rows(), 1)) * 4;
      sc.uticket.alloc(ub);
      MF_HIP(hipMemsetAsync(sc.uticket.get(), 0, ub, s.stream));
      sc.err.alloc(4);
      MF_HIP(hipMemsetAsync(sc.err.get(), 0, 4, s.stream));
      // the wave table goes through the host once (W descriptors): det_slot_table pairs each
      // single-item wave with its helper and gives the longest chains a CU each (queued behind the
      // device lookup on that path, so that one sync brings back the miss count and the table)
      if (!det_entries) {
        queue_det_entries();
        MF_HIP(hipStreamSynchronize(s.stream));
      }
      DetWave* slots = s.slots_pin.as<DetWave>();
      const int64_t nslots =
          det_slot_table(slots, W, cap / 2, test_knob("det_alone") != "0", device_cu_count(s.device));
      MF_HIP(hipMemcpyAsync(sc.waves.get(), slots, static_cast<size_t>(nslots) * sizeof(DetWave),
                            hipMemcpyHostToDevice, s.stream));
      LaunchTimer t(s, ctx->profiling, true);
      launch_online_det(s.stream, sc.waves.as<DetWave>(), static_cast<int>(nslots), det_eu, det_ei, det_eq, det_er,
                        s.uf.as<double>(), s.itf.as<double>(), s.uf.bytes(), s.itf.bytes(), k,
                        ctx->P.online_learning_rate, sc.uticket.as<int32_t>(), sc.err.as<int32_t>(), t.start(),
                        t.stop());
    } else {
      const size_t ub = static_cast<size_t>(std::max<int64_t>(ctx->U.rows(), 1)) * 4;
      sc.uticket.alloc(ub);
      MF_HIP(hipMemsetAsync(sc.uticket.get(), 0, ub, s.stream));
      sc.err.alloc(4);
      MF_HIP(hipMemsetAsync(sc.err.get(), 0, 4, s.stream));
      LaunchTimer t(s, ctx->profiling);
      launch_online_sweep(s.stream, static_cast<int>(W), sc.wbeg.as<int64_t>(), s.det_dev.as<DetEntry>(),
                          reinterpret_cast<const uint32_t*>(s.det_dev.as<char>() + ebytes), s.uf.get(), s.itf.get(), k,
                          ctx->P.online_learning_rate, ctx->f64, sc.uticket.as<int32_t>(), sc.err.as<int32_t>());
    }
    MF_HIP(hipGetLastError());
    if (!f32_online) {
      MF_HIP(hipMemcpyAsync(pin4 + 1, sc.err.get(), 4, hipMemcpyDeviceToHost, s.stream));
      MF_HIP(hipMemcpyAsync(pin4 + 2, sc.touched.get(), 8, hipMemcpyDeviceToHost, s.stream));
    }
    MF_HIP(hipStreamSynchronize(s.stream));
    clk.lap("online: sweep (device)");
    const int32_t err = pin4[1], touched[2] = {pin4[2], pin4[3]};
    if (err) {
      // waves that gave up skipped the rest of their updates and the batch's new ids are already
      // in the index: the model is partly updated, so the context refuses further work (as the
      // DSGD sweeps do, sync_all) until a fit is prepared again
      ctx->failed = "online sweep: a wave waited > 1 s for a user ticket (waves not co-resident?); "
                    "set MFHIP_TEST=online_kernel=level (INTEGRATION.md section 5)";
      fail(MF_ERR_TIMEOUT, ctx->failed);
    }
    if (tu) *tu = touched[0];
    if (ti) *ti = touched[1];
    ctx->stats.kernel_launches += 1;
    ctx->stats.updates += n;
    return;
  }
  std::vector<double> rr(r, r + n);
  OrderedSeq sq;
  sq.u = ur;
  sq.i = ir;
  sq.r = rr.data();
  sq.order = order.data();
  sq.len = n;
  sq.u_lo = 0;
  sq.u_hi = static_cast<uint32_t>(ctx->U.rows());
  sq.i_lo = 0;
  sq.i_hi = static_cast<uint32_t>(ctx->I.rows());
  LevelPlan lp;
  std::vector<int32_t> src;
  clk.lap("online: new rows + order");
  build_level_plan({sq}, lp, outs ? &src : nullptr);
  clk.lap("online: level plan");
  DeviceGuard g(s.device);
  const size_t bytes = lp.entries.size() * sizeof(DetEntry);
  MF_HIP(hipStreamSynchronize(s.stream));
  s.det_pin.alloc(bytes);
  s.det_dev.alloc(bytes);
  std::memcpy(s.det_pin.as<void>(), lp.entries.data(), bytes);
  MF_HIP(hipMemcpyAsync(s.det_dev.get(), s.det_pin.as<void>(), bytes, hipMemcpyHostToDevice, s.stream));
  DevBuf dsrc, duo, dio;
  const size_t obytes = static_cast<size_t>(n) * k * sizeof(double);
  if (outs) {
    dsrc.alloc(src.size() * sizeof(int32_t));
    MF_HIP(hipMemcpyAsync(dsrc.get(), src.data(), src.size() * sizeof(int32_t), hipMemcpyHostToDevice, s.stream));
    if (uout) duo.alloc(obytes);
    if (iout) dio.alloc(obytes);
  }
  const OnlineOut om = flavour == MF_ONLINE_DELTA ? OnlineOut::kOutDelta : OnlineOut::kOutNext;
  for (int64_t l = 0; l < lp.levels(); ++l) {
    const int64_t b0 = lp.level_start[l], cnt = lp.level_start[l + 1] - b0;
    LaunchTimer t(s, ctx->profiling);
    if (outs)
      launch_level_out(s.stream, s.det_dev.as<DetEntry>() + b0, cnt, s.uf.get(), s.itf.get(), k,
                       ctx->P.online_learning_rate, ctx->f64, om, dsrc.as<int32_t>() + b0,
                       uout ? duo.as<double>() : nullptr, iout ? dio.as<double>() : nullptr);
    else
      launch_level(s.stream, s.det_dev.as<DetEntry>() + b0, cnt, s.uf.get(), s.itf.get(), s.regu.get(),
                   s.regi.get(), k, ctx->P.online_learning_rate, Arith::kSgdNext, ctx->f64);
  }
  MF_HIP(hipGetLastError());
  clk.lap("online: H2D + level launches queued");
  MF_HIP(hipStreamSynchronize(s.stream));
  clk.lap("online: kernels done");
  if (uout) MF_HIP(hipMemcpy(uout, duo.get(), obytes, hipMemcpyDeviceToHost));
  if (iout) MF_HIP(hipMemcpy(iout, dio.get(), obytes, hipMemcpyDeviceToHost));
  ctx->stats.levels += lp.levels();
  ctx->stats.kernel_launches += lp.levels();
  ctx->stats.updates += n;
}

mf_ctx* new_ctx(const mf_params* p) {
  validate_params(p);
  auto* ctx = new mf_ctx();
  ctx->P = *p;
  ctx->f64 = p->mode == MF_MODE_DETERMINISTIC_F64;
  ctx->es = ctx->f64 ? 8 : 4;
  ctx->fast_persistent = choose_fast_kernel(p->num_factors) == FastKernel::kPersistent;
  return ctx;
}

}  // namespace
}  // namespace mfhip

using namespace mfhip;

extern "C" {

void mf_params_init(mf_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->num_factors = 10;        // MatrixFactorization.scala:201-203
  p->iterations = 10;         // :209-211
  p->lambda = 1.0;            // :205-207
  p->learning_rate = 0.001;   // DSGDforMF.scala:163-165
  p->lr_method = MF_LR_DEFAULT;  // :167-169
  p->lr_arg = 0.0;
  p->num_blocks = 1;          // Blocks None -> getOrElse(1) (:270)
  p->seed = 0;                // Seed Some(0L) (:217-219)
  p->has_seed = 1;
  p->mode = MF_MODE_DETERMINISTIC_F64;
  p->online_learning_rate = 0.01;  // SparkExample.scala:33 SGDUpdater(0.01)
  p->online_init = MF_INIT_PSEUDO_RANDOM;
  p->fast_waves = 0;
}

const char* mf_last_error(void) { return g_last_error.c_str(); }
const char* mf_version(void) { return "mfhip 0.1.0 (gfx950)"; }

int mf_device_count(int* n) {
  return guarded([&] {
    MF_REQUIRE(n, "null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
  });
}

int mf_create(const mf_params* p, const int* device_ids, int n_devices, mf_ctx** out) {
  return guarded([&] {
    MF_REQUIRE(out, "out is null");
    *out = nullptr;
    MF_REQUIRE(n_devices >= 1, "n_devices must be >= 1");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1)
      fail(MF_ERR_NO_DEVICE, "no HIP device available (libmfhip has no CPU fallback)");
    std::unique_ptr<mf_ctx> ctx(new_ctx(p));
    ctx->G = n_devices;
    { std::vector<Shard> tmp(n_devices); ctx->shards.swap(tmp); }
    for (int d = 0; d < n_devices; ++d) {
      const int dev = device_ids ? device_ids[d] : d % count;  // shards may share a device
      MF_REQUIRE(dev >= 0 && dev < count, "device id out of range");
      init_shard(ctx->shards[d], dev, d);
    }
    // enable peer access between distinct devices (ignore "already enabled")
    for (auto& a : ctx->shards)
      for (auto& b : ctx->shards)
        if (a.device != b.device) {
          int ok = 0;
          (void)hipDeviceCanAccessPeer(&ok, a.device, b.device);
          if (ok) {
            DeviceGuard g(a.device);
            (void)hipDeviceEnablePeerAccess(b.device, 0);
            (void)hipGetLastError();
          }
        }
    *out = ctx.release();
  });
}

int mf_comm_unique_id(uint8_t uid_out[MF_UID_BYTES]) {
  return guarded([&] {
    MF_REQUIRE(uid_out, "null");
    static_assert(sizeof(ncclUniqueId) <= MF_UID_BYTES, "uid size");
    ncclUniqueId id;
    MF_NCCL(ncclGetUniqueId(&id));
    std::memset(uid_out, 0, MF_UID_BYTES);
    std::memcpy(uid_out, &id, sizeof(id));
  });
}

int mf_create_rank(const mf_params* p, int device_id, int nranks, int rank, const uint8_t uid[MF_UID_BYTES],
                   mf_ctx** out) {
  return guarded([&] {
    MF_REQUIRE(out && uid, "null argument");
    *out = nullptr;
    MF_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1)
      fail(MF_ERR_NO_DEVICE, "no HIP device available (libmfhip has no CPU fallback)");
    MF_REQUIRE(device_id >= 0 && device_id < count, "device id out of range");
    std::unique_ptr<mf_ctx> ctx(new_ctx(p));
    ctx->G = nranks;
    ctx->rank_mode = true;
    { std::vector<Shard> tmp(1); ctx->shards.swap(tmp); }
    init_shard(ctx->shards[0], device_id, rank);
    if (nranks > 1) {
      DeviceGuard g(device_id);
      ncclUniqueId id;
      std::memcpy(&id, uid, sizeof(id));
      MF_NCCL(ncclCommInitRank(&ctx->comm, nranks, id, rank));
    }
    *out = ctx.release();
  });
}

int mf_destroy(mf_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    try {
      det_spec_wait(ctx, true);
    } catch (...) {  // a failed speculative build only matters to a run that would have used it
    }
    for (auto& s : ctx->shards) {
      DeviceGuard g(s.device);
      (void)hipStreamSynchronize(s.stream);
    }
    dump_wave_trace(ctx);
    for (auto& s : ctx->shards) destroy_shard(s);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    delete ctx;
  });
}

int mf_dsgd_prepare(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    prepare(ctx, u, i, r, n);
  });
}

int mf_dsgd_run(mf_ctx* ctx, int64_t supersteps) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    MF_REQUIRE(supersteps >= 0, "negative superstep count");
    run_supersteps(ctx, supersteps);
  });
}

int mf_dsgd_superstep(mf_ctx* ctx, int64_t* done) {
  return guarded([&] {
    MF_REQUIRE(ctx && done, "null argument");
    *done = ctx->superstep_done;
  });
}

int mf_dsgd_set_superstep(mf_ctx* ctx, int64_t done) {
  return guarded([&] {
    MF_REQUIRE(ctx && done >= 0, "bad argument");
    MF_REQUIRE(ctx->prepared, "mf_dsgd_set_superstep before mf_dsgd_prepare");
    det_spec_wait(ctx, true);
    sync_all(ctx);
    ctx->superstep_done = done;
    reset_item_loc(ctx);
  });
}

int mf_dsgd_restart(mf_ctx* ctx) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    MF_REQUIRE(ctx->prepared, "mf_dsgd_restart before mf_dsgd_prepare");
    det_spec_wait(ctx, true);
    ctx->failed.clear();
    sync_all(ctx);
    init_factors(ctx);
    ctx->superstep_done = 0;
    reset_item_loc(ctx);
  });
}

int mf_sync(mf_ctx* ctx) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    sync_all(ctx);
  });
}

int mf_dsgd_fit(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    prepare(ctx, u, i, r, n);
    run_supersteps(ctx, static_cast<int64_t>(ctx->P.iterations) * ctx->nb);
    sync_all(ctx);
  });
}

int mf_num_factors(mf_ctx* ctx, int side, int64_t* count) {
  return guarded([&] {
    MF_REQUIRE(ctx && count, "null argument");
    MF_REQUIRE(side == MF_SIDE_USER || side == MF_SIDE_ITEM, "bad side");
    const SideLayout& S = side_of(ctx, side);
    if (!ctx->rank_mode || side == MF_SIDE_ITEM || !ctx->prepared) { *count = S.rows(); return; }
    const int me = ctx->shards[0].index;
    *count = S.block_start[(me + 1) * ctx->c] - S.block_start[me * ctx->c];
  });
}

int mf_get_factors(mf_ctx* ctx, int side, int32_t* ids, double* vecs, int64_t cap, int64_t* written) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    MF_REQUIRE(side == MF_SIDE_USER || side == MF_SIDE_ITEM, "bad side");
    MF_REQUIRE(ctx->have_model, "The MatrixFactorization model has not been fitted to data.");
    require_healthy(ctx);
    Shard& s = ctx->shards[0];
    if (ctx->rank_mode) { if (side == MF_SIDE_ITEM) allgather_items(ctx); }
    else consolidate(ctx, s);
    sync_all(ctx);
    ensure_order(ctx);
    const SideLayout& S = side_of(ctx, side);
    const int k = ctx->P.num_factors;
    std::vector<double> all(static_cast<size_t>(std::max<int64_t>(S.rows(), 1)) * k);
    download_rows(ctx, s, side, 0, S.rows(), all.data());
    const auto& ord = side == kSideU ? ctx->rows_by_id_u : ctx->rows_by_id_i;
    int64_t w = 0;
    const int me = s.index;
    for (int64_t x = 0; x < S.rows(); ++x) {
      const int32_t row = ord[x];
      if (ctx->rank_mode && side == kSideU && S.row_block[row] / ctx->c != me) continue;
      if (w >= cap) fail(MF_ERR_CAPACITY, "output capacity too small");
      if (ids) ids[w] = S.row_id[row];
      if (vecs) std::memcpy(vecs + static_cast<size_t>(w) * k, all.data() + static_cast<size_t>(row) * k, sizeof(double) * k);
      ++w;
    }
    if (written) *written = w;
  });
}

int mf_set_factors(mf_ctx* ctx, int side, const int32_t* ids, const double* vecs, int64_t n) {
  return guarded([&] {
    MF_REQUIRE(ctx && (n == 0 || (ids && vecs)), "null argument");
    MF_REQUIRE(side == MF_SIDE_USER || side == MF_SIDE_ITEM, "bad side");
    det_spec_wait(ctx, true);  // rows may be added: the layouts change
    if (!ctx->have_model) { ctx->U = SideLayout(); ctx->I = SideLayout(); ctx->have_model = true; }
    SideLayout& S = side_of(ctx, side);
    std::vector<int32_t> fresh;
    std::vector<int32_t> rows(n);
    for (int64_t j = 0; j < n; ++j) rows[j] = online_row(ctx, S, ids[j], fresh);
    const int k = ctx->P.num_factors;
    sync_all(ctx);
    for (auto& s : ctx->shards) {
      ensure_rows(ctx, s, side, std::max<int64_t>(S.rows(), 1));
      if (n < 64) {
        for (int64_t j = 0; j < n; ++j) upload_rows(ctx, s, side, rows[j], vecs + static_cast<size_t>(j) * k, 1);
        continue;
      }
      // many rows: patch a host copy of the slab and upload it once
      std::vector<double> all(static_cast<size_t>(S.rows()) * k);
      download_rows(ctx, s, side, 0, S.rows(), all.data());
      for (int64_t j = 0; j < n; ++j)
        std::memcpy(all.data() + static_cast<size_t>(rows[j]) * k, vecs + static_cast<size_t>(j) * k, k * sizeof(double));
      upload_rows(ctx, s, side, 0, all.data(), S.rows());
    }
  });
}

int mf_get_params(mf_ctx* ctx, mf_params* out) {
  return guarded([&] {
    MF_REQUIRE(ctx && out, "null argument");
    *out = ctx->P;
  });
}

int mf_predict(mf_ctx* ctx, const int32_t* u, const int32_t* i, int64_t n, double* out, uint8_t* found) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    MF_REQUIRE(n == 0 || (u && i && out && found), "null argument");
    evaluate(ctx, u, i, nullptr, n, nullptr, 0.0, out, found);
  });
}

int mf_rmse(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n, double* rmse,
            int64_t* matched) {
  return guarded([&] {
    MF_REQUIRE(ctx && rmse, "null argument");
    MF_REQUIRE(n == 0 || (u && i && r), "null argument");
    EvalOut e = evaluate(ctx, u, i, r, n, nullptr, 0.0, nullptr, nullptr);
    *rmse = e.cnt > 0 ? std::sqrt(e.sse / e.cnt) : std::nan("");
    if (matched) *matched = static_cast<int64_t>(e.cnt);
  });
}

int mf_empirical_risk(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n,
                      double lambda, double* risk) {
  return guarded([&] {
    MF_REQUIRE(ctx && risk, "null argument");
    MF_REQUIRE(n == 0 || (u && i && r), "null argument");
    // the (user, item)-keyed join multiplies duplicate pairs (MatrixFactorization.scala:175)
    std::vector<uint64_t> key(n);
    for (int64_t j = 0; j < n; ++j)
      key[j] = (static_cast<uint64_t>(static_cast<uint32_t>(u[j])) << 32) | static_cast<uint32_t>(i[j]);
    std::vector<uint64_t> sorted = key;
    std::sort(sorted.begin(), sorted.end());
    std::vector<int32_t> mult(n);
    for (int64_t j = 0; j < n; ++j) {
      auto rg = std::equal_range(sorted.begin(), sorted.end(), key[j]);
      mult[j] = static_cast<int32_t>(rg.second - rg.first);
    }
    EvalOut e = evaluate(ctx, u, i, r, n, mult.data(), lambda, nullptr, nullptr);
    *risk = e.risk;
  });
}

// mf_block_update: one rating block's updateLocalFactors (DSGDforMF.scala:378-418) on caller
// buffers, as a Flink-resident task would call it.  The block's shuffle (new Random(iteration ^
// ratingBlockId ^ seed), :392-393) runs on the host; the block then runs as ONE persistent launch of
// the deterministic split sweep (k_det_sweep_split, kernels_detsweep.hip) -- the superstep's kernel
// with a one-block superstep: every item's updates in shuffle order inside one wave (the hottest
// items as chain + helper pairs on CUs of their own), every user's through per-user tickets -- with
// its wave lists and tickets built on the device by the online plan (kernels_online.hip
// online_sweep_plan / online_det_entries: any item -> wave map gives the same factors).  Bitwise the
// sequential reference order (tests/test_gpu_dsgd.py test_block_update_*).  k outside 64 / 128 /
// 256, slabs past the 32-bit row offsets, or MFHIP_TEST det_kernel=level: one launch per dependency
// level (k_level), the same factors.
namespace {
void block_update_levels(Shard& s, const std::vector<int32_t>& order, const double* r, const int32_t* uidx,
                         const int32_t* iidx, int64_t len, DevBuf& du, DevBuf& di, DevBuf& dru, DevBuf& dri, int64_t nu,
                         int64_t ni, int k, double eta, int64_t& levels) {
  std::vector<uint32_t> uu(uidx, uidx + len), ii(iidx, iidx + len);
  OrderedSeq sq{uu.data(), ii.data(), r, order.data(), len, 0, static_cast<uint32_t>(nu), 0, static_cast<uint32_t>(ni)};
  LevelPlan lp;
  build_level_plan({sq}, lp);
  DevBuf de;
  de.alloc(lp.entries.size() * sizeof(DetEntry));
  MF_HIP(hipMemcpyAsync(de.get(), lp.entries.data(), lp.entries.size() * sizeof(DetEntry), hipMemcpyHostToDevice,
                        s.stream));
  for (int64_t l = 0; l < lp.levels(); ++l) {
    const int64_t b0 = lp.level_start[l], cnt = lp.level_start[l + 1] - b0;
    launch_level(s.stream, de.as<DetEntry>() + b0, cnt, du.get(), di.get(), dru.get(), dri.get(), k, eta, Arith::kDsgd,
                 true);
  }
  MF_HIP(hipGetLastError());
  MF_HIP(hipStreamSynchronize(s.stream));  // lp and de are released on return
  levels = lp.levels();
}
}  // namespace

int mf_block_update(mf_ctx* ctx, const double* r, const int32_t* uidx, const int32_t* iidx, int64_t len,
                    double* users, const int32_t* uomega, int64_t nu, double* items, const int32_t* iomega,
                    int64_t ni, int k, int iteration, int rating_block_id, int64_t seed, double lr,
                    int lr_method, double lr_arg, double lambda) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    MF_REQUIRE(len >= 0 && nu >= 0 && ni >= 0 && k >= 1 && k <= 512, "bad sizes");
    MF_REQUIRE(len == 0 || (r && uidx && iidx && users && items && uomega && iomega), "null argument");
    MF_REQUIRE(len < (int64_t{1} << 31), "a rating block holds fewer than 2^31 ratings");
    std::atomic<int64_t> bad{0};
    parallel_for(len, [&](int64_t b, int64_t e, int) {
      int64_t m = 0;
      for (int64_t j = b; j < e; ++j) m += !(uidx[j] >= 0 && uidx[j] < nu && iidx[j] >= 0 && iidx[j] < ni);
      bad += m;
    });
    MF_REQUIRE(bad == 0, "rating index out of block range");
    if (len == 0) return;
    require_healthy(ctx);
    Shard& s = ctx->shards[0];
    DeviceGuard g(s.device);
    PhaseClock clk;
    std::vector<int32_t> order(len);
    JavaRandom rng(static_cast<int64_t>(iteration ^ rating_block_id) ^ seed);  // DSGDforMF.scala:392
    scala_shuffle(rng, order.data(), len);
    clk.lap("block_update: shuffle");
    const double eta = learning_rate(lr_method, lr, iteration + 1, lambda, lr_arg);  // :383-386
    const size_t ub = static_cast<size_t>(nu) * k * 8, ib = static_cast<size_t>(ni) * k * 8;
    // the block's rows and reg vectors live in the shard's scratch across calls (grow-only)
    DevBuf &du = s.blk_u, &di = s.blk_i, &dru = s.blk_ru, &dri = s.blk_ri;
    du.alloc(std::max<size_t>(ub, 8));
    di.alloc(std::max<size_t>(ib, 8));
    dru.alloc(static_cast<size_t>(std::max<int64_t>(nu, 1)) * 8);
    dri.alloc(static_cast<size_t>(std::max<int64_t>(ni, 1)) * 8);
    {
      std::vector<double> ru(nu), ri(ni);
      for (int64_t x = 0; x < nu; ++x) ru[x] = lambda / static_cast<double>(uomega[x]);
      for (int64_t x = 0; x < ni; ++x) ri[x] = lambda / static_cast<double>(iomega[x]);
      MF_HIP(hipMemcpyAsync(du.get(), users, ub, hipMemcpyHostToDevice, s.stream));
      MF_HIP(hipMemcpyAsync(di.get(), items, ib, hipMemcpyHostToDevice, s.stream));
      MF_HIP(hipMemcpyAsync(dru.get(), ru.data(), static_cast<size_t>(nu) * 8, hipMemcpyHostToDevice, s.stream));
      MF_HIP(hipMemcpyAsync(dri.get(), ri.data(), static_cast<size_t>(ni) * 8, hipMemcpyHostToDevice, s.stream));
      MF_HIP(hipStreamSynchronize(s.stream));  // ru / ri are released here
    }
    const int cap = det_split_capacity(k);
    const bool sweep = cap >= 2 && test_knob("det_kernel") != "level" && ub < 0xFFFFF000ull && ib < 0xFFFFF000ull;
    int64_t levels = 0;
    if (!sweep) {
      block_update_levels(s, order, r, uidx, iidx, len, du, di, dru, dri, nu, ni, k, eta, levels);
    } else {
      // the block in shuffle order, as the online plan takes a batch: rows, rows, ratings (16 B each)
      const size_t in_bytes = static_cast<size_t>(len) * 16;
      MF_HIP(hipStreamSynchronize(s.stream));  // det_pin may still feed an earlier copy
      s.det_pin.alloc(in_bytes);
      uint32_t* pu = s.det_pin.as<uint32_t>();
      uint32_t* pi = pu + len;
      double* pr = reinterpret_cast<double*>(pi + len);
      parallel_for(len, [&](int64_t b, int64_t e, int) {
        for (int64_t x = b; x < e; ++x) {
          const int32_t j = order[x];
          pu[x] = static_cast<uint32_t>(uidx[j]);
          pi[x] = static_cast<uint32_t>(iidx[j]);
          pr[x] = r[j];
        }
      });
      clk.lap("block_update: gather");
      OnlineSweepScratch& sc = s.online_sc;
      sc.in.alloc(in_bytes);
      MF_HIP(hipMemcpyAsync(sc.in.get(), pu, in_bytes, hipMemcpyHostToDevice, s.stream));
      const int64_t W = std::max<int64_t>(1, std::min<int64_t>({static_cast<int64_t>(cap / 2), 4096, len}));
      const size_t ebytes = static_cast<size_t>(len) * sizeof(DetEntry), qbytes = static_cast<size_t>(len) * 4;
      s.det_dev.alloc(ebytes + qbytes);
      sc.wbeg.alloc(static_cast<size_t>(W + 1) * 8);
      sc.touched.alloc(8);
      const uint32_t* dpu = sc.in.as<uint32_t>();
      online_sweep_plan(s.stream, sc, dpu, dpu + len, reinterpret_cast<const double*>(dpu + 2 * len), len,
                        static_cast<uint32_t>(W), static_cast<uint32_t>(nu), static_cast<uint32_t>(ni),
                        s.det_dev.as<DetEntry>(), reinterpret_cast<uint32_t*>(s.det_dev.as<char>() + ebytes),
                        sc.wbeg.as<int64_t>(), sc.touched.as<int32_t>());
      uint32_t *eu = nullptr, *ei = nullptr, *eq = nullptr;
      double* er = nullptr;
      sc.waves.alloc(static_cast<size_t>(det_slot_room(W)) * sizeof(DetWave));
      online_det_entries(s.stream, sc, s.det_dev.as<DetEntry>(),
                         reinterpret_cast<const uint32_t*>(s.det_dev.as<char>() + ebytes), sc.wbeg.as<int64_t>(), len,
                         static_cast<uint32_t>(W), eu, ei, eq, er, sc.waves.as<DetWave>());
      std::vector<DetWave> slots(static_cast<size_t>(det_slot_room(W)));
      MF_HIP(hipMemcpyAsync(slots.data(), sc.waves.get(), static_cast<size_t>(W) * sizeof(DetWave),
                            hipMemcpyDeviceToHost, s.stream));
      MF_HIP(hipStreamSynchronize(s.stream));
      const int64_t nslots =
          det_slot_table(slots.data(), W, cap / 2, test_knob("det_alone") != "0", device_cu_count(s.device));
      MF_HIP(hipMemcpyAsync(sc.waves.get(), slots.data(), static_cast<size_t>(nslots) * sizeof(DetWave),
                            hipMemcpyHostToDevice, s.stream));
      sc.uticket.alloc(static_cast<size_t>(std::max<int64_t>(nu, 1)) * 4);
      MF_HIP(hipMemsetAsync(sc.uticket.get(), 0, static_cast<size_t>(std::max<int64_t>(nu, 1)) * 4, s.stream));
      sc.err.alloc(4);
      MF_HIP(hipMemsetAsync(sc.err.get(), 0, 4, s.stream));
      {
        LaunchTimer t(s, ctx->profiling, true);
        launch_det_sweep_split(s.stream, sc.waves.as<DetWave>(), static_cast<int>(nslots), eu, ei, eq, er,
                               du.as<double>(), di.as<double>(), ub, ib, dru.as<double>(), dri.as<double>(), k, eta,
                               sc.uticket.as<int32_t>(), sc.err.as<int32_t>(), t.start(), t.stop());
      }
      MF_HIP(hipGetLastError());
      int32_t err = 0;
      MF_HIP(hipMemcpyAsync(&err, sc.err.get(), 4, hipMemcpyDeviceToHost, s.stream));
      MF_HIP(hipStreamSynchronize(s.stream));
      clk.lap("block_update: plan + sweep");
      if (err) {
        ctx->failed = "block update sweep: a wave waited > 1 s for a user ticket (waves not co-resident?); "
                      "set MFHIP_TEST=det_kernel=level (INTEGRATION.md section 5)";
        fail(MF_ERR_TIMEOUT, ctx->failed);
      }
      ctx->stats.kernel_launches += 1;
    }
    MF_HIP(hipMemcpyAsync(users, du.get(), ub, hipMemcpyDeviceToHost, s.stream));
    MF_HIP(hipMemcpyAsync(items, di.get(), ib, hipMemcpyDeviceToHost, s.stream));
    MF_HIP(hipStreamSynchronize(s.stream));
    clk.lap("block_update: download");
    ctx->stats.updates += len;
    ctx->stats.levels += levels;
  });
}

int mf_online_update(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n, int flavour,
                     int num_partitions, int64_t* touched_users, int64_t* touched_items) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    det_spec_wait(ctx, true);  // new ids change the layouts the builds read
    online_update(ctx, u, i, r, n, flavour, num_partitions, touched_users, touched_items);
  });
}

int mf_online_update_out(mf_ctx* ctx, const int32_t* u, const int32_t* i, const double* r, int64_t n, int flavour,
                         int num_partitions, int64_t* touched_users, int64_t* touched_items, double* user_out,
                         double* item_out) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    det_spec_wait(ctx, true);  // new ids change the layouts the builds read
    online_update(ctx, u, i, r, n, flavour, num_partitions, touched_users, touched_items, user_out, item_out);
  });
}

int mf_lookup(mf_ctx* ctx, int side, const int32_t* ids, int64_t n, double* vecs_out, uint8_t* found) {
  return guarded([&] {
    MF_REQUIRE(ctx && (n == 0 || (ids && vecs_out && found)), "null argument");
    MF_REQUIRE(side == MF_SIDE_USER || side == MF_SIDE_ITEM, "bad side");
    MF_REQUIRE(ctx->have_model, "no model");
    Shard& s = ctx->shards[0];
    if (!ctx->rank_mode) consolidate(ctx, s);
    else if (side == MF_SIDE_ITEM) allgather_items(ctx);
    sync_all(ctx);
    const SideLayout& S = side_of(ctx, side);
    const int k = ctx->P.num_factors;
    std::vector<double> row(k);
    for (int64_t j = 0; j < n; ++j) {
      const int32_t x = S.index.find(ids[j]);
      found[j] = x >= 0;
      if (x < 0) { std::fill(vecs_out + j * k, vecs_out + (j + 1) * k, 0.0); continue; }
      download_rows(ctx, s, side, x, 1, vecs_out + static_cast<size_t>(j) * k);
    }
  });
}

int mf_set_profiling(mf_ctx* ctx, int on) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    sync_all(ctx);
    ctx->profiling = on != 0;
  });
}

int mf_get_stats(mf_ctx* ctx, mf_stats* out) {
  return guarded([&] {
    MF_REQUIRE(ctx && out, "null argument");
    sync_all(ctx);
    ctx->stats.algorithmic_bytes = static_cast<double>(ctx->stats.updates) * bytes_per_update(ctx);
    *out = ctx->stats;
  });
}

int mf_reset_stats(mf_ctx* ctx) {
  return guarded([&] {
    MF_REQUIRE(ctx, "null context");
    sync_all(ctx);
    const int32_t groups = ctx->stats.groups;
    const int64_t pads = ctx->stats.pads;
    ctx->stats = mf_stats{};
    ctx->stats.groups = groups;
    ctx->stats.pads = pads;
  });
}

int mf_jvm_shuffle(int64_t seed, int64_t len, int32_t* out) {
  return guarded([&] {
    MF_REQUIRE(len >= 0 && (len == 0 || out), "bad argument");
    JavaRandom rng(seed);
    scala_shuffle(rng, out, len);
  });
}

int mf_jvm_block_of(int32_t id, int64_t seed, int32_t n_blocks, int32_t* out) {
  return guarded([&] {
    MF_REQUIRE(out && n_blocks >= 1, "bad argument");
    JavaRandom rng(static_cast<int64_t>(id) ^ seed);
    *out = rng.nextInt(n_blocks);
  });
}

int mf_jvm_random_factors(int64_t rng_seed, int32_t k, double* out) {
  return guarded([&] {
    MF_REQUIRE(out && k >= 0, "bad argument");
    JavaRandom rng(rng_seed);
    for (int32_t f = 0; f < k; ++f) out[f] = rng.nextDouble();
  });
}

int mf_debug_levels(const uint32_t* urow, const uint32_t* irow, const int32_t* order, int64_t n, int32_t* level_out) {
  return guarded([&] {
    MF_REQUIRE(n >= 0 && (n == 0 || (urow && irow && level_out)), "bad argument");
    if (n == 0) return;
    uint32_t umax = 0, imax = 0;
    for (int64_t j = 0; j < n; ++j) { umax = std::max(umax, urow[j]); imax = std::max(imax, irow[j]); }
    std::vector<double> zero(n, 0.0);
    OrderedSeq sq{urow, irow, zero.data(), order, n, 0, umax + 1, 0, imax + 1};
    // levels in sequence order: replay the same recurrence build_level_plan uses
    LevelPlan lp;
    build_level_plan({sq}, lp);
    std::vector<int32_t> lu(umax + 1, 0), li(imax + 1, 0);
    for (int64_t j = 0; j < n; ++j) {
      const int64_t e = order ? order[j] : j;
      const int32_t l = std::max(lu[urow[e]], li[irow[e]]) + 1;
      lu[urow[e]] = l;
      li[irow[e]] = l;
      level_out[j] = l;
    }
    MF_REQUIRE(lp.levels() == (n ? *std::max_element(level_out, level_out + n) : 0), "level count mismatch");
  });
}

int mf_debug_fast_schedule(const int32_t* u, const int32_t* i, int64_t n, int32_t n_blocks, int64_t seed,
                           int32_t groups, int32_t blocking, int32_t window, int32_t k, int32_t* block_out,
                           int32_t* substep_out, int32_t* group_out, int64_t* pos_out) {
  return mf_debug_fast_split(u, i, n, n_blocks, seed, groups, blocking, window, k, 0, block_out, substep_out, group_out,
                             pos_out, nullptr);
}

namespace mfhip {
namespace {
int debug_fast_plan(const int32_t* u, const int32_t* i, int64_t n, int32_t n_blocks, int64_t seed, int32_t groups,
                    int32_t blocking, int32_t window, int32_t k, int32_t item_split, int32_t* block_out, int32_t* substep_out, int32_t* group_out, int64_t* pos_out,
                    int32_t* replica_out) {
  return guarded([&] {
    MF_REQUIRE(n >= 0 && n_blocks >= 1 && groups != 0 && item_split >= 0 && k >= 1, "bad argument");
    MF_REQUIRE(n == 0 || (u && i && block_out && substep_out && group_out && pos_out), "null argument");
    SideLayout U, I;
    const Blocking bl = blocking == MF_BLOCKING_BALANCED ? Blocking::kBalanced : Blocking::kJvm;
    build_side(U, u, n, n_blocks, seed, true, bl);
    build_side(I, i, n, n_blocks, seed, true, bl);
    std::vector<double> r(n, 1.0);
    RatingBlocks rb;
    build_rating_blocks(rb, U, I, u, i, r.data(), n, 0, n_blocks, false, true);
    FastPlan fp;
    std::vector<int64_t> src;
    std::vector<int32_t> block_groups;  // groups < 0: the systolic per-block choice for -groups waves
    if (groups < 0)
      block_groups = choose_block_groups(rb, I, n_blocks, 0, -groups, item_split, sys_cell_ns(k), sys_run_pair_ns(k));
    const uint32_t scratch_base = static_cast<uint32_t>(I.rows() + 1);
    build_fast_plan(fp, rb, U, I, groups > 0 ? groups : 8, 1, 1.0,
                    static_cast<uint64_t>(seed) * 0x9E3779B97F4A7C15ULL + 1, static_cast<uint32_t>(U.rows()), &src,
                    window > 0 ? window : kHazardWindow, block_groups.empty() ? nullptr : &block_groups, item_split,
                    scratch_base);
    const int64_t nb2 = static_cast<int64_t>(n_blocks) * n_blocks;
    for (int64_t b = 0; b < nb2; ++b) {
      if (fp.rec_base[b] < 0) continue;
      const int32_t G = fp.Gb[b];
      const int64_t GG = static_cast<int64_t>(G) * G;
      const int32_t* off = fp.cell_off.data() + fp.cell_base[b];
      for (int64_t cidx = 0; cidx < GG; ++cidx)
        for (int64_t x = off[cidx]; x < off[cidx + 1]; ++x) {
          if (src[fp.rec_base[b] + x] < 0) continue;  // padding
          const int64_t j = rb.src[src[fp.rec_base[b] + x]];
          block_out[j] = static_cast<int32_t>(b);
          substep_out[j] = static_cast<int32_t>(cidx / G);
          group_out[j] = static_cast<int32_t>(cidx % G);
          pos_out[j] = x - off[cidx];
          if (replica_out) {  // 0: the item's own row; r: its replica r (scratch row)
            const uint32_t row = fp.recs[fp.rec_base[b] + x].i & ~kPadBit;
            int32_t rep = 0;
            if (row >= scratch_base)
              for (int64_t h = fp.split_off[b]; h < fp.split_off[b + 1]; ++h)
                if (row >= fp.splits[h].scratch_row && row < fp.splits[h].scratch_row + fp.splits[h].R - 1)
                  rep = static_cast<int32_t>(row - fp.splits[h].scratch_row) + 1;
            replica_out[j] = rep;
          }
        }
    }
  });
}

}  // namespace
}  // namespace mfhip

int mf_debug_fast_split(const int32_t* u, const int32_t* i, int64_t n, int32_t n_blocks, int64_t seed,
                        int32_t groups, int32_t blocking, int32_t window, int32_t k, int32_t item_split,
                        int32_t* block_out, int32_t* substep_out, int32_t* group_out, int64_t* pos_out,
                        int32_t* replica_out) {
  return mfhip::debug_fast_plan(u, i, n, n_blocks, seed, groups, blocking, window, k, item_split, block_out,
                                substep_out, group_out, pos_out, replica_out);
}

const char* mf_fast_kernel_name(int32_t k) {
  switch (choose_fast_kernel(k)) {
    case FastKernel::kPair: return want_pair_sys() ? "k_sweep_pair_sys" : "k_sweep_pair";
    case FastKernel::kPersistent: return "k_fast_superstep";
    default: return "k_fast_substep";
  }
}

int32_t mf_debug_build_flags(void) { return mfhip::kExperiments ? 1 : 0; }

int mf_debug_device_bytes(int64_t out[2]) {
  if (!out) return MF_ERR_INVALID;
  out[0] = mfhip::dev_bytes_live().load();
  out[1] = mfhip::dev_bytes_peak().load();
  return MF_OK;
}

int mf_debug_plan_digest(mf_ctx* ctx, uint64_t out[2]) {
  return guarded([&] {
    MF_REQUIRE(ctx && out, "null argument");
    MF_REQUIRE(ctx->prepared && !ctx->f64 && ctx->fast_pair && ctx->shards.size() == 1,
               "mf_debug_plan_digest needs a prepared fast-mode pair fit on one shard");
    sync_all(ctx);
    Shard& s = ctx->shards[0];
    DeviceGuard g(s.device);
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const DevBuf& d, size_t bytes) {
      std::vector<unsigned char> v(bytes);
      if (bytes) MF_HIP(hipMemcpy(v.data(), d.get(), bytes, hipMemcpyDeviceToHost));
      for (unsigned char c : v) { h ^= c; h *= 1099511628211ull; }
    };
    mix(s.st_recs, static_cast<size_t>(s.st_nrecs) * sizeof(PairRec));
    mix(s.st_waves, s.st_sub_off.empty() ? 0 : static_cast<size_t>(s.st_sub_off.back()) * sizeof(WaveDesc));
    if (ctx->fast_sys) {
      mix(s.st_sys, s.st_sys.bytes());
      mix(s.st_sysw, s.st_sysw.bytes());
    }
    out[0] = h;
    out[1] = static_cast<uint64_t>(s.st_nrecs);
  });
}

int mf_debug_ring_schedule(int32_t rank, int32_t world, int32_t n_blocks, int64_t superstep, int32_t* out_blk,
                           int32_t* in_blk, int32_t* dst, int32_t* src) {
  return guarded([&] {
    MF_REQUIRE(out_blk && in_blk && dst && src, "null argument");
    MF_REQUIRE(world >= 1 && rank >= 0 && rank < world && n_blocks >= 1 && n_blocks % world == 0 && superstep >= 1,
               "bad ring arguments (n_blocks must be a multiple of world, superstep >= 1)");
    const RingStep rs = ring_step(rank, world, n_blocks / world, n_blocks, superstep);
    *out_blk = rs.out_blk;
    *in_blk = rs.in_blk;
    *dst = rs.dst;
    *src = rs.src;
  });
}

int mf_fast_plan_window(int32_t k, int32_t* window_out) {
  return guarded([&] {
    MF_REQUIRE(window_out, "null");
    const FastKernel fk = choose_fast_kernel(k);
    *window_out = fk == FastKernel::kPair ? plan_window(k) : kHazardWindow;
  });
}

int mf_learning_rate(int method, double lr, int32_t iteration, double lambda, double arg, double* out) {
  return guarded([&] {
    MF_REQUIRE(out, "null");
    MF_REQUIRE(method >= MF_LR_DEFAULT && method <= MF_LR_XU, "unknown lr_method");
    *out = learning_rate(method, lr, iteration, lambda, arg);
  });
}

}  // extern "C"
