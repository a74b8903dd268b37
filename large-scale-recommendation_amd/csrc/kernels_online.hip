// kernels_online.hip -- the inputs of k_online_sweep (kernels_det.hip) built on the device from
// one micro-batch in sequence order (SGDUpdater.nextFactors applied in arrival order,
// core/FactorUpdater.scala:37-53, OnlineSpark.scala:191-194 / FlinkOnlineMF.scala's per-rating
// updates).  The host version of the same plan (a sequential counting sort) cost more than the
// sweep it fed; this one is two stable radix sorts and three gathers:
//   tickets : stable sort of (user row, x) -> an update's ticket value is its rank inside its
//             user's run = the number of earlier updates of that user (the kernel waits until
//             the user's ticket word reaches it)
//   waves   : stable sort of (wave of the item row, x) -> wave w's updates in sequence order; every
//             update of an item lands in one wave, so the item's order is the sequence order.  An
//             item with at least the mean wave load (on a 1-in-4 sample) gets a wave of its own
//             (waves 0 .. H-1 in row order; any item -> wave map gives the same factors), the others
//             go to H + row mod (W - H).  The hottest items' chains bound the launch, so they should
//             not share their wave with other items' updates.
//   wbeg[w] : first position of wave w (lower bound in the sorted wave keys), wbeg[W] = n
//   touched : distinct user rows (run heads of the user sort) and item rows (a flag per item row)
//             of the batch (UpdateSeparatedHashMap.updates, OfflineSpark.scala:33-67)
// HBM-bound integer work (4-byte keys, 4-byte payloads).  Bitwise the host plan: the factors of
// the sweep equal the level replay's (tests/test_gpu_online.py).

#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_reduce.hpp>
#include <hipcub/device/device_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "common.hpp"
#include "kernels.hpp"

namespace mfhip {
namespace {

constexpr int kThreads = 256;
unsigned grid_for(int64_t n) {
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, 1 << 16)));
}

// per item row, the updates of every S-th entry of the batch (the heavy items only need to be found,
// not counted exactly: any item -> wave map gives the same factors; a sample cuts the atomics on
// the hottest counters S-fold).  Rows >= rows (an id the device lookup did not find: the plan is
// built before the host has seen the miss count, and rebuilt when there are misses) are skipped.
__global__ void k_item_count(const uint32_t* __restrict__ ei, int64_t n, int S, uint32_t rows,
                             uint32_t* __restrict__ cnt) {
  for (int64_t x = (blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x) * S; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x * S) {
    const uint32_t i = ei[x];
    if (i < rows) atomicAdd(cnt + i, 1u);
  }
}

// iwave[item] = its rank among the items with cnt >= Ts in row order when that rank is < H, else
// -1: one block, each thread a contiguous run of rows, a block-wide exclusive scan of the runs'
// counts in LDS (one launch instead of flags + a device scan + an assign pass: ~4 launches of
// 8-9 us each on the critical path of a batch's plan)
constexpr int kHeavyThreads = 1024;
__global__ __launch_bounds__(kHeavyThreads) void k_heavy_assign(const uint32_t* __restrict__ cnt, uint32_t rows,
                                                                 uint32_t Ts, uint32_t H, int32_t* __restrict__ iwave) {
  __shared__ uint32_t part[kHeavyThreads];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (rows + kHeavyThreads - 1) / kHeavyThreads;
  const uint32_t lo = min(rows, t * per), hi = min(rows, lo + per);
  uint32_t c = 0;
  for (uint32_t i = lo; i < hi; ++i) c += cnt[i] >= Ts;
  part[t] = c;
  __syncthreads();
  for (uint32_t d = 1; d < kHeavyThreads; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t pos = part[t] - c;  // exclusive
  for (uint32_t i = lo; i < hi; ++i) {
    const bool heavy = cnt[i] >= Ts;
    iwave[i] = heavy && pos < H ? static_cast<int32_t>(pos) : -1;
    pos += heavy;
  }
}

__global__ void k_iota(int64_t n, int32_t* __restrict__ iota) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    iota[i] = static_cast<int32_t>(i);
}

__global__ void k_keys(const uint32_t* __restrict__ eu, const uint32_t* __restrict__ ei, int64_t n, uint32_t W,
                       uint32_t H, const int32_t* __restrict__ iwave, uint32_t rows, uint32_t* __restrict__ wkey,
                       int32_t* __restrict__ iota) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t i = ei[x];
    const int32_t w = iwave && i < rows ? iwave[i] : -1;  // (i >= rows: a miss, k_item_count)
    wkey[x] = w >= 0 ? static_cast<uint32_t>(w) : H + i % (W - H);
    iota[x] = static_cast<int32_t>(x);
  }
}

// head[p] = p where a user's run starts in the user-sorted keys, else 0 (a max-scan then gives
// every position its run start)
__global__ void k_run_heads(const uint32_t* __restrict__ ukey, int64_t n, int32_t* __restrict__ head) {
  for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < n;
       p += static_cast<int64_t>(gridDim.x) * blockDim.x)
    head[p] = (p == 0 || ukey[p] != ukey[p - 1]) ? static_cast<int32_t>(p) : 0;
}

__global__ void k_tickets(const int32_t* __restrict__ ux, const int32_t* __restrict__ start, int64_t n,
                          uint32_t* __restrict__ ticket) {
  for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < n;
       p += static_cast<int64_t>(gridDim.x) * blockDim.x)
    ticket[ux[p]] = static_cast<uint32_t>(p - start[p]);
}

// R: the uploaded ratings' type (float: the f32 sweep's upload, rounded on the host -- the sweep
// rounds r to float first in any case, online_f32.hpp)
template <typename R>
__global__ void k_gather(const int32_t* __restrict__ wx, const uint32_t* __restrict__ eu,
                         const uint32_t* __restrict__ ei, const R* __restrict__ er,
                         const uint32_t* __restrict__ ticket, int64_t n, DetEntry* __restrict__ ent,
                         uint32_t* __restrict__ useq) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < n;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t x = wx[y];
    ent[y] = DetEntry{eu[x], ei[x], static_cast<double>(er[x])};
    useq[y] = ticket[x];
  }
}

__global__ void k_wave_begin(const uint32_t* __restrict__ wsorted, int64_t n, uint32_t W, int64_t* __restrict__ wbeg) {
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w <= W;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t lo = 0, hi = n;  // first position whose key is >= w
    while (lo < hi) {
      const int64_t mid = (lo + hi) / 2;
      if (wsorted[mid] < static_cast<uint32_t>(w)) lo = mid + 1;
      else hi = mid;
    }
    wbeg[w] = lo;
  }
}

// flag[row] = 1 for every row of the batch (rows >= rows: lookup misses, skipped)
__global__ void k_row_flags(const uint32_t* __restrict__ rowv, int64_t n, uint32_t rows, int32_t* __restrict__ flag) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t r = rowv[x];
    if (r < rows) flag[r] = 1;
  }
}

__global__ void k_head_flags(const uint32_t* __restrict__ sorted, int64_t n, int32_t* __restrict__ flag) {
  for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < n;
       p += static_cast<int64_t>(gridDim.x) * blockDim.x)
    flag[p] = (p == 0 || sorted[p] != sorted[p - 1]) ? 1 : 0;
}

// The plan's stable sorts: rocprim's radix sort with the merge-sort path off.  Its default config
// sorts up to 2^20 keys by block sort + 8 merge passes (17 launches of 5-10 us for a 1M batch,
// gpurun_out/r6o); onesweep takes a histogram, a scan and one pass per 8 key bits.  Both are stable:
// the same output.
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

int bits_for(uint64_t v) {  // radix bits that hold every key < v
  int b = 1;
  while (b < 32 && (uint64_t{1} << b) < v) ++b;
  return b;
}

// The deterministic sweep's entry arrays (SoA, padded with kDetPad zero entries: the sweep reads
// whole chunks past a wave's end) from the plan's wave-ordered entries
__global__ void k_det_soa(const DetEntry* __restrict__ ent, const uint32_t* __restrict__ useq, int64_t n,
                          int64_t total, uint32_t* __restrict__ eu, uint32_t* __restrict__ ei, uint32_t* __restrict__ eq,
                          double* __restrict__ er) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < total;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const bool live = y < n;
    eu[y] = live ? ent[y].u : 0u;
    ei[y] = live ? ent[y].i : 0u;
    eq[y] = live ? useq[y] : 0u;
    er[y] = live ? ent[y].r : 0.0;
  }
}

// multi[w] = 1 when wave w holds more than one item (wkey = the sorted wave keys: wave of position y)
__global__ void k_multi(const DetEntry* __restrict__ ent, const uint32_t* __restrict__ wkey,
                        const int64_t* __restrict__ wbeg, int64_t n, int32_t* __restrict__ multi) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < n;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t w = wkey[y];
    if (ent[y].i != ent[wbeg[w]].i) multi[w] = 1;
  }
}

__global__ void k_det_waves(const int64_t* __restrict__ wbeg, const int32_t* __restrict__ multi, uint32_t W,
                            DetWave* __restrict__ waves) {
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w < W;
       w += static_cast<int64_t>(gridDim.x) * blockDim.x)
    waves[w] = DetWave{wbeg[w], static_cast<int32_t>(wbeg[w + 1] - wbeg[w]), multi[w] ? 0 : kDetWaveSingleItem};
}

}  // namespace

namespace {
// IdIndex::hash (id_index.hpp), the same bits on the device
__device__ __forceinline__ uint64_t id_hash(int32_t id) {
  uint64_t x = static_cast<uint32_t>(id);
  x ^= x >> 16; x *= 0x7feb352dULL; x ^= x >> 15; x *= 0x846ca68bULL; x ^= x >> 16;
  return x;
}
// linear probing over a mirror of the host table: the row, or 0xFFFFFFFF (absent / empty table)
__device__ __forceinline__ uint32_t id_find(const int2* __restrict__ slots, uint64_t mask, int32_t id) {
  if (!slots) return 0xFFFFFFFFu;
  uint64_t h = id_hash(id) & mask;
  for (;;) {
    const int2 sl = slots[h];
    if (sl.y < 0) return 0xFFFFFFFFu;
    if (sl.x == id) return static_cast<uint32_t>(sl.y);
    h = (h + 1) & mask;
  }
}
__global__ __launch_bounds__(kThreads) void k_id_lookup(uint32_t* __restrict__ in, int64_t n,
                                                       const int2* __restrict__ us, uint64_t um,
                                                       const int2* __restrict__ is, uint64_t im,
                                                       int32_t* __restrict__ misses) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  int m = 0;
  if (j < n) {
    const uint32_t ur = id_find(us, um, static_cast<int32_t>(in[j]));
    const uint32_t ir = id_find(is, im, static_cast<int32_t>(in[n + j]));
    in[j] = ur;
    in[n + j] = ir;
    m = (ur == 0xFFFFFFFFu) + (ir == 0xFFFFFFFFu);
  }
  // one atomic per wave
  const int tot = __popcll(__ballot(m >= 1)) + __popcll(__ballot(m == 2));
  if ((threadIdx.x & 63) == 0 && tot) atomicAdd(misses, tot);
}
__global__ __launch_bounds__(kThreads) void k_id_scatter(int2* __restrict__ slots, const uint32_t* __restrict__ pos,
                                                        const int2* __restrict__ vals, int64_t m) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (j < m) slots[pos[j]] = vals[j];
}
}  // namespace

void launch_id_lookup(hipStream_t st, uint32_t* in, int64_t n, const void* uslots, uint64_t umask, const void* islots,
                      uint64_t imask, int32_t* misses) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_id_lookup, dim3(grid_for(n)), dim3(kThreads), 0, st, in, n, static_cast<const int2*>(uslots),
                     umask, static_cast<const int2*>(islots), imask, misses);
  MF_HIP(hipGetLastError());
}

void launch_id_scatter(hipStream_t st, void* slots, const uint32_t* pos, const void* vals, int64_t m) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_id_scatter, dim3(grid_for(m)), dim3(kThreads), 0, st, static_cast<int2*>(slots), pos,
                     static_cast<const int2*>(vals), m);
  MF_HIP(hipGetLastError());
}

void online_det_entries(hipStream_t st, OnlineSweepScratch& sc, const DetEntry* ent, const uint32_t* useq,
                        const int64_t* wbeg, int64_t n, uint32_t W, uint32_t*& eu, uint32_t*& ei, uint32_t*& eq,
                        double*& er, DetWave* waves) {
  const int64_t total = n + kDetPad;
  sc.soa.alloc(static_cast<size_t>(total) * 20);
  er = sc.soa.as<double>();
  eu = reinterpret_cast<uint32_t*>(er + total);
  ei = eu + total;
  eq = ei + total;
  hipLaunchKernelGGL(k_det_soa, dim3(grid_for(total)), dim3(kThreads), 0, st, ent, useq, n, total, eu, ei, eq, er);
  sc.multi.alloc(static_cast<size_t>(W) * 4);
  MF_HIP(hipMemsetAsync(sc.multi.get(), 0, static_cast<size_t>(W) * 4, st));
  hipLaunchKernelGGL(k_multi, dim3(grid_for(n)), dim3(kThreads), 0, st, ent, sc.wkey2.as<uint32_t>(), wbeg, n,
                     sc.multi.as<int32_t>());
  hipLaunchKernelGGL(k_det_waves, dim3(grid_for(W)), dim3(kThreads), 0, st, wbeg, sc.multi.as<int32_t>(), W, waves);
  MF_HIP(hipGetLastError());
}

uint32_t online_sweep_plan(hipStream_t st, OnlineSweepScratch& sc, const uint32_t* eu, const uint32_t* ei,
                           const double* er, int64_t n, uint32_t W, uint32_t user_rows, uint32_t item_rows,
                           DetEntry* ent, uint32_t* useq, int64_t* wbeg, int32_t* touched, const float* erf) {
  MF_REQUIRE(n > 0 && n < (int64_t{1} << 31) && W >= 1, "online sweep plan: bad batch shape");
  const int N = static_cast<int>(n);
  sc.ukey.alloc(n * 4);
  sc.wkey.alloc(n * 4);
  sc.wkey2.alloc(n * 4);
  sc.iota.alloc(n * 4);
  sc.ux.alloc(n * 4);
  sc.wx.alloc(n * 4);
  sc.head.alloc(n * 4);
  sc.start.alloc(n * 4);
  sc.ticket.alloc(n * 4);
  // heavy items: at least the mean wave load, at most a quarter of the waves (MFHIP_TEST
  // online_heavy=m: m times the mean instead, 0: none; online_heavy_cap=d: at most W/d -- the A/B
  // switches, profiles/r05_online_heavy_ab.txt)
  double mult = 1.0;
  if (const std::string v = test_knob("online_heavy"); !v.empty()) mult = std::atof(v.c_str());
  uint32_t cap_div = 4;
  if (const std::string v = test_knob("online_heavy_cap"); !v.empty()) cap_div = std::max(2, std::atoi(v.c_str()));
  const uint32_t H = W >= 8 && mult > 0.0 ? W / cap_div : 0;
  const uint32_t T = static_cast<uint32_t>(std::max<double>(2.0, std::ceil(mult * static_cast<double>(n) / W)));
  size_t tb = 0;
  if (H > 0 && item_rows > 0) {
    // the items that reach T on a 1-in-kSample sample of the batch, in row order, at most H of them
    // (round 5 sorted the exact counts and took the H largest: 78 us of contended atomics and a
    // radix sort per NFLX 1M batch, profiles/r06_online_batch_timeline.txt; a batch has a few dozen
    // heavy items against H = W / 4)
    constexpr int kSample = 4;
    const size_t ib = static_cast<size_t>(item_rows) * 4;
    sc.icnt.alloc(ib);
    sc.iwave.alloc(ib);
    uint32_t* cnt = sc.icnt.as<uint32_t>();
    MF_HIP(hipMemsetAsync(cnt, 0, ib, st));
    hipLaunchKernelGGL(k_item_count, dim3(grid_for((n + kSample - 1) / kSample)), dim3(kThreads), 0, st, ei, n, kSample,
                       item_rows, cnt);
    const uint32_t Ts = std::max<uint32_t>(1, (T + kSample - 1) / kSample);
    hipLaunchKernelGGL(k_heavy_assign, dim3(1), dim3(kHeavyThreads), 0, st, cnt, item_rows, Ts, H,
                       sc.iwave.as<int32_t>());
  }
  hipLaunchKernelGGL(k_keys, dim3(grid_for(n)), dim3(kThreads), 0, st, eu, ei, n, W, H,
                     H > 0 && item_rows > 0 ? sc.iwave.as<int32_t>() : nullptr, item_rows, sc.wkey.as<uint32_t>(),
                     sc.iota.as<int32_t>());
  const int ub = bits_for(user_rows), wb = bits_for(W);
  // tickets on s2 (user sort, run starts, ranks) and the touched items on s3 (item-row flags)
  // run beside the wave keys and the wave sort on st; both only read the uploaded batch
  sc.side_streams();
  sc.iota2.alloc(n * 4);
  sc.iflag.alloc(static_cast<size_t>(std::max<uint32_t>(item_rows, 1)) * 4);
  MF_HIP(hipEventRecord(sc.ev_in, st));
  MF_HIP(hipStreamWaitEvent(sc.s2, sc.ev_in, 0));
  MF_HIP(hipStreamWaitEvent(sc.s3, sc.ev_in, 0));
  size_t tb2 = 0, tb3 = 0;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kThreads), 0, sc.s2, n, sc.iota2.as<int32_t>());
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, tb2, eu, sc.ukey.as<uint32_t>(), sc.iota2.as<int32_t>(),
                                             sc.ux.as<int32_t>(), N, 0, ub, sc.s2));
  sc.tmp2.alloc(std::max<size_t>(tb2, 256));
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(sc.tmp2.get(), tb2, eu, sc.ukey.as<uint32_t>(), sc.iota2.as<int32_t>(),
                                             sc.ux.as<int32_t>(), N, 0, ub, sc.s2));
  hipLaunchKernelGGL(k_run_heads, dim3(grid_for(n)), dim3(kThreads), 0, sc.s2, sc.ukey.as<uint32_t>(), n,
                     sc.head.as<int32_t>());
  MF_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb2, sc.head.as<int32_t>(), sc.start.as<int32_t>(), hipcub::Max(),
                                           N, sc.s2));
  sc.tmp2.alloc(std::max<size_t>(tb2, 256));
  MF_HIP(hipcub::DeviceScan::InclusiveScan(sc.tmp2.get(), tb2, sc.head.as<int32_t>(), sc.start.as<int32_t>(),
                                           hipcub::Max(), N, sc.s2));
  hipLaunchKernelGGL(k_tickets, dim3(grid_for(n)), dim3(kThreads), 0, sc.s2, sc.ux.as<int32_t>(), sc.start.as<int32_t>(),
                     n, sc.ticket.as<uint32_t>());
  // touched users: run heads of the user-sorted keys (s2)
  hipLaunchKernelGGL(k_head_flags, dim3(grid_for(n)), dim3(kThreads), 0, sc.s2, sc.ukey.as<uint32_t>(), n,
                     sc.head.as<int32_t>());
  MF_HIP(hipcub::DeviceReduce::Sum(nullptr, tb2, sc.head.as<int32_t>(), touched, N, sc.s2));
  sc.tmp2.alloc(std::max<size_t>(tb2, 256));
  MF_HIP(hipcub::DeviceReduce::Sum(sc.tmp2.get(), tb2, sc.head.as<int32_t>(), touched, N, sc.s2));
  MF_HIP(hipEventRecord(sc.ev2, sc.s2));
  // touched items (s3): a flag per item row, summed
  const int nir = static_cast<int>(std::max<uint32_t>(item_rows, 1));
  MF_HIP(hipMemsetAsync(sc.iflag.get(), 0, static_cast<size_t>(nir) * 4, sc.s3));
  hipLaunchKernelGGL(k_row_flags, dim3(grid_for(n)), dim3(kThreads), 0, sc.s3, ei, n, item_rows, sc.iflag.as<int32_t>());
  MF_HIP(hipcub::DeviceReduce::Sum(nullptr, tb3, sc.iflag.as<int32_t>(), touched + 1, nir, sc.s3));
  sc.tmp3.alloc(std::max<size_t>(tb3, 256));
  MF_HIP(hipcub::DeviceReduce::Sum(sc.tmp3.get(), tb3, sc.iflag.as<int32_t>(), touched + 1, nir, sc.s3));
  MF_HIP(hipEventRecord(sc.ev3, sc.s3));
  // waves (st): the wave sort, then the gather once the tickets are in
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, tb, sc.wkey.as<uint32_t>(), sc.wkey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.wx.as<int32_t>(), N, 0, wb, st));
  sc.tmp.alloc(std::max<size_t>(tb, 256));
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(sc.tmp.get(), tb, sc.wkey.as<uint32_t>(), sc.wkey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.wx.as<int32_t>(), N, 0, wb, st));
  hipLaunchKernelGGL(k_wave_begin, dim3(grid_for(W + 1)), dim3(kThreads), 0, st, sc.wkey2.as<uint32_t>(), n, W,
                     wbeg);
  MF_HIP(hipStreamWaitEvent(st, sc.ev2, 0));
  if (erf)
    hipLaunchKernelGGL(k_gather<float>, dim3(grid_for(n)), dim3(kThreads), 0, st, sc.wx.as<int32_t>(), eu, ei, erf,
                       sc.ticket.as<uint32_t>(), n, ent, useq);
  else
    hipLaunchKernelGGL(k_gather<double>, dim3(grid_for(n)), dim3(kThreads), 0, st, sc.wx.as<int32_t>(), eu, ei, er,
                       sc.ticket.as<uint32_t>(), n, ent, useq);
  MF_HIP(hipStreamWaitEvent(st, sc.ev3, 0));  // touched[1]; and nothing on s3 outlives the plan
  MF_HIP(hipGetLastError());
  return H > 0 && item_rows > 0 ? H : 0;
}

}  // namespace mfhip

// ---------------------------------------------------------------------------------------------
// The deterministic sweep's superstep input on the device (kernels.hpp det_device_build): the host
// build of plan.cpp build_det_step as a gather, two stable radix sorts and a scatter.  The host
// keeps only the JVM shuffle (sequential per block) and uploads the permutation (4 B per rating
// instead of the 20-B entries), and the ~15 ms of host gather / prefix / scatter per NFLX
// superstep become ~1 ms of kernels on the copy stream beside the previous superstep's sweep.
namespace mfhip {
namespace {

__global__ void k_db_gather(const int32_t* __restrict__ ord, int64_t n, const DetBuildBlock* __restrict__ blocks,
                            int nblk, const DetEntry* __restrict__ aos, const int32_t* __restrict__ iw,
                            DetEntry* __restrict__ ent, uint32_t* __restrict__ wkey, uint32_t* __restrict__ ukey,
                            int32_t* __restrict__ iota) {
  for (int64_t j = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; j < n;
       j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int x = 0;
    while (x + 1 < nblk && blocks[x + 1].e0 <= j) ++x;  // a superstep holds c blocks (a handful)
    const DetBuildBlock b = blocks[x];
    const DetEntry d = aos[b.st + ord[j]];
    ent[j] = d;
    wkey[j] = b.w0 + static_cast<uint32_t>(iw[b.iwoff + (d.i - b.i0)]);
    ukey[j] = d.u;
    iota[j] = static_cast<int32_t>(j);
  }
}

// entry p of the wave-major order: rating j = wx[p] (a wave's ratings in shuffle order)
__global__ void k_db_scatter(const int32_t* __restrict__ wx, int64_t n, const DetEntry* __restrict__ ent,
                             const uint32_t* __restrict__ ticket, uint32_t* __restrict__ ou, uint32_t* __restrict__ oi,
                             uint32_t* __restrict__ oq, double* __restrict__ orr) {
  for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < n;
       p += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t j = wx[p];
    const DetEntry d = ent[j];
    ou[p] = d.u;
    oi[p] = d.i;
    oq[p] = ticket[j];
    orr[p] = d.r;
  }
}

}  // namespace

void det_device_build_reserve(DetBuildScratch& sc, int64_t n_max, uint32_t wave_bound, uint32_t user_rows) {
  MF_REQUIRE(n_max >= 0 && n_max < (int64_t{1} << 31), "det device build: superstep too large");
  const int64_t n = std::max<int64_t>(n_max, 1);
  const int N = static_cast<int>(n);
  sc.ent.alloc(n * sizeof(DetEntry));
  for (DevBuf* b : {&sc.wkey, &sc.wkey2, &sc.ukey, &sc.ukey2, &sc.iota, &sc.wx, &sc.ux, &sc.head, &sc.start, &sc.ticket})
    b->alloc(n * 4);
  size_t a = 0, b2 = 0, c = 0;
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, a, sc.wkey.as<uint32_t>(), sc.wkey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.wx.as<int32_t>(), N, 0, bits_for(wave_bound)));
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, b2, sc.ukey.as<uint32_t>(), sc.ukey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.ux.as<int32_t>(), N, 0, bits_for(user_rows)));
  MF_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, c, sc.head.as<int32_t>(), sc.start.as<int32_t>(), hipcub::Max(), N));
  sc.tmp_bytes = std::max<size_t>(std::max(a, b2), 256);
  sc.tmp2_bytes = std::max<size_t>(c, 256);
  sc.tmp.alloc(sc.tmp_bytes);
  sc.tmp2.alloc(sc.tmp2_bytes);
  sc.n_max = n_max;
}

void det_device_build(hipStream_t st, DetBuildScratch& sc, const int32_t* ord, int64_t n, const DetBuildBlock* blocks,
                      int nblk, const DetEntry* aos, const int32_t* item_wave, uint32_t wave_bound,
                      uint32_t user_rows, uint32_t* ou, uint32_t* oi, uint32_t* oq, double* orr) {
  if (n <= 0) return;
  MF_REQUIRE(n <= sc.n_max, "det device build: more ratings than the scratch was reserved for");
  const int N = static_cast<int>(n);
  hipLaunchKernelGGL(k_db_gather, dim3(grid_for(n)), dim3(kThreads), 0, st, ord, n, blocks, nblk, aos, item_wave,
                     sc.ent.as<DetEntry>(), sc.wkey.as<uint32_t>(), sc.ukey.as<uint32_t>(), sc.iota.as<int32_t>());
  size_t tb = 0;
  // wave-major order, a wave's ratings in shuffle order (stable)
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, tb, sc.wkey.as<uint32_t>(), sc.wkey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.wx.as<int32_t>(), N, 0, bits_for(wave_bound), st));
  MF_REQUIRE(tb <= sc.tmp_bytes, "det device build: sort scratch");
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(sc.tmp.get(), tb, sc.wkey.as<uint32_t>(), sc.wkey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.wx.as<int32_t>(), N, 0, bits_for(wave_bound), st));
  // useq: the rank of a rating among its user's ratings in shuffle order (users of a superstep's
  // blocks are disjoint: each block has its own user block)
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(nullptr, tb, sc.ukey.as<uint32_t>(), sc.ukey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.ux.as<int32_t>(), N, 0, bits_for(user_rows), st));
  MF_REQUIRE(tb <= sc.tmp_bytes, "det device build: sort scratch");
  MF_HIP(rocprim::radix_sort_pairs<SortCfg>(sc.tmp.get(), tb, sc.ukey.as<uint32_t>(), sc.ukey2.as<uint32_t>(),
                                             sc.iota.as<int32_t>(), sc.ux.as<int32_t>(), N, 0, bits_for(user_rows), st));
  hipLaunchKernelGGL(k_run_heads, dim3(grid_for(n)), dim3(kThreads), 0, st, sc.ukey2.as<uint32_t>(), n,
                     sc.head.as<int32_t>());
  tb = 0;
  MF_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, sc.head.as<int32_t>(), sc.start.as<int32_t>(), hipcub::Max(),
                                           N, st));
  MF_REQUIRE(tb <= sc.tmp2_bytes, "det device build: scan scratch");
  MF_HIP(hipcub::DeviceScan::InclusiveScan(sc.tmp2.get(), tb, sc.head.as<int32_t>(), sc.start.as<int32_t>(),
                                           hipcub::Max(), N, st));
  hipLaunchKernelGGL(k_tickets, dim3(grid_for(n)), dim3(kThreads), 0, st, sc.ux.as<int32_t>(), sc.start.as<int32_t>(), n,
                     sc.ticket.as<uint32_t>());
  hipLaunchKernelGGL(k_db_scatter, dim3(grid_for(n)), dim3(kThreads), 0, st, sc.wx.as<int32_t>(), n,
                     sc.ent.as<DetEntry>(), sc.ticket.as<uint32_t>(), ou, oi, oq, orr);
  MF_HIP(hipGetLastError());
}

}  // namespace mfhip
