// kernels_block.hip -- DSGD blocking on the GPU: initFactorBlockAndIndices
// (DSGDforMF.scala:513-588) and the rating blocks (:301-327), as device radix sorts, scans and
// scatters.  Bitwise the host build_side / build_rating_blocks (plan.cpp) for the reference's
// seeded blocking; tests/test_gpu_dsgd.py compares the two.
//
// Per side (users, items), n rating ids:
//   1. stable sort (id, rating index)                         -> ids in ascending order
//   2. run heads -> distinct ids (ascending, :520), counts = omega (:537-541)
//   3. block of each distinct id: new Random(id ^ seed).nextInt(n) (:531-533), JDK LCG
//   4. stable sort of the distinct ids by block               -> rows grouped by block, ids
//      ascending inside a block (:556), the reference's FactorBlock order
//   5. row of every rating (scatter through both permutations)
// Rating blocks: key ub*n + ib (toRatingBlockId, :597-601) per rating; stable sort by key, after a
// stable sort by (user id, item id) when seeded (:319-323; ties keep the input order).  Ratings of
// user blocks outside [ub_lo, ub_hi) (other ranks) get key n*n and are dropped.
// All of it is HBM-bound integer work (sorts of 4-8-byte keys with 4-byte payloads).
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace mfhip {
namespace {

constexpr int kThreads = 256;
unsigned grid_for(int64_t n) { return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, 1 << 20))); }

__global__ void k_iota(int32_t* __restrict__ out, int64_t n) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    out[x] = static_cast<int32_t>(x);
}

// head[x] = 1 where a run of equal sorted ids starts
__global__ void k_heads(const int32_t* __restrict__ sorted, int64_t n, int32_t* __restrict__ head) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    head[x] = (x == 0 || sorted[x] != sorted[x - 1]) ? 1 : 0;
}

// seg = inclusive scan of heads: distinct index = seg - 1; the run start of distinct d is start[d]
__global__ void k_runs(const int32_t* __restrict__ sorted, const int32_t* __restrict__ head,
                       const int32_t* __restrict__ seg, int64_t n, int32_t* __restrict__ distinct,
                       int64_t* __restrict__ start) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    if (head[x]) {
      distinct[seg[x] - 1] = sorted[x];
      start[seg[x] - 1] = x;
    }
}

// java.util.Random(id ^ seed).nextInt(nb) (JDK 8): scrambled seed, next(31), power-of-two path
// or the int32 rejection loop -- as JavaRandom::nextInt (jvm_random.hpp)
__global__ void k_jvm_block(const int32_t* __restrict__ distinct, int64_t d, int64_t seed, int32_t nb,
                            int32_t* __restrict__ blk, int32_t* __restrict__ iota) {
  constexpr uint64_t kMult = 0x5DEECE66DULL, kMask = (1ULL << 48) - 1;
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < d;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint64_t s = (static_cast<uint64_t>(static_cast<int64_t>(distinct[x]) ^ seed) ^ kMult) & kMask;
    auto next31 = [&]() {
      s = (s * kMult + 0xBULL) & kMask;
      return static_cast<int32_t>(static_cast<uint32_t>(s >> 17));
    };
    int32_t r = next31();
    const int32_t m = nb - 1;
    if ((nb & m) == 0) {
      r = static_cast<int32_t>((static_cast<int64_t>(nb) * r) >> 31);
    } else {
      for (int32_t u = r;; u = next31()) {
        r = u % nb;
        if (static_cast<int32_t>(static_cast<uint32_t>(u) - static_cast<uint32_t>(r) + static_cast<uint32_t>(m)) >= 0)
          break;
      }
    }
    blk[x] = r;
    iota[x] = static_cast<int32_t>(x);
  }
}

// order = distinct indices sorted by block (stable): row y holds distinct order[y]
__global__ void k_rows(const int32_t* __restrict__ order, int64_t d, int32_t* __restrict__ row_of) {
  for (int64_t y = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; y < d;
       y += static_cast<int64_t>(gridDim.x) * blockDim.x)
    row_of[order[y]] = static_cast<int32_t>(y);
}

// rating perm[x] (sorted position x, distinct seg[x]-1) -> its row
__global__ void k_rating_rows(const int32_t* __restrict__ perm, const int32_t* __restrict__ seg,
                              const int32_t* __restrict__ row_of, int64_t n, uint32_t* __restrict__ rows) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    rows[perm[x]] = static_cast<uint32_t>(row_of[seg[x] - 1]);
}

// per rating: the rating block key (n*n = not on this rank) and, when sorting, the (u, i) key
__global__ void k_block_keys(const uint32_t* __restrict__ urow, const uint32_t* __restrict__ irow,
                             const int32_t* __restrict__ ublk_of_row, const int32_t* __restrict__ iblk_of_row,
                             const int32_t* __restrict__ u, const int32_t* __restrict__ i, int64_t n, int32_t nb,
                             int32_t ub_lo, int32_t ub_hi, uint32_t* __restrict__ bkey, uint64_t* __restrict__ uikey) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int32_t ub = ublk_of_row[urow[x]];
    bkey[x] = (ub < ub_lo || ub >= ub_hi) ? static_cast<uint32_t>(nb) * nb
                                          : static_cast<uint32_t>(ub) * nb + static_cast<uint32_t>(iblk_of_row[irow[x]]);
    if (uikey)
      uikey[x] = (static_cast<uint64_t>(static_cast<uint32_t>(u[x]) ^ 0x80000000u) << 32) |
                 (static_cast<uint32_t>(i[x]) ^ 0x80000000u);
  }
}

__global__ void k_gather_u32(const int32_t* __restrict__ perm, const uint32_t* __restrict__ src, int64_t n,
                             uint32_t* __restrict__ dst) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[x] = src[perm[x]];
}
__global__ void k_gather_f64(const int32_t* __restrict__ perm, const double* __restrict__ src, int64_t n,
                             double* __restrict__ dst) {
  for (int64_t x = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; x < n;
       x += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[x] = src[perm[x]];
}

// start[b] = lower_bound(keys, b) over the sorted rating-block keys, b = 0..nb2 (one thread each)
__global__ void k_block_starts(const uint32_t* __restrict__ keys, int64_t n, int64_t nb2, int64_t* __restrict__ start) {
  const int64_t b = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (b > nb2) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (keys[mid] < static_cast<uint32_t>(b)) lo = mid + 1;
    else hi = mid;
  }
  start[b] = lo;
}

int bits_for(uint64_t maxval) {
  int b = 1;
  while (b < 64 && (maxval >> b) != 0) ++b;
  return b;
}

// hipcub temp storage, grown on demand
struct Temp {
  DevBuf buf;
  void* get(size_t bytes) {
    buf.alloc(std::max<size_t>(bytes, 256));
    return buf.get();
  }
};

// One side: rows of every rating (device) and the host SideLayout.
void block_side(hipStream_t st, Temp& tmp, const int32_t* d_ids, int64_t n, int32_t nb, int64_t seed, SideLayout& S,
                DevBuf& d_rows, DevBuf& d_blk_of_row) {
  S = SideLayout();
  S.n_blocks = nb;
  S.block_start.assign(nb + 1, 0);
  d_rows.alloc(std::max<int64_t>(n, 1) * 4);
  if (n == 0) {
    d_blk_of_row.alloc(4);
    return;
  }
  DevBuf keys_out, idx_in, perm, head, seg, distinct, start;
  keys_out.alloc(n * 4);
  idx_in.alloc(n * 4);
  perm.alloc(n * 4);
  head.alloc(n * 4);
  seg.alloc(n * 4);
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kThreads), 0, st, idx_in.as<int32_t>(), n);
  size_t tb = 0;
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_ids, keys_out.as<int32_t>(), idx_in.as<int32_t>(),
                                            perm.as<int32_t>(), static_cast<int>(n), 0, 32, st));
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, d_ids, keys_out.as<int32_t>(), idx_in.as<int32_t>(),
                                            perm.as<int32_t>(), static_cast<int>(n), 0, 32, st));
  hipLaunchKernelGGL(k_heads, dim3(grid_for(n)), dim3(kThreads), 0, st, keys_out.as<int32_t>(), n, head.as<int32_t>());
  MF_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, head.as<int32_t>(), seg.as<int32_t>(), static_cast<int>(n), st));
  MF_HIP(hipcub::DeviceScan::InclusiveSum(tmp.get(tb), tb, head.as<int32_t>(), seg.as<int32_t>(), static_cast<int>(n), st));
  int32_t dcount = 0;
  MF_HIP(hipMemcpyAsync(&dcount, seg.as<int32_t>() + n - 1, 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  const int64_t d = dcount;
  distinct.alloc(d * 4);
  start.alloc((d + 1) * 8);
  hipLaunchKernelGGL(k_runs, dim3(grid_for(n)), dim3(kThreads), 0, st, keys_out.as<int32_t>(), head.as<int32_t>(),
                     seg.as<int32_t>(), n, distinct.as<int32_t>(), start.as<int64_t>());
  DevBuf blk, blk_sorted, iota, order, row_of;
  blk.alloc(d * 4);
  blk_sorted.alloc(d * 4);
  iota.alloc(d * 4);
  order.alloc(d * 4);
  row_of.alloc(d * 4);
  hipLaunchKernelGGL(k_jvm_block, dim3(grid_for(d)), dim3(kThreads), 0, st, distinct.as<int32_t>(), d, seed, nb,
                     blk.as<int32_t>(), iota.as<int32_t>());
  const int bb = bits_for(static_cast<uint64_t>(nb));
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, blk.as<int32_t>(), blk_sorted.as<int32_t>(), iota.as<int32_t>(),
                                            order.as<int32_t>(), static_cast<int>(d), 0, bb, st));
  MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, blk.as<int32_t>(), blk_sorted.as<int32_t>(),
                                            iota.as<int32_t>(), order.as<int32_t>(), static_cast<int>(d), 0, bb, st));
  hipLaunchKernelGGL(k_rows, dim3(grid_for(d)), dim3(kThreads), 0, st, order.as<int32_t>(), d, row_of.as<int32_t>());
  hipLaunchKernelGGL(k_rating_rows, dim3(grid_for(n)), dim3(kThreads), 0, st, perm.as<int32_t>(), seg.as<int32_t>(),
                     row_of.as<int32_t>(), n, d_rows.as<uint32_t>());
  // host side of the layout: row y = distinct order[y]
  std::vector<int32_t> h_distinct(d), h_order(d), h_blk_sorted(d);
  std::vector<int64_t> h_start(d + 1);
  MF_HIP(hipMemcpyAsync(h_distinct.data(), distinct.get(), d * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipMemcpyAsync(h_order.data(), order.get(), d * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipMemcpyAsync(h_blk_sorted.data(), blk_sorted.get(), d * 4, hipMemcpyDeviceToHost, st));
  MF_HIP(hipMemcpyAsync(h_start.data(), start.get(), d * 8, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  h_start[d] = n;
  d_blk_of_row = std::move(blk_sorted);  // row y's block = blk_sorted[y]
  S.row_id.resize(d);
  S.omega.resize(d);
  S.row_block.resize(d);
  S.index.reserve(d);
  for (int64_t y = 0; y < d; ++y) {
    const int32_t x = h_order[y];
    S.row_id[y] = h_distinct[x];
    S.omega[y] = static_cast<int32_t>(h_start[x + 1] - h_start[x]);
    S.row_block[y] = h_blk_sorted[y];
    S.block_start[h_blk_sorted[y] + 1]++;
    S.index.insert(h_distinct[x], static_cast<int32_t>(y));
  }
  for (int32_t b = 0; b < nb; ++b) S.block_start[b + 1] += S.block_start[b];
}

}  // namespace

void device_blocking(hipStream_t st, const int32_t* u, const int32_t* i, const double* r, int64_t n, int32_t nb,
                     int64_t seed, int32_t ub_lo, int32_t ub_hi, bool sort_ui, SideLayout& U, SideLayout& I,
                     RatingBlocks& rb, DevRatingBlocks* keep, bool host_arrays) {
  MF_REQUIRE(n < (int64_t{1} << 31), "device blocking sorts with 32-bit indices (< 2^31 ratings)");
  const int64_t nb2 = static_cast<int64_t>(nb) * nb;
  Temp tmp;
  DevBuf du, di, dr;
  du.alloc(std::max<int64_t>(n, 1) * 4);
  di.alloc(std::max<int64_t>(n, 1) * 4);
  dr.alloc(std::max<int64_t>(n, 1) * 8);
  if (n > 0) {
    MF_HIP(hipMemcpyAsync(du.get(), u, n * 4, hipMemcpyHostToDevice, st));
    MF_HIP(hipMemcpyAsync(di.get(), i, n * 4, hipMemcpyHostToDevice, st));
    MF_HIP(hipMemcpyAsync(dr.get(), r, n * 8, hipMemcpyHostToDevice, st));
  }
  DevBuf urow, irow, ublk, iblk;
  block_side(st, tmp, du.as<int32_t>(), n, nb, seed, U, urow, ublk);
  block_side(st, tmp, di.as<int32_t>(), n, nb, seed, I, irow, iblk);
  rb = RatingBlocks();
  rb.n_blocks = nb;
  rb.start.assign(nb2 + 1, 0);
  if (n == 0) return;
  // rating block keys, then stable sorts: (u, i) first when seeded, then the block key
  DevBuf bkey, bkey2, uikey, uikey2, idx, perm;
  bkey.alloc(n * 4);
  bkey2.alloc(n * 4);
  idx.alloc(n * 4);
  perm.alloc(n * 4);
  if (sort_ui) {
    uikey.alloc(n * 8);
    uikey2.alloc(n * 8);
  }
  hipLaunchKernelGGL(k_block_keys, dim3(grid_for(n)), dim3(kThreads), 0, st, urow.as<uint32_t>(), irow.as<uint32_t>(),
                     ublk.as<int32_t>(), iblk.as<int32_t>(), du.as<int32_t>(), di.as<int32_t>(), n, nb, ub_lo, ub_hi,
                     bkey.as<uint32_t>(), sort_ui ? uikey.as<uint64_t>() : nullptr);
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kThreads), 0, st, idx.as<int32_t>(), n);
  size_t tb = 0;
  const int kb = bits_for(static_cast<uint64_t>(nb2));
  if (sort_ui) {
    DevBuf p1;
    p1.alloc(n * 4);
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, uikey.as<uint64_t>(), uikey2.as<uint64_t>(), idx.as<int32_t>(),
                                              p1.as<int32_t>(), static_cast<int>(n), 0, 64, st));
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, uikey.as<uint64_t>(), uikey2.as<uint64_t>(),
                                              idx.as<int32_t>(), p1.as<int32_t>(), static_cast<int>(n), 0, 64, st));
    hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n)), dim3(kThreads), 0, st, p1.as<int32_t>(), bkey.as<uint32_t>(), n,
                       bkey2.as<uint32_t>());
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, bkey2.as<uint32_t>(), bkey.as<uint32_t>(), p1.as<int32_t>(),
                                              perm.as<int32_t>(), static_cast<int>(n), 0, kb, st));
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, bkey2.as<uint32_t>(), bkey.as<uint32_t>(),
                                              p1.as<int32_t>(), perm.as<int32_t>(), static_cast<int>(n), 0, kb, st));
  } else {
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, bkey.as<uint32_t>(), bkey2.as<uint32_t>(), idx.as<int32_t>(),
                                              perm.as<int32_t>(), static_cast<int>(n), 0, kb, st));
    MF_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(tb), tb, bkey.as<uint32_t>(), bkey2.as<uint32_t>(),
                                              idx.as<int32_t>(), perm.as<int32_t>(), static_cast<int>(n), 0, kb, st));
  }
  // the sorted keys are in bkey (sort_ui) or bkey2: block starts from their histogram
  const uint32_t* sorted_keys = sort_ui ? bkey.as<uint32_t>() : bkey2.as<uint32_t>();
  DevBuf gu, gi, gr;
  gu.alloc(n * 4);
  gi.alloc(n * 4);
  gr.alloc(n * 8);
  hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n)), dim3(kThreads), 0, st, perm.as<int32_t>(), urow.as<uint32_t>(), n,
                     gu.as<uint32_t>());
  hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n)), dim3(kThreads), 0, st, perm.as<int32_t>(), irow.as<uint32_t>(), n,
                     gi.as<uint32_t>());
  hipLaunchKernelGGL(k_gather_f64, dim3(grid_for(n)), dim3(kThreads), 0, st, perm.as<int32_t>(), dr.as<double>(), n,
                     gr.as<double>());
  MF_HIP(hipGetLastError());
  // keys are sorted: block b spans [lower_bound(b), lower_bound(b+1)); n*n (other ranks) last
  DevBuf dstart;
  dstart.alloc(static_cast<size_t>(nb2 + 1) * 8);
  hipLaunchKernelGGL(k_block_starts, dim3(static_cast<unsigned>((nb2 + 1 + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                     sorted_keys, n, nb2, dstart.as<int64_t>());
  MF_HIP(hipGetLastError());
  MF_HIP(hipMemcpyAsync(rb.start.data(), dstart.get(), static_cast<size_t>(nb2 + 1) * 8, hipMemcpyDeviceToHost, st));
  MF_HIP(hipStreamSynchronize(st));
  const int64_t total = rb.start[nb2];
  if (!keep) host_arrays = true;
  if (host_arrays) {
    resize_huge(rb.urow, total);
    resize_huge(rb.irow, total);
    resize_huge(rb.r, total);
  }
  if (total > 0 && host_arrays) {
    MF_HIP(hipMemcpyAsync(rb.urow.data(), gu.get(), total * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(rb.irow.data(), gi.get(), total * 4, hipMemcpyDeviceToHost, st));
    MF_HIP(hipMemcpyAsync(rb.r.data(), gr.get(), total * 8, hipMemcpyDeviceToHost, st));
  }
  MF_HIP(hipStreamSynchronize(st));
  if (keep) {
    keep->urow = std::move(gu);
    keep->irow = std::move(gi);
    keep->r = std::move(gr);
    keep->total = total;
  }
}

}  // namespace mfhip
