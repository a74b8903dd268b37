// kernels_det.hip -- bit-exact f64 kernels.  Compiled with -ffp-contract=off: every a*b+c
// stays two rounded operations, as on the JVM.
//
//  k_level    one dependency level of a replayed sequential order (DSGDforMF.scala:395-414
//             or SGDUpdater.nextFactors, core/FactorUpdater.scala:37-45).  One wave per
//             rating; a level never holds two ratings that share a row, so the updates of a
//             level commute and the level-by-level replay equals the sequential loop.
//  k_predict  predictRating / RMSE / empiricalRisk gathers (MatrixFactorization.scala:133-274).
//
// Roofline: both are HBM/L2 row gathers (B_f64(k) = 32k+24 bytes per update); the dot
// product is summed left to right (netlib F2jBLAS.ddot order) with v_readlane broadcasts,
// a k-long dependent f64 add chain per wave, so the deterministic path is latency-bound by
// design; the fast path (kernels_fast.hip) is the throughput path.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.hpp"

namespace mfhip {
namespace {

__device__ __forceinline__ double readlane(double v, int l) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffffu), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b >> 32), l));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
__device__ __forceinline__ float readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Sequential dot over f = 0..k-1 where lane l holds element l + 64c in prod[c]:
// acc = ((0 + x0) + x1) + ... exactly as F2jBLAS.ddot / Scala's foldLeft sum.
template <typename T, int KPL>
__device__ __forceinline__ T seq_dot(const T (&prod)[KPL], int k) {
  T acc = T(0);
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    if (64 * (c + 1) <= k) {
      // a full chunk: constant lane indices, no loop (the adds are one dependent chain; the
      // readlanes run ahead of it)
#pragma unroll
      for (int l = 0; l < 64; ++l) acc = acc + readlane(prod[c], l);
    } else {
      const int lim = min(64, k - 64 * c);
      for (int l = 0; l < lim; ++l) acc = acc + readlane(prod[c], l);
    }
  }
  return acc;
}

#include "online_f32.hpp"
#include "seq_fold.hpp"
#include "ticket_wait.hpp"

// SGDUpdater.nextFactors of one rating in f32 with online_f32.hpp's arithmetic and k_online_f32's
// row layout (kernels_online_sweep.hip), so the level replay equals the one-launch sweep bit for
// bit (k <= 256).  pv / qv: the rows before the update; returns le = lr * e.
template <int KPL>
__device__ __forceinline__ float f32_online_rows(const float* p, const float* q, int k, int lane, float (&pv)[KPL],
                                                 float (&qv)[KPL], int (&fi)[KPL], bool (&ok)[KPL], double r,
                                                 float eta) {
  const int nc = (k + 63) >> 6;  // the sweep's KPL
  const bool full = k == 64 * nc && nc != 3;
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    fi[c] = full ? lane * nc + c : lane + 64 * c;
    ok[c] = c < nc && fi[c] < k;
    pv[c] = ok[c] ? p[fi[c]] : 0.f;
    qv[c] = ok[c] ? q[fi[c]] : 0.f;
  }
  float part = pv[0] * qv[0];
#pragma unroll
  for (int c = 1; c < KPL; ++c)
    if (c < nc) part = __builtin_fmaf(pv[c], qv[c], part);
  return f32_err(r, f32_wave_sum(part), eta);
}

template <typename T, int KPL, int ARITH>
__global__ __launch_bounds__(256) void k_level(const DetEntry* __restrict__ ent, int64_t n,
                                               T* __restrict__ U, T* __restrict__ I,
                                               const T* __restrict__ regU, const T* __restrict__ regI,
                                               int k, T eta) {
  const int lane = threadIdx.x & 63;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (j >= n) return;
  const uint32_t ur = ent[j].u, ir = ent[j].i;
  const T r = static_cast<T>(ent[j].r);
  T* p = U + static_cast<size_t>(ur) * k;
  T* q = I + static_cast<size_t>(ir) * k;
  if constexpr (sizeof(T) == 4 && ARITH == static_cast<int>(Arith::kSgdNext) && KPL <= 4) {
    // f32 online: online_f32.hpp, as k_online_f32
    float pv[KPL], qv[KPL];
    int fi[KPL];
    bool ok[KPL];
    const float le = f32_online_rows<KPL>(p, q, k, lane, pv, qv, fi, ok, ent[j].r, eta);
#pragma unroll
    for (int c = 0; c < KPL; ++c)
      if (ok[c]) {
        p[fi[c]] = __builtin_fmaf(le, qv[c], pv[c]);
        q[fi[c]] = __builtin_fmaf(le, pv[c], qv[c]);
      }
    return;
  }
  T pv[KPL], qv[KPL], pr[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const int f = lane + 64 * c;
    pv[c] = f < k ? p[f] : T(0);
    qv[c] = f < k ? q[f] : T(0);
    pr[c] = pv[c] * qv[c];
  }
  const T e = r - seq_dot<T, KPL>(pr, k);
  if constexpr (ARITH == static_cast<int>(Arith::kDsgd)) {
    const T ru = regU[ur], ri = regI[ir];  // lambda / omega, as `lambda / omegai * p` (:408)
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane + 64 * c;
      if (f < k) {
        p[f] = pv[c] - eta * (ru * pv[c] - e * qv[c]);
        q[f] = qv[c] - eta * (ri * qv[c] - e * pv[c]);
      }
    }
  } else {
    const T le = eta * e;  // learningRate * e * i == (learningRate * e) * i
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane + 64 * c;
      if (f < k) {
        p[f] = pv[c] + le * qv[c];
        q[f] = qv[c] + le * pv[c];
      }
    }
  }
}

// Online micro-batch in ONE launch (SGDUpdater.nextFactors, core/FactorUpdater.scala:37-45, in
// sequence order): wave w applies, in order, every update of the items it owns, so an item's
// updates follow program order; an update waits for the earlier updates of its user (other waves)
// through a per-user ticket -- the count of that user's updates done in this batch -- and runs
// when it equals its useq.  The unfinished update earliest in the sequence is always runnable,
// so with every wave resident the launch cannot deadlock.  Hand-off as in kernels_detsweep.hip
// (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms row 1): rows are loaded and
// stored with agent-scope relaxed atomics (sc1), the wave drains its stores, then lane 0 stores
// the ticket.  The per-update arithmetic is k_level's (kSgdNext), so the factors are bitwise the
// level-by-level replay (tests/test_gpu_online.py).  A wait over ~1 s sets err and the wave leaves.
template <typename T, int KPL, bool FULL>
__global__ __launch_bounds__(64) void k_online_sweep(const int64_t* __restrict__ wbeg, const DetEntry* __restrict__ ent,
                                                     const uint32_t* __restrict__ useq, T* U, T* I, int k, T eta,
                                                     int32_t* ticket, int32_t* err) {
  const int lane = threadIdx.x;
  // this wave's updates as 32-bit offsets from its first one (uniform, so the loop's tests are
  // scalar 32-bit compares; gfx9 has no scalar 64-bit less-than)
  const int64_t jb = wbeg[blockIdx.x];
  const int32_t j1 = static_cast<int32_t>(wbeg[blockIdx.x + 1] - jb);
  if (j1 <= 0) return;
  ent += jb;
  useq += jb;
  __shared__ __attribute__((aligned(16))) T lds[64 * KPL];
  auto ld = [&](const T* row, int c) {
    const int f = lane + 64 * c;
    return FULL || f < k ? __hip_atomic_load(row + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : T(0);
  };
  // loads ahead: every lane issues one load per c (clamped address), so the vmcnt count of a row
  // loaded ahead is exactly KPL; lanes past k are zeroed where the row is used (not here, which
  // would wait for the load at once)
  auto ld_row = [&](const T* row, T (&v)[KPL]) {
#pragma unroll
    for (int c = 0; c < KPL; ++c)
      v[c] = __hip_atomic_load(row + min(lane + 64 * c, k - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // The item row stays in registers while consecutive updates of this wave share the item (a hot
  // item's chain).  User rows are loaded ahead into two slots: update j's row sits in slot
  // j & 1, loaded during update j - 2 when its ticket was already due (or during j - 1, or
  // else by j itself after waiting).  The loads ahead are issued after the update's stores, so the
  // drain before the ticket store waits for the stores only (vmcnt = the loads issued after them).
  // With every lane in use (k == 64 * KPL, so every store instruction really issues) the ticket
  // store is also deferred by one update: update j's ticket goes out during update j + 1, after
  // a vmcnt that counts only j + 1's own stores and loads, so j's store drain overlaps j + 1's
  // dot.  A wave never waits for a ticket while holding one back (it publishes first), so the
  // earliest unfinished update stays runnable and the launch cannot deadlock.
  constexpr bool defer = FULL;  // FULL: k == 64 * KPL (the host picks the instance)
  uint32_t pend_u = 0;
  int32_t pend_q = 0;
  bool has_pend = false;
  T qv[KPL], sa[KPL], sb[KPL];
  bool ha = false, hb = false;
  bool have_q = false;
  uint32_t cur_i = 0;
  auto step = [&](int32_t j, T (&slot)[KPL], bool& have, T (&oslot)[KPL], bool& ohave) {
    const uint32_t ur = ent[j].u, ir = ent[j].i;
    const int32_t q = static_cast<int32_t>(useq[j]);
    const T r = static_cast<T>(ent[j].r);
    T* p = U + static_cast<size_t>(ur) * k;
    T pv[KPL], pr[KPL];
    if (have) {
#pragma unroll
      for (int c = 0; c < KPL; ++c) pv[c] = FULL || lane + 64 * c < k ? slot[c] : T(0);
    } else {
      if (has_pend) {  // publish the held-back ticket before any wait
        __builtin_amdgcn_s_waitcnt(0x0F70);
        if (lane == 0) __hip_atomic_store(ticket + pend_u, pend_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        has_pend = false;
      }
      if (q != 0) wait_ticket_or_fail(ticket + ur, q, err, lane);  // no early return (ticket_wait.hpp)
#pragma unroll
      for (int c = 0; c < KPL; ++c) pv[c] = ld(p, c);
    }
    if (!have_q || ir != cur_i) {
      const T* qi = I + static_cast<size_t>(ir) * k;
#pragma unroll
      for (int c = 0; c < KPL; ++c) qv[c] = ld(qi, c);
      cur_i = ir;
      have_q = true;
    }
    // tickets of update j + 1 (unless its row is loaded already) and j + 2, read here and looked
    // at after the dot (their round trip overlaps it).  A row is loaded ahead only when its
    // ticket is due, i.e. every earlier update of that user is done (so never this update's user
    // nor update j + 1's, whose updates are still to come)
    const bool n1 = j + 1 < j1 && !ohave, n2 = j + 2 < j1;
    const uint32_t u1 = n1 ? ent[j + 1].u : 0u, u2 = n2 ? ent[j + 2].u : 0u;
    const int32_t q1 = n1 ? static_cast<int32_t>(useq[j + 1]) : 0, q2 = n2 ? static_cast<int32_t>(useq[j + 2]) : 0;
    // (both reads unconditional, so the compiler's wait before the dot can leave them in flight)
    const int32_t t1 = __hip_atomic_load(ticket + (n1 ? u1 : ur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int32_t t2 = __hip_atomic_load(ticket + (n2 ? u2 : ur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int c = 0; c < KPL; ++c) pr[c] = pv[c] * qv[c];
    T dot;
    if constexpr (FULL) dot = seq_fold_dpp<T, KPL>(pr);  // registers + DPP, no LDS round trip
    else dot = seq_fold<T, KPL>(pr, k, lds, lane);
    const T e = r - dot;
    // the tickets are looked at before the stores (so no wait for them lands behind the stores)
    const bool g1 = n1 && u1 != ur && (q1 == 0 || __builtin_amdgcn_readfirstlane(t1) == q1);
    const bool g2 = n2 && u2 != ur && (q2 == 0 || __builtin_amdgcn_readfirstlane(t2) == q2);
    const T le = eta * e;  // learningRate * e * i == (learningRate * e) * i
    T qnew[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane + 64 * c;
      qnew[c] = qv[c] + le * pv[c];
      if (FULL || f < k) __hip_atomic_store(p + f, pv[c] + le * qv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int c = 0; c < KPL; ++c) qv[c] = qnew[c];
    // the item row is written back when the wave's next update is on another item (or at the end)
    const bool istore = j + 1 == j1 || ent[j + 1].i != ir;
    if (istore) {
      T* qi = I + static_cast<size_t>(ir) * k;
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        const int f = lane + 64 * c;
        if (FULL || f < k) __hip_atomic_store(qi + f, qv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      have_q = false;
    }
    // the loads ahead must issue after this update's stores (the vmcnt below counts on it)
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (g1) {
      ld_row(U + static_cast<size_t>(u1) * k, oslot);
      ohave = true;
    }
    have = g2;
    if (g2) ld_row(U + static_cast<size_t>(u2) * k, slot);
    // vmcnt(n): every operation older than the n just issued has landed (vector memory
    // operations complete in issue order)
    constexpr int kW1 = 0x0F70 | ((1 * KPL) & 15) | (((1 * KPL) >> 4) << 14);
    constexpr int kW2 = 0x0F70 | ((2 * KPL) & 15) | (((2 * KPL) >> 4) << 14);
    constexpr int kW3 = 0x0F70 | ((3 * KPL) & 15) | (((3 * KPL) >> 4) << 14);
    constexpr int kW4 = 0x0F70 | ((4 * KPL) & 15) | (((4 * KPL) >> 4) << 14);
    if (defer) {
      // n = this update's stores (its user row, its item row when written back) and the loads
      // ahead: the previous update's stores have landed, so its ticket goes out now
      const int m = (istore ? 2 : 1) + (g1 ? 1 : 0) + (g2 ? 1 : 0);
      if (m == 1) __builtin_amdgcn_s_waitcnt(kW1);
      else if (m == 2) __builtin_amdgcn_s_waitcnt(kW2);
      else if (m == 3) __builtin_amdgcn_s_waitcnt(kW3);
      else __builtin_amdgcn_s_waitcnt(kW4);
      if (has_pend && lane == 0)
        __hip_atomic_store(ticket + pend_u, pend_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pend_u = ur;
      pend_q = q + 1;
      has_pend = true;
    } else {
      // n = the loads just issued: this update's stores have landed
      if (g1 && g2) __builtin_amdgcn_s_waitcnt(kW2);
      else if (g1 || g2) __builtin_amdgcn_s_waitcnt(kW1);
      else __builtin_amdgcn_s_waitcnt(0x0F70);
      if (lane == 0) __hip_atomic_store(ticket + ur, q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // whole pairs of steps, then an odd last one: no exit test between the steps of the loop body
  // (a join there makes the compiler's wait counts conservative, ticket_wait.hpp)
  const int32_t jp = j1 & ~1;
  for (int32_t j = 0; j < jp; j += 2) {
    step(j, sa, ha, sb, hb);
    step(j + 1, sb, hb, sa, ha);
  }
  if (jp < j1) step(jp, sa, ha, sb, hb);
  if (has_pend) {
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if (lane == 0) __hip_atomic_store(ticket + pend_u, pend_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T, int KPL>
int online_capacity() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_online_sweep<T, KPL, false>, 64, 0) != hipSuccess)
    return 0;
  int per_cu_full = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_full, k_online_sweep<T, KPL, true>, 64, 0) != hipSuccess)
    return 0;
  per_cu = std::min(per_cu, per_cu_full);
  return cus * per_cu;
}

// k_level's SGDUpdater arithmetic (core/FactorUpdater.scala:37-53) plus the per-rating record
// the online operator emits, f64 row src[j] of uout / iout (either may be null):
//   OUT == 1: (user', item'), FlinkOnlineMF.ItemOperator's collect (:131-135)
//   OUT == 2: (user + deltaItem, deltaItem), deltaItem = (lr*e)*user with user BEFORE the
//             update: the PS worker's ps.output and ps.push (PSOfflineOnlineMF.scala:174-176)
template <typename T, int KPL, int OUT>
__global__ __launch_bounds__(256) void k_level_out(const DetEntry* __restrict__ ent, int64_t n, T* __restrict__ U,
                                                   T* __restrict__ I, int k, T eta, const int32_t* __restrict__ src,
                                                   double* __restrict__ uout, double* __restrict__ iout) {
  const int lane = threadIdx.x & 63;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (j >= n) return;
  const uint32_t ur = ent[j].u, ir = ent[j].i;
  const T r = static_cast<T>(ent[j].r);
  T* p = U + static_cast<size_t>(ur) * k;
  T* q = I + static_cast<size_t>(ir) * k;
  const size_t o = static_cast<size_t>(src[j]) * k;
  if constexpr (sizeof(T) == 4 && KPL <= 4) {
    // f32 online: online_f32.hpp, as k_online_f32 (the model rows bitwise the sweep's)
    float pv[KPL], qv[KPL];
    int fi[KPL];
    bool ok[KPL];
    const float le = f32_online_rows<KPL>(p, q, k, lane, pv, qv, fi, ok, ent[j].r, eta);
#pragma unroll
    for (int c = 0; c < KPL; ++c)
      if (ok[c]) {
        const float pn = __builtin_fmaf(le, qv[c], pv[c]), qn = __builtin_fmaf(le, pv[c], qv[c]);
        p[fi[c]] = pn;
        q[fi[c]] = qn;
        if constexpr (OUT == 1) {
          if (uout) uout[o + fi[c]] = static_cast<double>(pn);
          if (iout) iout[o + fi[c]] = static_cast<double>(qn);
        } else {
          const float di = le * pv[c];
          if (uout) uout[o + fi[c]] = static_cast<double>(pv[c] + di);
          if (iout) iout[o + fi[c]] = static_cast<double>(di);
        }
      }
    return;
  }
  T pv[KPL], qv[KPL], pr[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const int f = lane + 64 * c;
    pv[c] = f < k ? p[f] : T(0);
    qv[c] = f < k ? q[f] : T(0);
    pr[c] = pv[c] * qv[c];
  }
  const T e = r - seq_dot<T, KPL>(pr, k);
  const T le = eta * e;
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const int f = lane + 64 * c;
    if (f < k) {
      const T pn = pv[c] + le * qv[c], qn = qv[c] + le * pv[c];
      p[f] = pn;
      q[f] = qn;
      if constexpr (OUT == 1) {
        if (uout) uout[o + f] = static_cast<double>(pn);
        if (iout) iout[o + f] = static_cast<double>(qn);
      } else {
        const T di = le * pv[c];
        if (uout) uout[o + f] = static_cast<double>(pv[c] + di);
        if (iout) iout[o + f] = static_cast<double>(di);
      }
    }
  }
}

// predictRating gathers, one pair per LANE: every lane sums its own pair's products in order
// f = 0..k-1 (the F2jBLAS.ddot order, bit-exact in f64), so a wave runs 64 independent
// k-long add chains instead of one readlane chain per pair.  Rows are staged through LDS in
// chunks of CE = 128/sizeof(T) elements: CE consecutive lanes load one 128-B row chunk
// (coalesced), then each lane reads its own pair's chunk back from a padded LDS row.
// Bytes per pair: 2*k*sizeof(T) (HBM gather-bound).
template <typename T>
__global__ __launch_bounds__(256) void k_predict(const int32_t* __restrict__ urow,
                                                 const int32_t* __restrict__ irow, int64_t n,
                                                 const T* __restrict__ U, const T* __restrict__ I,
                                                 int k, double* __restrict__ out,
                                                 const double* __restrict__ r,
                                                 const int32_t* __restrict__ mult, double lambda,
                                                 double* __restrict__ partials) {
  constexpr int CE = 128 / sizeof(T);  // elements per row chunk
  constexpr int LPR = CE;               // lanes loading one row chunk (one element each)
  constexpr int PPI = 64 / LPR;         // pairs covered by one load instruction
  constexpr int STR = CE + 1;           // padded LDS row stride (elements): conflict-free reads
  __shared__ T su[4][64 * STR], si[4][64 * STR];
  __shared__ double red[4][3];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T* lu = su[wave];
  T* li = si[wave];
  double sse = 0.0, cnt = 0.0, risk = 0.0;
  const int64_t groups = (n + 63) / 64;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * 4 + wave; g < groups; g += static_cast<int64_t>(gridDim.x) * 4) {
    const int64_t j = g * 64 + lane;
    const int32_t ur = j < n ? urow[j] : -1, ir = j < n ? irow[j] : -1;
    const bool ok = ur >= 0 && ir >= 0;
    double pq = 0.0, pp = 0.0, qq = 0.0;
    for (int c0 = 0; c0 < k; c0 += CE) {
      // stage: pair y of the group, element e of the chunk, loaded by lane (y % PPI) * LPR + e
#pragma unroll 4
      for (int y0 = 0; y0 < 64; y0 += PPI) {
        const int y = y0 + lane / LPR, e = lane % LPR, f = c0 + e;
        const int32_t uy = __shfl(ur, y), iy = __shfl(ir, y);
        const bool v = uy >= 0 && iy >= 0 && f < k;
        lu[y * STR + e] = v ? U[static_cast<int64_t>(uy) * k + f] : T(0);
        li[y * STR + e] = v ? I[static_cast<int64_t>(iy) * k + f] : T(0);
      }
      const int lim = min(CE, k - c0);
      for (int e = 0; e < lim; ++e) {
        const double a = static_cast<double>(lu[lane * STR + e]), b = static_cast<double>(li[lane * STR + e]);
        pq = pq + a * b;
        if (mult) { pp = pp + a * a; qq = qq + b * b; }
      }
    }
    if (j < n && out) out[j] = ok ? pq : 0.0;
    if (ok && r) {
      const double d = r[j] - pq;
      sse += d * d;
      cnt += 1.0;
      if (mult) {
        const double term = d * d + lambda * (pp + qq);
        for (int m = 0; m < mult[j]; ++m) risk += term;
      }
    }
  }
  if (!partials) return;
  // fixed-order reduction: an XOR butterfly over the 64 lanes (deterministic, not a sequential
  // left fold), then the 4 waves in order
  for (int l = 1; l < 64; l <<= 1) {
    sse += __shfl_xor(sse, l);
    cnt += __shfl_xor(cnt, l);
    risk += __shfl_xor(risk, l);
  }
  if (lane == 0) { red[wave][0] = sse; red[wave][1] = cnt; red[wave][2] = risk; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const double s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
    partials[static_cast<size_t>(blockIdx.x) * 3 + threadIdx.x] = s;
  }
}

template <typename T, int ARITH>
void level_dispatch(hipStream_t st, const DetEntry* e, int64_t n, void* U, void* I, const void* rU,
                    const void* rI, int k, double eta) {
  const dim3 grid(static_cast<unsigned>((n + 3) / 4)), block(256);
  T* u = static_cast<T*>(U);
  T* i = static_cast<T*>(I);
  const T* ru = static_cast<const T*>(rU);
  const T* ri = static_cast<const T*>(rI);
  const T et = static_cast<T>(eta);
  if (k <= 64) hipLaunchKernelGGL((k_level<T, 1, ARITH>), grid, block, 0, st, e, n, u, i, ru, ri, k, et);
  else if (k <= 128) hipLaunchKernelGGL((k_level<T, 2, ARITH>), grid, block, 0, st, e, n, u, i, ru, ri, k, et);
  else if (k <= 256) hipLaunchKernelGGL((k_level<T, 4, ARITH>), grid, block, 0, st, e, n, u, i, ru, ri, k, et);
  else hipLaunchKernelGGL((k_level<T, 8, ARITH>), grid, block, 0, st, e, n, u, i, ru, ri, k, et);
}

// JVM LCG with jump-ahead (java.util.Random, JDK 8): element (x, f) needs the states after
// 2f+1 and 2f+2 steps from the scrambled seed; nextDouble = ((next(26) << 27) + next(27)) * 2^-53.
template <typename T>
__global__ __launch_bounds__(256) void k_jvm_init_rows(const int32_t* __restrict__ ids, int64_t rows, int k,
                                                       int xor_seed, int64_t seed, const uint64_t* __restrict__ jump,
                                                       T* __restrict__ out) {
  constexpr uint64_t kMult = 0x5DEECE66DULL, kMask = (1ULL << 48) - 1;
  const int64_t total = rows * k;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t x = e / k;
    const int f = static_cast<int>(e - x * k);
    const int64_t id = ids[x];
    const uint64_t s0 = (static_cast<uint64_t>(xor_seed ? (id ^ seed) : id) ^ kMult) & kMask;
    const uint64_t s1 = (jump[4 * f] * s0 + jump[4 * f + 1]) & kMask;      // after 2f+1 steps
    const uint64_t s2 = (jump[4 * f + 2] * s0 + jump[4 * f + 3]) & kMask;  // after 2f+2 steps
    const int64_t hi = static_cast<int32_t>(static_cast<uint32_t>(s1 >> 22));  // next(26)
    const int64_t lo = static_cast<int32_t>(static_cast<uint32_t>(s2 >> 21));  // next(27)
    out[e] = static_cast<T>(static_cast<double>((hi << 27) + lo) * 0x1.0p-53);
  }
}

template <typename T>
void predict_dispatch(hipStream_t st, const int32_t* ur, const int32_t* ir, int64_t n, const void* U,
                      const void* I, int k, double* out, const double* r, const int32_t* mult,
                      double lambda, double* partials, int grid_blocks) {
  const dim3 grid(static_cast<unsigned>(grid_blocks)), block(256);
  const T* u = static_cast<const T*>(U);
  const T* i = static_cast<const T*>(I);
  hipLaunchKernelGGL((k_predict<T>), grid, block, 0, st, ur, ir, n, u, i, k, out, r, mult, lambda, partials);
}

}  // namespace

void launch_level(hipStream_t st, const DetEntry* entries, int64_t n, void* U, void* I,
                  const void* regU, const void* regI, int k, double eta, Arith arith, bool f64) {
  if (n <= 0) return;
  if (f64) {
    if (arith == Arith::kDsgd) level_dispatch<double, 0>(st, entries, n, U, I, regU, regI, k, eta);
    else level_dispatch<double, 1>(st, entries, n, U, I, regU, regI, k, eta);
  } else {
    if (arith == Arith::kDsgd) level_dispatch<float, 0>(st, entries, n, U, I, regU, regI, k, eta);
    else level_dispatch<float, 1>(st, entries, n, U, I, regU, regI, k, eta);
  }
}

template <typename T, int OUT>
void level_out_dispatch(hipStream_t st, const DetEntry* e, int64_t n, void* U, void* I, int k, double eta,
                        const int32_t* src, double* uo, double* io) {
  const dim3 grid(static_cast<unsigned>((n + 3) / 4)), block(256);
  T* u = static_cast<T*>(U);
  T* i = static_cast<T*>(I);
  const T et = static_cast<T>(eta);
  if (k <= 64) hipLaunchKernelGGL((k_level_out<T, 1, OUT>), grid, block, 0, st, e, n, u, i, k, et, src, uo, io);
  else if (k <= 128) hipLaunchKernelGGL((k_level_out<T, 2, OUT>), grid, block, 0, st, e, n, u, i, k, et, src, uo, io);
  else if (k <= 256) hipLaunchKernelGGL((k_level_out<T, 4, OUT>), grid, block, 0, st, e, n, u, i, k, et, src, uo, io);
  else hipLaunchKernelGGL((k_level_out<T, 8, OUT>), grid, block, 0, st, e, n, u, i, k, et, src, uo, io);
}

int online_sweep_capacity(int k, bool f64) {
  if (f64) return k <= 64 ? online_capacity<double, 1>() : k <= 128 ? online_capacity<double, 2>()
                : k <= 256 ? online_capacity<double, 4>() : online_capacity<double, 8>();
  return k <= 64 ? online_capacity<float, 1>() : k <= 128 ? online_capacity<float, 2>()
         : k <= 256 ? online_capacity<float, 4>() : online_capacity<float, 8>();
}

void launch_online_sweep(hipStream_t st, int nw, const int64_t* wbeg, const DetEntry* ent, const uint32_t* useq,
                         void* U, void* I, int k, double eta, bool f64, int32_t* ticket, int32_t* err) {
  if (nw <= 0) return;
  const dim3 g(static_cast<unsigned>(nw)), b(64);
#define MF_OS(T, KPL)                                                                                       \
  do {                                                                                                      \
    if (k == 64 * (KPL))                                                                                    \
      hipLaunchKernelGGL((k_online_sweep<T, KPL, true>), g, b, 0, st, wbeg, ent, useq, static_cast<T*>(U),  \
                         static_cast<T*>(I), k, static_cast<T>(eta), ticket, err);                          \
    else                                                                                                    \
      hipLaunchKernelGGL((k_online_sweep<T, KPL, false>), g, b, 0, st, wbeg, ent, useq, static_cast<T*>(U), \
                         static_cast<T*>(I), k, static_cast<T>(eta), ticket, err);                          \
  } while (0)
  if (f64) {
    if (k <= 64) MF_OS(double, 1);
    else if (k <= 128) MF_OS(double, 2);
    else if (k <= 256) MF_OS(double, 4);
    else MF_OS(double, 8);
  } else {
    if (k <= 64) MF_OS(float, 1);
    else if (k <= 128) MF_OS(float, 2);
    else if (k <= 256) MF_OS(float, 4);
    else MF_OS(float, 8);
  }
#undef MF_OS
}

void launch_level_out(hipStream_t st, const DetEntry* entries, int64_t n, void* U, void* I, int k, double eta, bool f64,
                      OnlineOut mode, const int32_t* src, double* uout, double* iout) {
  if (n <= 0) return;
  const bool next = mode == OnlineOut::kOutNext;
  if (f64) {
    if (next) level_out_dispatch<double, 1>(st, entries, n, U, I, k, eta, src, uout, iout);
    else level_out_dispatch<double, 2>(st, entries, n, U, I, k, eta, src, uout, iout);
  } else {
    if (next) level_out_dispatch<float, 1>(st, entries, n, U, I, k, eta, src, uout, iout);
    else level_out_dispatch<float, 2>(st, entries, n, U, I, k, eta, src, uout, iout);
  }
}

int predict_grid(int64_t n) {
  const int64_t g = (n + 255) / 256;  // 4 waves x 64 pairs per workgroup pass
  return static_cast<int>(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

void launch_predict(hipStream_t st, const int32_t* urow, const int32_t* irow, int64_t n,
                    const void* U, const void* I, int k, bool f64, double* out, const double* r,
                    const int32_t* mult, double lambda, double* partials) {
  if (n <= 0) return;
  const int g = predict_grid(n);
  if (f64) predict_dispatch<double>(st, urow, irow, n, U, I, k, out, r, mult, lambda, partials, g);
  else predict_dispatch<float>(st, urow, irow, n, U, I, k, out, r, mult, lambda, partials, g);
}

void launch_jvm_init_rows(hipStream_t st, const int32_t* ids, int64_t rows, int k, bool xor_seed, int64_t seed,
                          const uint64_t* jump, void* out, bool f64) {
  const int64_t total = rows * k;
  if (total <= 0) return;
  const unsigned grid = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 65536));
  if (f64)
    hipLaunchKernelGGL((k_jvm_init_rows<double>), dim3(grid), dim3(256), 0, st, ids, rows, k, xor_seed ? 1 : 0, seed,
                       jump, static_cast<double*>(out));
  else
    hipLaunchKernelGGL((k_jvm_init_rows<float>), dim3(grid), dim3(256), 0, st, ids, rows, k, xor_seed ? 1 : 0, seed,
                       jump, static_cast<float*>(out));
}

}  // namespace mfhip
