// kernels_detsweep.hip -- deterministic f64 DSGD superstep as ONE persistent launch (bit-exact
// with the reference's sequential order, DSGDforMF.scala:378-418).  Compiled with
// -ffp-contract=off: every a*b+c stays two rounded operations, as on the JVM.
//
// Schedule (plan.hpp DetSweepLayout / build_det_step): each item of a rating block belongs to
// one wave, which applies all updates of its items in the block's shuffled order (:392-393).
// An update depends on the previous update of its item (same wave: program order) and of its
// user (another wave, in general); the latter is awaited through a per-user ticket, the number
// of that user's updates done so far in this superstep.  The entry carries useq = how many
// earlier updates of its user the shuffled order has, so it runs when ticket[u] == useq and then
// publishes useq + 1.  Every wave's entries are in increasing shuffle position, so the unfinished
// entry with the smallest position is always runnable: with every wave resident there is no
// deadlock (the host launches at most the co-resident wave count).  Consecutive entries of the
// same item keep the item row in registers (the hot items' long chains).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms row 1): the user rows a
// wave publishes are stored sc1 (write-through), the wave drains them (s_waitcnt vmcnt(0)), then
// lane 0 stores the ticket with an agent-scope relaxed atomic; the consumer polls the ticket with
// agent-scope relaxed loads (sc1) and loads the user row with sc1 loads only after the poll has
// matched.  Item rows are touched by one wave only and are stored / reloaded with sc1 as well
// (the wave drains its stores before its next entry).  A wait longer than ~1 s sets err[0]; every
// wave then leaves (the host reports MF_ERR_TIMEOUT and refuses the partial model).
//
// Bytes per update: B_f64(k) = 32k + 24 plus the 20-B entry and the ticket word.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mfhip {
namespace {

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ double rld(double v, int l) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffffu), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b >> 32), l));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ((0 + x0) + x1) + ... over f = 0..k-1 (F2jBLAS.ddot / Scala foldLeft order); lane l holds
// element l + 64c in prod[c].
template <int KPL>
__device__ __forceinline__ double seq_dot(const double (&prod)[KPL], int k) {
  double acc = 0.0;
  if (k == 64 * KPL) {  // fully unrolled: the readlanes issue ahead of the dependent add chain
#pragma unroll
    for (int c = 0; c < KPL; ++c)
#pragma unroll
      for (int l = 0; l < 64; ++l) acc = acc + rld(prod[c], l);
    return acc;
  }
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    const int lim = min(64, k - 64 * c);
    for (int l = 0; l < lim; ++l) acc = acc + rld(prod[c], l);
  }
  return acc;
}

template <int KPL>
__global__ __launch_bounds__(64) void k_det_sweep(const DetWave* __restrict__ waves, const uint32_t* __restrict__ eu,
                                                  const uint32_t* __restrict__ ei, const uint32_t* __restrict__ eq,
                                                  const double* __restrict__ er, double* U, double* I,
                                                  const double* __restrict__ regU, const double* __restrict__ regI,
                                                  int k, double eta, int32_t* ticket, int32_t* err) {
  const int lane = threadIdx.x;
  const DetWave d = waves[blockIdx.x];
  double q[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = 0.0;
  for (int64_t c0 = 0; c0 < d.count; c0 += 64) {
    // 64 entries, one per lane (coalesced), broadcast with readlane
    const int64_t x = d.begin + c0 + lane;
    const bool in = c0 + lane < d.count;
    const uint32_t mu = in ? eu[x] : 0u, mi = in ? ei[x] : 0u, mq = in ? eq[x] : 0u;
    const double mr = in ? er[x] : 0.0;
    const int n = static_cast<int>(min<int64_t>(64, d.count - c0));
    for (int s = 0; s < n; ++s) {
      const uint32_t u = rl(mu, s), i = rl(mi, s), qf = rl(mq, s);
      const double r = rld(mr, s);
      const int32_t useq = static_cast<int32_t>(qf & kDetUseqMask);
      int32_t* tk = ticket + u;
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != useq) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        for (;;) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == useq)
            break;
          if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0)
            return;
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // ~1 s: a producer never ran
            if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
          }
        }
      }
      double* pp = U + static_cast<size_t>(u) * k;
      double* qp = I + static_cast<size_t>(i) * k;
      double pv[KPL], pr[KPL];
      const bool keep = (qf & kDetKeepQ) != 0;
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        const int f = lane + 64 * c;
        pv[c] = f < k ? ld_sc1(pp + f) : 0.0;
        if (!keep) q[c] = f < k ? ld_sc1(qp + f) : 0.0;
      }
      const double ru = regU[u], ri = regI[i];  // lambda / omega (read-only in the sweep)
#pragma unroll
      for (int c = 0; c < KPL; ++c) pr[c] = pv[c] * q[c];
      const double e = r - seq_dot<KPL>(pr, k);  // :405
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        const int f = lane + 64 * c;
        const double pn = pv[c] - eta * (ru * pv[c] - e * q[c]);  // :407-408
        const double qn = q[c] - eta * (ri * q[c] - e * pv[c]);   // :409-410 (old p)
        q[c] = qn;
        if (f < k) {
          st_sc1(pp + f, pn);
          if (!(qf & kDetDeferQ)) st_sc1(qp + f, qn);
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this entry's row stores have landed
      if (lane == 0) __hip_atomic_store(tk, useq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int KPL>
int det_capacity() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_det_sweep<KPL>, 64, 0) != hipSuccess) return 0;
  return cus * per_cu;
}

}  // namespace

int det_sweep_capacity(int k) {
  if (k <= 64) return det_capacity<1>();
  if (k <= 128) return det_capacity<2>();
  if (k <= 256) return det_capacity<4>();
  return det_capacity<8>();
}

void launch_det_sweep(hipStream_t st, const DetWave* waves, int nw, const uint32_t* eu, const uint32_t* ei,
                      const uint32_t* eq, const double* er, double* U, double* I, const double* regU,
                      const double* regI, int k, double eta, int32_t* ticket, int32_t* err, hipEvent_t ev0,
                      hipEvent_t ev1) {
  if (nw <= 0) return;
  const dim3 g(static_cast<unsigned>(nw)), b(64);
#define MF_DET(KPL)                                                                                              \
  hipExtLaunchKernelGGL((k_det_sweep<KPL>), g, b, 0, st, ev0, ev1, 0, waves, eu, ei, eq, er, U, I, regU, regI, k, \
                        eta, ticket, err)
  if (k <= 64) MF_DET(1);
  else if (k <= 128) MF_DET(2);
  else if (k <= 256) MF_DET(4);
  else MF_DET(8);
#undef MF_DET
}

}  // namespace mfhip
