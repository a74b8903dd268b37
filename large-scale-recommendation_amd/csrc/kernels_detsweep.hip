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
// element l + 64c in prod[c].  The products go through a wave-private LDS row and every lane
// reads them back in order as broadcast 16-B reads, so the dependent f64 add chain takes its
// operands from VGPRs (a v_readlane per element would add a readlane + hazard nop per add).
template <int KPL>
__device__ __forceinline__ double seq_dot(const double (&prod)[KPL], int k, double* lds, int lane) {
#pragma unroll
  for (int c = 0; c < KPL; ++c) lds[64 * c + lane] = prod[c];
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's own LDS writes are done
  __builtin_amdgcn_wave_barrier();
  double acc = 0.0;
  const double2* l2 = reinterpret_cast<const double2*>(lds);
  if (k == 64 * KPL) {
#pragma unroll
    for (int x = 0; x < 32 * KPL; ++x) {
      const double2 v = l2[x];
      acc = acc + v.x;
      acc = acc + v.y;
    }
  } else {
    const int half = k >> 1;
    for (int x = 0; x < half; ++x) {
      const double2 v = l2[x];
      acc = acc + v.x;
      acc = acc + v.y;
    }
    if (k & 1) acc = acc + lds[k - 1];
  }
  __builtin_amdgcn_wave_barrier();  // every lane has read before the next entry rewrites the row
  return acc;
}

// Entry fields of a wave's entry list, 64 per lane-register chunk.
struct DetChunk {
  uint32_t u, i, q;
  double r;
};
__device__ __forceinline__ DetChunk det_chunk(const uint32_t* eu, const uint32_t* ei, const uint32_t* eq,
                                              const double* er, int64_t begin, int64_t count, int64_t c0, int lane) {
  const int64_t j = c0 + lane;
  const bool in = j < count;
  const int64_t x = begin + (in ? j : 0);
  return DetChunk{in ? eu[x] : 0u, in ? ei[x] : 0u, in ? eq[x] : 0u, in ? er[x] : 0.0};
}

__device__ __forceinline__ int32_t poll(const int32_t* t) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Pipelined per wave: at entry j the row of entry j+1 is prefetched when the ticket poll issued
// one entry earlier already showed it ready, and entry j+2's ticket is polled; entry j-1's row
// stores drain while entry j computes, and its ticket is published after that drain (and always
// before the wave blocks on a ticket, so a published ticket never waits on this wave).
template <int KPL>
__global__ __launch_bounds__(64) void k_det_sweep(const DetWave* __restrict__ waves, const uint32_t* __restrict__ eu,
                                                  const uint32_t* __restrict__ ei, const uint32_t* __restrict__ eq,
                                                  const double* __restrict__ er, double* U, double* I,
                                                  const double* __restrict__ regU, const double* __restrict__ regI,
                                                  int k, double eta, int32_t* ticket, int32_t* err) {
  __shared__ double lds[64 * KPL];
  const int lane = threadIdx.x;
  const DetWave d = waves[blockIdx.x];
  const int64_t cnt = d.count;
  if (cnt == 0) return;
  auto row_load = [&](double (&v)[KPL], const double* base) {
#pragma unroll
    for (int c = 0; c < KPL; ++c) {
      const int f = lane + 64 * c;
      v[c] = f < k ? ld_sc1(base + f) : 0.0;
    }
  };
  DetChunk C0 = det_chunk(eu, ei, eq, er, d.begin, cnt, 0, lane);
  DetChunk C1 = det_chunk(eu, ei, eq, er, d.begin, cnt, 64, lane);
  // fields of entry j + dj (dj in 0..2) relative to the chunk pair (C0 = j's chunk)
  auto fu = [&](int s, int dj) { return s + dj < 64 ? rl(C0.u, s + dj) : rl(C1.u, s + dj - 64); };
  auto fq = [&](int s, int dj) { return s + dj < 64 ? rl(C0.q, s + dj) : rl(C1.q, s + dj - 64); };

  double q[KPL], P[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) q[c] = P[c] = 0.0;
  // entry 0: its ticket read now; entry 1's ticket polled ahead
  int32_t okP = 0;
  {
    const uint32_t u0 = rl(C0.u, 0);
    if (poll(ticket + u0) == static_cast<int32_t>(rl(C0.q, 0) & kDetUseqMask)) {
      okP = 1;
      row_load(P, U + static_cast<size_t>(u0) * k);
    }
  }
  int32_t tk1 = cnt > 1 ? poll(ticket + fu(0, 1)) : 0;
  int32_t* pend = nullptr;  // entry j-1's ticket, published once its stores have drained
  int32_t pend_val = 0;

  for (int64_t c0 = 0; c0 < cnt; c0 += 64) {
    if (c0 > 0) {
      C0 = C1;
      C1 = det_chunk(eu, ei, eq, er, d.begin, cnt, c0 + 64, lane);
    }
    const int n = static_cast<int>(min<int64_t>(64, cnt - c0));
    for (int s = 0; s < n; ++s) {
      const int64_t j = c0 + s;
      const uint32_t u = rl(C0.u, s), i = rl(C0.i, s), qf = rl(C0.q, s);
      const double r = rld(C0.r, s);
      const int32_t useq = static_cast<int32_t>(qf & kDetUseqMask);
      // prefetch entry j+1's row if its ticket was ready when polled; poll entry j+2
      double PN[KPL];
      int32_t okN = 0;
#pragma unroll
      for (int c = 0; c < KPL; ++c) PN[c] = 0.0;
      if (j + 1 < cnt) {
        const uint32_t un = fu(s, 1);
        if (tk1 == static_cast<int32_t>(fq(s, 1) & kDetUseqMask) && un != u) {
          okN = 1;
          row_load(PN, U + static_cast<size_t>(un) * k);
        }
      }
      const int32_t tk2 = j + 2 < cnt ? poll(ticket + fu(s, 2)) : 0;
      // entry j's user row: prefetched, or (rarely) wait for its ticket now
      if (!okP) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): entry j-1's stores landed
        if (lane == 0 && pend) __hip_atomic_store(pend, pend_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend = nullptr;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // bounded wait (100 MHz clock)
        while (poll(ticket + u) != useq) {
          if (poll(err) != 0) return;
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // ~1 s: a producer never ran
            if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        row_load(P, U + static_cast<size_t>(u) * k);
      }
      double* qp = I + static_cast<size_t>(i) * k;
      if (!(qf & kDetKeepQ)) row_load(q, qp);  // the item's previous store drained at entry j-1
      const double ru = regU[u], ri = regI[i];  // lambda / omega (read-only in the sweep)
      double pr[KPL];
#pragma unroll
      for (int c = 0; c < KPL; ++c) pr[c] = P[c] * q[c];
      const double e = r - seq_dot<KPL>(pr, k, lds, lane);  // :405
      double pn[KPL];
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        pn[c] = P[c] - eta * (ru * P[c] - e * q[c]);  // :407-408
        q[c] = q[c] - eta * (ri * q[c] - e * P[c]);   // :409-410 (old p)
      }
      // entry j-1's stores are long issued: drain them and publish its ticket
      __builtin_amdgcn_s_waitcnt(0x0F70);
      if (lane == 0 && pend) __hip_atomic_store(pend, pend_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      double* pp = U + static_cast<size_t>(u) * k;
#pragma unroll
      for (int c = 0; c < KPL; ++c) {
        const int f = lane + 64 * c;
        if (f < k) {
          st_sc1(pp + f, pn[c]);
          if (!(qf & kDetDeferQ)) st_sc1(qp + f, q[c]);
        }
      }
      pend = ticket + u;
      pend_val = useq + 1;
#pragma unroll
      for (int c = 0; c < KPL; ++c) P[c] = PN[c];
      okP = okN;
      tk1 = tk2;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if (lane == 0 && pend) __hip_atomic_store(pend, pend_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
