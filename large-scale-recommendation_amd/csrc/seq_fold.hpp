// seq_fold.hpp -- the reference's sequential dot product (kernels_detsweep.hip,
// k_online_sweep in kernels_det.hip).  Included inside namespace mfhip { namespace { ... } }.
//
// acc = ((0 + x0) + x1) + ... + x_{k-1} exactly as netlib F2jBLAS.ddot / Scala's foldLeft sum
// (DSGDforMF.scala:405, core/FactorUpdater.scala:39), where lane l holds x_{l + 64c} in prod[c].
// The order is fixed, so the fold is one dependent chain of k adds (5.4 cycles each for f64 on
// gfx950, profiles/r03_valu_latency_microbench.txt): the floor of every chained update.
//
// The products go through a wave-private LDS row and are read back 16 B at a time.  For f32 the
// reads are pinned kPre ahead of the add chain with scheduling barriers (the compiler's own
// schedule keeps only ~4 in flight, under the ~64-cycle LDS latency; online f32 batches 1.43e8 ->
// 1.57e8 ratings/s); for f64 the compiler's schedule is the faster one (det NFLX 233 -> 223 ms per
// epoch, online f64 1.33e8 -> 1.44e8 ratings/s without the barriers, profiles/r03_det_online_ab.txt).  Every lane folds (64-lane broadcast reads, no readlane afterwards); LANE0 = one
// lane folds and the sum is read back with v_readlane -- measured the same ~1660 cycles per
// 128-element f64 fold (profiles/r03_det_probe.txt), i.e. ~13 cycles per add against the 5.4-cycle
// add latency: a single wave's LDS reads, not the adds, set the pace.  LDS operations of one wave
// execute in issue order, so the reads see every lane's writes without an lgkmcnt(0) drain in
// between, and the next call's writes cannot overtake this call's reads; the compiler barriers
// only keep the compiler from moving them.
#pragma once

template <typename T>
__device__ __forceinline__ T lane0_value(T v) {
  if constexpr (sizeof(T) == 8) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b & 0xffffffffu), 0));
    const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b >> 32), 0));
    return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
  } else {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  }
}

template <typename T, int KPL, bool LANE0 = false>
__device__ __forceinline__ T seq_fold(const T (&prod)[KPL], int k, T* lds, int lane) {
#pragma unroll
  for (int c = 0; c < KPL; ++c) lds[64 * c + lane] = prod[c];
  __builtin_amdgcn_wave_barrier();
  T acc = T(0);
  if (!LANE0 || lane == 0) {
    if (k == 64 * KPL) {
      typedef T V __attribute__((ext_vector_type(16 / sizeof(T))));
      constexpr int E = 16 / sizeof(T);     // elements per 16-B read
      constexpr int R = 64 * KPL / E;       // reads
      constexpr int kPre = R < 8 ? R : 8;   // reads in flight ahead of the chain
      const V* l = reinterpret_cast<const V*>(lds);
      V buf[kPre];
#pragma unroll
      for (int x = 0; x < kPre; ++x) buf[x] = l[x];
#pragma unroll
      for (int x = 0; x < R; ++x) {
        // the read kPre ahead is issued before read x's adds, and the scheduler may not pull it
        // down (left alone it keeps only ~4 reads in flight, under the ~64-cycle LDS latency)
        const V v = buf[x % kPre];
        if (x + kPre < R) buf[x % kPre] = l[x + kPre];
        if constexpr (sizeof(T) == 4) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < E; ++e) acc = acc + v[e];
      }
    } else {
      for (int x = 0; x < k; ++x) acc = acc + lds[x];
    }
  }
  __builtin_amdgcn_wave_barrier();
  return LANE0 ? lane0_value(acc) : acc;
}
