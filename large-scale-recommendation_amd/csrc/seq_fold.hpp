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

// The same fold with no LDS round trip, for k == 64 * KPL.  A single wave issues at most one LDS
// read every ~24 cycles (profiles/r04_fold_microbench.txt: 12-13 cycles per f64 add whatever the
// read width, window or EXEC), so the operands are brought to row 0 (lanes 0-15) in registers
// instead: v_permlane16_swap / v_permlane32_swap copy rows 1-3 of each product register to row 0
// of three more registers (3 swaps per dword), then every add reads its operand straight from the
// register file through DPP row_newbcast:n (lane n of the row, the only DPP mode the f64 ALU
// has).  f64 has no v_add_f64_dpp, so the add is v_fmac_f64_dpp acc, x, 1.0: x * 1.0 is exact, so
// fma(x, 1.0, acc) is the single rounding of acc + x -- bitwise the add.  Element 64c + 16r + n is
// register (c, r), lane n: the adds run f = 0, 1, ..., 64 KPL - 1 in order.  Every lane of row 0
// ends with the sum (rows 1-3 hold garbage); returned as a wave-uniform value.
// One dword d: rows 1, 2, 3 of d to row 0 of three registers, three swaps and no copies.  A swap
// delivers one new row-0 value (into its second operand), so three per dword is the minimum; the
// second operands start as don't-care registers (an empty asm defines them), since only their row
// 0 after the swap is read.  swap16(a, b): b.row0 <- a.row1, b.row2 <- a.row3 (a keeps rows 0, 2);
// swap32(a, b): b.rows0,1 <- a.rows2,3 (a keeps rows 0, 1).
__device__ __forceinline__ void dword_views(unsigned d, unsigned (&v)[4]) {
  unsigned t1, t2, t3;
  asm volatile("" : "=v"(t1), "=v"(t2), "=v"(t3));
  const auto s16 = __builtin_amdgcn_permlane16_swap(d, t1, false, false);   // s16[1].row0 = d.row1, .row2 = d.row3
  const auto s32 = __builtin_amdgcn_permlane32_swap(s16[0], t2, false, false);  // s32[1].row0 = d.row2, s32[0].row0 = d.row0
  const auto s3 = __builtin_amdgcn_permlane32_swap(s16[1], t3, false, false);   // s3[1].row0 = d.row3, s3[0].row0 = d.row1
  v[0] = s32[0];
  v[1] = s3[0];
  v[2] = s32[1];
  v[3] = s3[1];
}
template <typename T>
__device__ __forceinline__ void row_views(T x, T (&v)[4]) {
  if constexpr (sizeof(T) == 8) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(x));
    unsigned lo[4], hi[4];
    dword_views(static_cast<unsigned>(b), lo);
    dword_views(static_cast<unsigned>(b >> 32), hi);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[r] = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi[r]) << 32) | lo[r]));
  } else {
    unsigned d[4];
    dword_views(static_cast<unsigned>(__float_as_int(x)), d);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __int_as_float(static_cast<int>(d[r]));
  }
}

#define MFHIP_FOLD_D(R, N) "v_fmac_f64_dpp %0, %" #R ", %5 row_newbcast:" #N " row_mask:0xf bank_mask:0xf\n\t"
#define MFHIP_FOLD_S(R, N) "v_add_f32_dpp %0, %" #R ", %0 row_newbcast:" #N " row_mask:0xf bank_mask:0xf\n\t"
#define MFHIP_FOLD_ROW(M, R)                                                                         \
  M(R, 0) M(R, 1) M(R, 2) M(R, 3) M(R, 4) M(R, 5) M(R, 6) M(R, 7) M(R, 8) M(R, 9) M(R, 10) M(R, 11) \
      M(R, 12) M(R, 13) M(R, 14) M(R, 15)

template <typename T, int KPL>
__device__ __forceinline__ T seq_fold_dpp(const T (&prod)[KPL]) {
  T acc = T(0);
#pragma unroll
  for (int c = 0; c < KPL; ++c) {
    T v[4];
    row_views<T>(prod[c], v);
    // s_nop 1: the two wait states a DPP source needs after the VALU (swap) that wrote it
    if constexpr (sizeof(T) == 8) {
      const double one = 1.0;
      asm volatile("s_nop 1\n\t" MFHIP_FOLD_ROW(MFHIP_FOLD_D, 1) MFHIP_FOLD_ROW(MFHIP_FOLD_D, 2)
                       MFHIP_FOLD_ROW(MFHIP_FOLD_D, 3) MFHIP_FOLD_ROW(MFHIP_FOLD_D, 4)
                   : "+v"(acc)
                   : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(one));
    } else {
      asm volatile("s_nop 1\n\t" MFHIP_FOLD_ROW(MFHIP_FOLD_S, 1) MFHIP_FOLD_ROW(MFHIP_FOLD_S, 2)
                       MFHIP_FOLD_ROW(MFHIP_FOLD_S, 3) MFHIP_FOLD_ROW(MFHIP_FOLD_S, 4)
                   : "+v"(acc)
                   : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
    }
  }
  return lane0_value(acc);
}
#undef MFHIP_FOLD_ROW
#undef MFHIP_FOLD_S
#undef MFHIP_FOLD_D

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
