// pair_device.hpp -- device helpers of the pair sweep (kernels_pair.hip):
// wave reductions, raw-buffer row access, and the 64-B pair record chunks (plan.hpp PairRec).
// Included inside namespace mfhip { namespace { ... } } of each kernel file.
#pragma once

typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef uint32_t u3v __attribute__((ext_vector_type(3)));

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ float rlf(float v, int l) { return __uint_as_float(rl(__float_as_uint(v), l)); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float u2f(uint32_t v) { return __uint_as_float(v); }
__device__ __forceinline__ uint32_t f2u(float v) { return __float_as_uint(v); }

// Three 64-lane sums at once, uniform results.  gfx950's half swaps fold the three values into
// one register first (v_permlane32_swap: x | y halves; v_permlane16_swap: rows of x, z, y, z),
// so only one 16-lane butterfly remains: 10 VALU operations instead of 18 interleaved DPP adds
// (measured equal per step: a swap costs ~14 cycles against ~4.6 for an interleaved DPP add).
__device__ __forceinline__ void wave_sum3(float& x, float& y, float& z) {
  const auto xy = __builtin_amdgcn_permlane32_swap(f2u(x), f2u(y), false, false);  // [x_lo y_lo], [x_hi y_hi]
  const auto zz = __builtin_amdgcn_permlane32_swap(f2u(z), f2u(z), false, false);  // [z_lo z_lo], [z_hi z_hi]
  const float v = u2f(xy[0]) + u2f(xy[1]);  // lanes 0-31: x halves summed, 32-63: y
  const float w = u2f(zz[0]) + u2f(zz[1]);  // z halves summed (both halves)
  const auto vw = __builtin_amdgcn_permlane16_swap(f2u(v), f2u(w), false, false);
  float s = u2f(vw[0]) + u2f(vw[1]);  // row 0: x, row 1: z, row 2: y, row 3: z (16-lane partials)
  s += dpp<0xB1>(s);
  s += dpp<0x4E>(s);
  s += dpp<0x141>(s);
  s += dpp<0x140>(s);
  x = rlf(s, 0);
  z = rlf(s, 16);
  y = rlf(s, 32);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0xFFFFF000ull ? 0xFFFFF000u : static_cast<uint32_t>(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}

// A lane holds floats [lane*KPL, (lane+1)*KPL) of a row, as NV float pairs.
template <int KPL>
struct Row {
  static constexpr int NV = KPL == 1 ? 1 : KPL / 2;
  f2 v[NV];
};

// Cache policy of a row access: 0 = plain; kSC1 = sc1 (L1 bypass on loads, write-through and
// dropped from the XCD's L2 on stores), used for user rows handed between waves of the
// systolic sweep (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms).
constexpr int kSC1 = 16;

template <int KPL, int POL = 0>
__device__ __forceinline__ Row<KPL> ld(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off) {
  Row<KPL> r;
  if constexpr (KPL == 1) {
    r.v[0] = f2{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, off, POL)), 0.f};
  } else if constexpr (KPL == 2) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, off, POL);
    r.v[0] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
  } else {
#pragma unroll
    for (int c = 0; c < KPL / 4; ++c) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u * c, off, POL);
      r.v[2 * c] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
      r.v[2 * c + 1] = f2{__uint_as_float(x[2]), __uint_as_float(x[3])};
    }
  }
  return r;
}

// A 16-B buffer store, then two wait states before its data VGPRs can be rewritten.  gfx950
// reads a store's data after issuing it: a VALU that overwrites the data VGPRs right behind a
// buffer_store_dwordx4 corrupts the stored row under load -- 1.2% of 16-B records with the offset
// in an SGPR and no wait state, 1.5% with soffset 0 and one wait state, none with two
// (tools/micro/store_data_hazard.hip, profiles/r05_store_data_hazard.txt).  LLVM pads one wait
// state, and none at all when soffset is an SGPR (the table's exemption), so the round-4 k = 256
// lean sweep, whose compiler reused the data VGPRs one or two instructions after the store, wrote
// torn user rows: it did not repeat itself and biased RMSE by 0.27%.  The s_nop below takes the
// data as operands, so no instruction can rewrite those VGPRs before it, and it is ordered after
// the store (both have side effects).  tests/test_isa.py checks every wide store of the library.
__device__ __forceinline__ void store_b128(u4v d, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off, int pol_sc1) {
  if (pol_sc1) __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, off, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, off, 0);
  asm volatile("s_nop 1" ::"v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]));
}

template <int KPL, int POL = 0>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t off, const Row<KPL>& r) {
  if constexpr (KPL == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.v[0].x), rs, voff, off, POL);
  } else if constexpr (KPL == 2) {
    using u2 = uint32_t __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(r.v[0].x), __float_as_uint(r.v[0].y)}, rs, voff, off, POL);
  } else {
    static_assert(POL == 0 || POL == 16, "store policy");
#pragma unroll
    for (int c = 0; c < KPL / 4; ++c)
      store_b128(u4v{__float_as_uint(r.v[2 * c].x), __float_as_uint(r.v[2 * c].y), __float_as_uint(r.v[2 * c + 1].x),
                     __float_as_uint(r.v[2 * c + 1].y)},
                 rs, voff + 16u * c, off, POL == 16);
  }
}

// s * x + y as one packed fused multiply-add (v_pk_fma_f32): the compiler does not contract a
// scalar-times-vector product into the add by itself (it emitted v_pk_mul + v_pk_add)
__device__ __forceinline__ f2 vfma(float s, f2 x, f2 y) { return __builtin_elementwise_fma(f2{s, s}, x, y); }

template <int KPL>
__device__ __forceinline__ float dot_part(const Row<KPL>& a, const Row<KPL>& b) {
  f2 acc = a.v[0] * b.v[0];
#pragma unroll
  for (int e = 1; e < Row<KPL>::NV; ++e) acc = a.v[e] * b.v[e] + acc;
  return KPL == 1 ? acc.x : acc.x + acc.y;
}

// CH consecutive pair records of the cell, pair y in lane y (index clamped to the cell).
struct Chunk {
  uint32_t ua, ub, ia, ib;  // loads (byte offsets)
  uint32_t sa, sb, sia, si; // stores
  uint32_t flags;
  float era, erb;           // eta * r
  float aa, ab, ba, bb;     // 1 - eta * ri, 1 - eta * ru (1 for no-op records)
  float sr, m;              // 1 - split; split ? 1 : aa (B's coupling to A's update)
};

// A chunk's records as loaded (raw words, one pair per lane).  The next chunk is loaded a whole
// chunk ahead and only converted (eta folded in) when it becomes current, so nothing reads a
// just-loaded register at the chunk boundary and the factor-row ring keeps running across it
// (converting at load time made every chunk boundary wait for its own record loads).
// s_waitcnt vmcnt(0) the compiler can see (gfx9 encoding: expcnt 7, lgkmcnt 15).  Round 4 issued
// it after a cell's ring prefill: otherwise the loop header inherited the preheader's "just loaded"
// ring rows and the compiler drained the ring at every chunk boundary.  With the exit-free chunk
// loop (sweep_chunks) the header waits are the same with or without it at KPL <= 2
// (tools/isa_waits.py), so those cells start on their first pair's rows instead of waiting for the
// whole ring (~56 loads issued back to back, ~0.25 us per cell); KPL = 4 keeps it (without it
// its header waits turn conservative).
__device__ __forceinline__ void drain_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

struct ChunkRaw {
  u4v w0, w1, w2;
  u3v w3;  // the fourth word group's last word is unused: a 12-B load (no dead VGPR a load still writes)
};

// A cell's pair records as a raw buffer of exactly its records: a lane past the cell's last pair
// reads zeros (no clamp, no per-cell vector address arithmetic: the cell is an SGPR base and size,
// the lane a constant voffset), which only the prefetch of rows for pairs past the end consumes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cell_records(const u4v* recs, int64_t base, int npairs) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<u4v*>(recs + 4 * base), 0,
                                           static_cast<uint32_t>(npairs > 0 ? npairs : 0) * 64u, 0x00020000);
}
// Chunk c of the cell: pair c * CH + lane in lane `lane` (vlane = lane * 64).  Records are
// read once: non-temporal (cache policy nt), so they do not push factor rows out of L2 / MALL.
template <int CH>
__device__ __forceinline__ ChunkRaw chunk_load(__amdgpu_buffer_rsrc_t rr, int c, uint32_t vlane) {
  // c is uniform, but the divergence analysis cannot always prove it through the cell loops'
  // exits (the generic k = 128 loop's chunk loads became a readfirstlane waterfall): say so
  const uint32_t so = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(c)) * CH * 64u;
  constexpr int kNT = 2;
  return ChunkRaw{__builtin_amdgcn_raw_buffer_load_b128(rr, vlane, so, kNT),
                  __builtin_amdgcn_raw_buffer_load_b128(rr, vlane + 16u, so, kNT),
                  __builtin_amdgcn_raw_buffer_load_b128(rr, vlane + 32u, so, kNT),
                  __builtin_amdgcn_raw_buffer_load_b96(rr, vlane + 48u, so, kNT)};
}

// A use of every word group of a chunk on a cell's exit path.  Without a use there, LLVM's IR
// sinking pass moves each record load of chunk c + 1 (issued when chunk c starts) down to the
// block of its first use -- 49 pairs later for the ring offsets, the chunk's end for the rest --
// where the wave then waits a whole memory round trip for it.  The exit is reached from every
// pair, so no block below the load dominates all uses and the loads stay where they are issued.
__device__ __forceinline__ void keep_chunk(const ChunkRaw& r) {
  __asm__ volatile("; keep %0 %1 %2 %3" ::"v"(r.w0[0]), "v"(r.w1[0]), "v"(r.w2[0]), "v"(r.w3[0]));
}

__device__ __forceinline__ Chunk chunk_convert(const ChunkRaw& r, float eta) {
  Chunk ch;
  ch.ua = r.w0[0]; ch.ub = r.w0[1]; ch.ia = r.w0[2]; ch.ib = r.w0[3];
  ch.sa = r.w1[0]; ch.sb = r.w1[1]; ch.sia = r.w1[2]; ch.si = r.w1[3];
  ch.flags = r.w2[0];
  ch.era = eta * __uint_as_float(r.w2[1]);
  ch.erb = eta * __uint_as_float(r.w2[2]);
  ch.ba = fmaf(-eta, __uint_as_float(r.w2[3]), 1.f);
  ch.bb = fmaf(-eta, __uint_as_float(r.w3[0]), 1.f);
  ch.aa = fmaf(-eta, __uint_as_float(r.w3[1]), 1.f);
  ch.ab = fmaf(-eta, __uint_as_float(r.w3[2]), 1.f);
  const bool split = (r.w2[0] & kPairSplit) != 0;
  ch.sr = split ? 0.f : 1.f;
  ch.m = split ? 1.f : ch.aa;  // == fmaf(sr, aa - 1, 1) exactly: aa - 1 and its sum with 1 are exact
  return ch;
}

// Calls f(std::integral_constant<int, 0>{}) ... f(integral_constant<int, N - 1>{}) in order: the
// pair index is a compile-time constant in every copy of the step (constant readlane lanes,
// constant ring slots).  unroll_while stops after the first call that returns false.
template <typename F, int... S>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <typename F, int... S>
__device__ __forceinline__ void unroll_while_seq(F&& f, std::integer_sequence<int, S...>) {
  (void)(f(std::integral_constant<int, S>{}) && ...);
}

// The pairs of one cell, CH per record chunk: pair(integral_constant<int, s>) runs pair s of the
// current chunk, load_next(c) loads chunk c + 1 when chunk c starts (a record is first read 49 pairs
// later), advance() makes it current.  Full chunks run without exit tests and with a scheduling
// barrier between pairs; only the last, partial chunk tests each pair.  (With a per-pair exit in
// every chunk -- the natural loop -- the structurizer's flow blocks for 56 exits ran on the normal
// path too and copied ring registers whose loads were still in flight: a vmcnt(3) wait, one memory
// round trip, at every chunk boundary.  The barriers keep the scheduler from interleaving pairs of
// the now branch-free chunk, which pulled later pairs' uses of just-loaded rows forward.)
template <int CH, typename P, typename L, typename A>
__device__ __forceinline__ void sweep_chunks(int npairs, P&& pair, L&& load_next, A&& advance) {
  const int full = __builtin_amdgcn_readfirstlane(npairs / CH);
  const int rem = __builtin_amdgcn_readfirstlane(npairs - full * CH);  // uniform: scalar tests
  int c = 0;
  for (; c < full; ++c) {
    load_next(c);
    unroll_seq(
        [&](auto S) __attribute__((always_inline)) {
          __builtin_amdgcn_sched_barrier(0);
          pair(S);
        },
        std::make_integer_sequence<int, CH>{});
    advance();
  }
  load_next(c);
  unroll_while_seq(
      [&](auto S) __attribute__((always_inline)) {
        if (decltype(S)::value >= rem) return false;
        __builtin_amdgcn_sched_barrier(0);
        pair(S);
        return true;
      },
      std::make_integer_sequence<int, CH>{});
}

// -eta in a VGPR: the per-pair scalar recurrence runs in the chunk layout (lane s = pair s), where
// each step reads one SGPR (a wave sum) and takes -eta from a register, so no SGPR is copied to a
// VGPR first (one SGPR per VALU instruction on gfx9).
__device__ __forceinline__ float vgpr_of(float x) {
  float v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
}
