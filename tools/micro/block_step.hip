// What one wave can do per update with the single-run "block solve" (round-6 review, item 1):
// L = 16 consecutive updates of one item solved as a block -- the Gram P P^T and the cross-Grams to
// the next two blocks on the matrix cores (v_mfma_f32_16x16x32_bf16), the block's start values P q
// as an f32 GEMV, and only a scalar forward substitution left on the chain:
//   w_j = eta r_j - eta t_j ;  t <- a_j t + w_j G[:, j]      (t_l = p_l . q_j, lane l)
//   p_j' = b_j p_j + w_j q_j ;  q_{j+1} = a_j q_j + w_j p_j  (DSGDforMF.scala:405-410)
// This is the instruction MIX of that design at k = 128 on one wave -- every per-update and every
// per-block operation the full kernel needs, with their true register dependencies on the chain
// (t -> w -> t, q -> q) -- not a numerically meaningful sweep (the tiles are not re-derived from
// the rows they would describe).  It bounds what the design can reach on one wave: the sweep is
// issue-bound (one wave issues about one instruction per ~4 cycles, profiles/r05_fold_fill_
// microbench.txt), so the instruction count per update sets ns per update.
//   mode 0: the per-update steps only (the floor: MFMA, GEMV and column work free)
//   mode 1: steps + the per-block work (row fields, MFMA-layout row loads, bf16 packing, 12 MFMAs,
//           the tiles' columns through LDS, the f32 GEMV for the next blocks' start values)
// Compare: the pair step of k_sweep_pair_sys runs the same one-wave chain at 53 ns per update
// (tools/chain_bench.py, profiles/r05_chain_bench.txt).
//
//   hipcc -O3 --offload-arch=gfx950 -o block_step block_step.hip && ./block_step
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

constexpr int L = 16;         // updates per block
constexpr int kRowBytes = 512;  // k = 128 f32
constexpr int kSC1 = 16;

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ float rlf(float v, int l) { return __uint_as_float(rl(__float_as_uint(v), l)); }
__device__ __forceinline__ f2 vfma(float s, f2 x, f2 y) { return __builtin_elementwise_fma(f2{s, s}, x, y); }

struct Fields {
  uint32_t uoff;  // lane n16: the block's record n16 (all four lane groups alike)
  float era, a, b;
};

template <int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_block(
    float* __restrict__ U, const uint32_t* __restrict__ uoff, const float* __restrict__ rv, const float* __restrict__ ru,
    const float* __restrict__ ri, int nblk, float eta, float* __restrict__ out, uint64_t* __restrict__ t) {
  const int lane = threadIdx.x, g = lane >> 4, n16 = lane & 15;
  const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(U, 0, 0xFFFFF000u, 0x00020000);
  __shared__ float tiles[4 * 272];  // tile d: [j][n] at d * 272 + j * 16 + n (272: no bank conflicts)
  __shared__ float qs[128];
  auto fields = [&](int blk) {
    const int x = blk * L + n16;
    Fields f;
    f.uoff = uoff[x];
    f.era = eta * rv[x];
    f.b = __builtin_fmaf(-eta, ru[x], 1.f);
    f.a = __builtin_fmaf(-eta, ri[x], 1.f);
    return f;
  };
  // MFMA-layout rows of a block: lane l holds row n16, K-slice c columns 32c + 8g .. +7
  auto load_m = [&](const Fields& f, f4 (&m)[8]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u4 x = __builtin_amdgcn_raw_buffer_load_b128(urs, f.uoff + (32 * c + 8 * g + 4 * h) * 4u, 0, kSC1);
        m[2 * c + h] = f4{__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]), __uint_as_float(x[3])};
      }
  };
  auto pack = [&](const f4 (&m)[8], bf8 (&mb)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mb[c][e] = static_cast<__bf16>(m[2 * c][e]);
        mb[c][4 + e] = static_cast<__bf16>(m[2 * c + 1][e]);
      }
  };
  f2 q = f2{out[2 * lane] * 1e-3f, out[2 * lane + 1] * 1e-3f};
  const float neta = -eta;
  Fields F0 = fields(0), F1 = fields(1), F2 = fields(2), F3 = fields(3);
  f2 P[2][L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(urs, lane * 8u, rl(F0.uoff, j), kSC1);
    P[0][j] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
  }
  // MFMA-layout rows two blocks ahead: M[0] = block b+2 (landed), M[1] = block b+3 (in flight);
  // the roles alternate between the two unrolled blocks of an iteration
  f4 M[2][8];
  load_m(F2, M[0]);
  load_m(F3, M[1]);
  bf8 B[2][4];
  pack(M[1], B[1]);  // stands for block b+1's operands at the first block
  float COL[L];
#pragma unroll
  for (int j = 0; j < L; ++j) COL[j] = 1e-3f * static_cast<float>(lane ^ j);
  float T = 1e-3f * static_cast<float>(lane);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const uint64_t c0 = __builtin_amdgcn_s_memrealtime();
  for (int b = 0; b < nblk; b += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // two blocks per iteration: static register-set indices
      const int cur = h, nxt = 1 - h;
      const Fields F4 = fields(b + h + 4);  // four blocks ahead (its rows' MFMA-layout load)
      float COLn[L], V = 0.f;
      if constexpr (MODE == 1) {
        // block b+2's rows (landed) as bf16 operands; the Gram / cross-Gram tiles of the next
        // block (rows b+1 x {b+1, b+2}, and one more cross tile) on the matrix cores; their
        // columns through LDS; the f32 GEMV of block b+2's start values against this block's
        // starting item row
        pack(M[h], B[h]);
        f4 C0 = {0.f, 0.f, 0.f, 0.f}, C1 = C0, C2 = C0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          C0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[1 - h][c], B[1 - h][c], C0, 0, 0, 0);
          C1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[1 - h][c], B[h][c], C1, 0, 0, 0);
          C2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[h][c], B[1 - h][c], C2, 0, 0, 0);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {  // C[4g + v][n16] of each tile
          tiles[0 * 272 + (4 * g + v) * 16 + n16] = C0[v];
          tiles[1 * 272 + (4 * g + v) * 16 + n16] = C1[v];
          tiles[2 * 272 + (4 * g + v) * 16 + n16] = C2[v];
        }
        qs[2 * lane] = q.x;
        qs[2 * lane + 1] = q.y;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < L; ++j) COLn[j] = tiles[(g < 3 ? g : 0) * 272 + j * 16 + n16];
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const f4 qa = *reinterpret_cast<const f4*>(&qs[32 * c + 8 * g]);
          const f4 qb = *reinterpret_cast<const f4*>(&qs[32 * c + 8 * g + 4]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc = __builtin_fmaf(M[h][2 * c][e], qa[e], acc);
            acc = __builtin_fmaf(M[h][2 * c + 1][e], qb[e], acc);
          }
        }
        const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc), __float_as_uint(acc), false, false);
        const float a2 = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
        const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a2), __float_as_uint(a2), false, false);
        V = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
        load_m(F4, M[h]);  // block b+4's rows, used two blocks on
      }
      // the chain: 16 updates
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const float wv = __builtin_fmaf(T, neta, F0.era);
        const float w = rlf(wv, j);
        const float aj = rlf(F0.a, j), bj = rlf(F0.b, j);
        T = __builtin_fmaf(COL[j], w, aj * T);
        const f2 p = P[cur][j];
        const f2 pn = vfma(w, q, f2{bj, bj} * p);
        q = vfma(w, p, f2{aj, aj} * q);
        using u2 = uint32_t __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(pn.x), __float_as_uint(pn.y)}, urs, lane * 8u,
                                              rl(F0.uoff, j), kSC1);
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(urs, lane * 8u, rl(F1.uoff, j), kSC1);
        P[nxt][j] = f2{__uint_as_float(x[0]), __uint_as_float(x[1])};
      }
      // block end: the next block's start values and columns
      T = __builtin_fmaf(V, 1e-6f, T);
      if constexpr (MODE == 1) {
#pragma unroll
        for (int j = 0; j < L; ++j) COL[j] = COLn[j];
      }
      F0 = F1;
      F1 = F2;
      F2 = F3;
      F3 = F4;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const uint64_t c1 = __builtin_amdgcn_s_memrealtime();
  out[2 * lane] = q.x + T;
  out[2 * lane + 1] = q.y;
  if (lane == 0) t[0] = c1 - c0;
}

int main() {
  const int n = 1 << 17;  // updates (131072), distinct users
  const int nblk = n / L;
  const int rows = n + 8 * L;
  std::vector<uint32_t> off(static_cast<size_t>(nblk + 8) * L);
  std::vector<float> r(off.size()), ru(off.size()), ri(off.size());
  uint64_t s = 12345;
  std::vector<uint32_t> perm(rows);
  for (int x = 0; x < rows; ++x) perm[x] = x;
  for (int x = rows - 1; x > 0; --x) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    std::swap(perm[x], perm[(s >> 33) % (x + 1)]);
  }
  for (size_t x = 0; x < off.size(); ++x) {
    off[x] = perm[x % rows] * kRowBytes;
    r[x] = 1.f + static_cast<float>(x % 5);
    ru[x] = 0.01f;
    ri[x] = 1e-5f;
  }
  float *U, *rv, *rud, *rid, *out;
  uint32_t* offd;
  uint64_t* t;
  CK(hipMalloc(&U, static_cast<size_t>(rows) * kRowBytes));
  CK(hipMemset(U, 0, static_cast<size_t>(rows) * kRowBytes));
  CK(hipMalloc(&offd, off.size() * 4));
  CK(hipMalloc(&rv, off.size() * 4));
  CK(hipMalloc(&rud, off.size() * 4));
  CK(hipMalloc(&rid, off.size() * 4));
  CK(hipMalloc(&out, 1024 * 4));
  CK(hipMalloc(&t, 8));
  CK(hipMemset(out, 0, 1024 * 4));
  CK(hipMemcpy(offd, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(rv, r.data(), off.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(rud, ru.data(), off.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(rid, ri.data(), off.size() * 4, hipMemcpyHostToDevice));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      if (mode == 0)
        hipLaunchKernelGGL(k_block<0>, dim3(1), dim3(64), 0, 0, U, offd, rv, rud, rid, nblk, 0.001f, out, t);
      else
        hipLaunchKernelGGL(k_block<1>, dim3(1), dim3(64), 0, 0, U, offd, rv, rud, rid, nblk, 0.001f, out, t);
      CK(hipDeviceSynchronize());
      uint64_t ticks = 0;
      CK(hipMemcpy(&ticks, t, 8, hipMemcpyDeviceToHost));
      std::printf("mode %d (%s) rep %d: %.2f ns per update (%d updates, one wave, k = 128, L = %d)\n", mode,
                  mode == 0 ? "per-update steps only" : "steps + per-block MFMA / GEMV / LDS work", rep,
                  ticks * 10.0 / n, n, L);
    }
  }
  return 0;
}
