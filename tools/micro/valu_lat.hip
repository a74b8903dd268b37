// One-wave VALU latency / issue microbenchmark for gfx950 (tools only, not part of libmfhip).
// Prints cycles (s_memtime) and ns (s_memrealtime, 100 MHz) per operation for dependent and
// independent instruction streams of the kinds the DSGD sweep kernels are made of.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R16(x) x x x x x x x x x x x x x x x x
constexpr int kIters = 512;

template <int T>
__global__ void k(float* out, unsigned long long* t, float a) {
  __shared__ float lds[256];
  if (T == 17 || T == 18) { for (int x = threadIdx.x; x < 256; x += blockDim.x) lds[x] = 0.f; __syncthreads(); }
  float v0 = threadIdx.x * 1e-3f, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  int s = 0;
  const unsigned long long c0 = clock64(), r0 = wall_clock64();
  for (int it = 0; it < kIters; ++it) {
    if constexpr (T == 0) {  // dependent v_add_f32
      asm volatile(R16("v_add_f32 %0, %0, %1\n\t") : "+v"(v0) : "v"(v1));
    } else if constexpr (T == 1) {  // 4 independent chains
      asm volatile(R16("v_add_f32 %0, %0, %4\n\tv_add_f32 %1, %1, %4\n\tv_add_f32 %2, %2, %4\n\tv_add_f32 %3, %3, %4\n\t")
                   : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "v"(v4));
    } else if constexpr (T == 2) {  // dependent DPP add (2 wait states required)
      asm volatile(R16("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t") : "+v"(v0));
    } else if constexpr (T == 3) {  // 3 interleaved DPP chains
      asm volatile(R16("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t")
                   : "+v"(v0), "+v"(v1), "+v"(v2));
    } else if constexpr (T == 4) {  // readlane -> VALU chain
      asm volatile(R16("v_readlane_b32 %1, %0, 0\n\tv_add_f32 %0, %1, %0\n\t") : "+v"(v0), "+s"(s));
    } else if constexpr (T == 5) {  // permlane32 swap + add chain
      asm volatile(R16("v_permlane32_swap_b32 %0, %1\n\ts_nop 1\n\tv_add_f32 %0, %0, %1\n\t") : "+v"(v0), "+v"(v1));
    } else if constexpr (T == 6) {  // dependent v_pk_fma_f32
      asm volatile(R16("v_pk_fma_f32 %0, %0, %1, %2\n\t") : "+v"(*(double*)&v0) : "v"(*(double*)&v2), "v"(*(double*)&v4));
    } else if constexpr (T == 7) {  // 4 independent pk_fma chains
      asm volatile(R16("v_pk_fma_f32 v[20:21], v[20:21], v[28:29], v[30:31]\n\tv_pk_fma_f32 v[22:23], v[22:23], v[28:29], v[30:31]\n\tv_pk_fma_f32 v[24:25], v[24:25], v[28:29], v[30:31]\n\tv_pk_fma_f32 v[26:27], v[26:27], v[28:29], v[30:31]\n\t")
                   ::: "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27");
    } else if constexpr (T == 8) {  // independent readlanes
      asm volatile(R16("v_readlane_b32 s40, %0, 1\n\tv_readlane_b32 s41, %0, 2\n\tv_readlane_b32 s42, %0, 3\n\tv_readlane_b32 s43, %0, 4\n\t") :: "v"(v0) : "s40", "s41", "s42", "s43");
    } else if constexpr (T == 9) {  // VALU with SGPR operand written by readlane, then VALU -> readlane
      asm volatile(R16("v_readlane_b32 %1, %0, 63\n\tv_fma_f32 %0, %1, %2, %0\n\t") : "+v"(v0), "+s"(s) : "v"(v2));
    } else if constexpr (T == 10) {  // dependent v_fma_f32
      asm volatile(R16("v_fma_f32 %0, %0, %1, %2\n\t") : "+v"(v0) : "v"(v1), "v"(v2));
    } else if constexpr (T == 11) {  // 8 independent v_fma
      asm volatile(R16("v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\tv_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\tv_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\tv_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8\n\t")
                   : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) : "v"(a));
    } else if constexpr (T == 12) {  // row_bcast DPP chain
      asm volatile(R16("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t") : "+v"(v0));
    } else if constexpr (T == 13) {  // ds_swizzle / bpermute chain
      asm volatile(R16("ds_swizzle_b32 %0, %0 offset:swizzle(SWAP,1)\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(v0));
    } else if constexpr (T == 14) {  // dependent v_add_f64
      asm volatile(R16("v_add_f64 %0, %0, %1\n\t") : "+v"(*(double*)&v0) : "v"(*(double*)&v2));
    } else if constexpr (T == 15) {  // dependent v_fma_f64
      asm volatile(R16("v_fma_f64 %0, %0, %1, %2\n\t") : "+v"(*(double*)&v0) : "v"(*(double*)&v2), "v"(*(double*)&v4));
    } else if constexpr (T == 16) {  // 4 independent v_add_f64 chains
      asm volatile(R16("v_add_f64 v[20:21], v[20:21], v[28:29]\n\tv_add_f64 v[22:23], v[22:23], v[28:29]\n\tv_add_f64 v[24:25], v[24:25], v[28:29]\n\tv_add_f64 v[26:27], v[26:27], v[28:29]\n\t")
                   ::: "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27");
    } else if constexpr (T == 17) {  // LDS broadcast b128 read -> use (latency), address from the data
      asm volatile(R16("ds_read_b128 v[20:23], %0\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %0, v20\n\t") : "+v"(s) :: "v20", "v21", "v22", "v23");
    } else if constexpr (T == 18) {  // 8 independent broadcast b128 reads then wait (throughput)
      asm volatile(R16("ds_read_b128 v[20:23], %0\n\tds_read_b128 v[24:27], %0 offset:16\n\tds_read_b128 v[28:31], %0 offset:32\n\tds_read_b128 v[32:35], %0 offset:48\n\tds_read_b128 v[36:39], %0 offset:64\n\tds_read_b128 v[40:43], %0 offset:80\n\tds_read_b128 v[44:47], %0 offset:96\n\tds_read_b128 v[48:51], %0 offset:112\n\ts_waitcnt lgkmcnt(0)\n\t")
                   :: "v"(0) : "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
    }
  }
  const unsigned long long c1 = clock64(), r1 = wall_clock64();
  out[threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + s;
  if (threadIdx.x == 0) { t[0] = c1 - c0; t[1] = r1 - r0; }
}

template <int T>
void run(const char* name, int ops_per_iter, int waves_per_simd) {
  float* out; unsigned long long* t;
  (void)hipMalloc(&out, 4096 * 4); (void)hipMalloc(&t, 16);
  // blocks of 64 threads; waves_per_simd * 4 waves per CU-ish (one block per wave)
  hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves_per_simd), 0, 0, out, t, 1.0f);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k<T>, dim3(1), dim3(64 * waves_per_simd), 0, 0, out, t, 1.0f);
  (void)hipDeviceSynchronize();
  unsigned long long h[2];
  (void)hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
  const double n = double(kIters) * 16 * ops_per_iter;
  std::printf("%-34s waves/blk %d: %7.2f clk/op  %6.3f ns/op\n", name, waves_per_simd, h[0] / n, h[1] * 10.0 / n);
  (void)hipFree(out); (void)hipFree(t);
}

int main() {
  int clk = 0; (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  std::printf("clock rate attr %d kHz\n", clk);
  run<0>("dep v_add_f32", 1, 1);
  run<1>("4 indep v_add_f32", 4, 1);
  run<10>("dep v_fma_f32", 1, 1);
  run<11>("8 indep v_fma_f32", 8, 1);
  run<6>("dep v_pk_fma_f32", 1, 1);
  run<7>("4 indep v_pk_fma_f32", 4, 1);
  run<2>("dep dpp add (+s_nop 1)", 1, 1);
  run<3>("3 interleaved dpp adds", 3, 1);
  run<12>("dep row_bcast15 (+s_nop 1)", 1, 1);
  run<4>("readlane->v_add chain (pair)", 1, 1);
  run<9>("readlane63->v_fma chain (pair)", 1, 1);
  run<8>("4 indep readlanes", 4, 1);
  run<5>("permlane32 swap + add (pair)", 1, 1);
  run<13>("ds_swizzle + wait (pair)", 1, 1);
  run<14>("dep v_add_f64", 1, 1);
  run<15>("dep v_fma_f64", 1, 1);
  run<16>("4 indep v_add_f64", 4, 1);
  run<17>("ds_read_b128 bcast latency (+mov)", 1, 1);
  run<18>("8 ds_read_b128 bcast, one wait", 8, 1);
  run<0>("dep v_add_f32", 1, 4);
  run<0>("dep v_add_f32", 1, 8);
  return 0;
}
