// Does independent work issued between the steps of the deterministic sweep's sequential f64
// fold (128 dependent v_fmac_f64_dpp row_newbcast, csrc/seq_fold.hpp) cost issue time, or does it
// hide in the fold's latency?  One wave, shader cycles per 128-step fold (s_memtime), with F
// filler instructions of one kind after every fold step.  Tools only, not part of libmfhip.
// Build: hipcc -O3 --offload-arch=gfx950 fold_fill.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define STEP "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define R128(x) R16(x) R16(x) R16(x) R16(x) R16(x) R16(x) R16(x) R16(x)

// fillers write registers nothing in the chain reads (%3, %4: f64 scratch; %5 SGPR scratch; %6, %7
// f32 scratch)
#define F_NONE ""
#define F_VMULF64 "v_mul_f64 %3, %3, %4\n\t"
#define F_VMULF64X2 "v_mul_f64 %3, %3, %4\n\tv_mul_f64 %4, %4, %3\n\t"
#define F_VMULF32 "v_mul_f32 %6, %6, %7\n\t"
#define F_SALU "s_movk_i32 %5, 0x1234\n\t"  // (no SCC write: the loop branch reads SCC)
#define F_SALU2 "s_movk_i32 %5, 0x1234\n\ts_mov_b32 %5, %5\n\t"
#define F_SNOP "s_nop 0\n\t"
#define F_DSW "ds_write_b64 %8, %3\n\t"
#define F_GST "global_store_dwordx2 %9, %3, off\n\t"
#define F_GLD "global_load_dwordx2 %4, %9, off\n\t"
#define F_READLANE "v_readlane_b32 %5, %7, 5\n\t"
#define F_VMOV "v_mov_b32 %6, %7\n\t"

#define KERNEL(NAME, FILL)                                                                           \
  __global__ __launch_bounds__(64) void NAME(const double* x, double* out, unsigned long long* t,    \
                                             int iters) {                                            \
    const int lane = threadIdx.x;                                                                    \
    double v = x[lane], acc = 0.0, s1 = x[lane + 64], s2 = x[lane + 128];                           \
    double one = 1.0;                                                                                \
    unsigned sg = 0;                                                                                 \
    float f1 = float(x[lane + 1]), f2 = float(x[lane + 2]);                                          \
    __shared__ double lds[64];                                                                       \
    const unsigned ldsa = static_cast<unsigned>(reinterpret_cast<uintptr_t>(&lds[lane]));            \
    double* gaddr = out + 8 + lane;                                                                  \
    const unsigned long long c0 = clock64();                                                         \
    for (int it = 0; it < iters; ++it) {                                                             \
      asm volatile("s_nop 1\n\t" R128(STEP FILL) "s_waitcnt vmcnt(0)\n\t"                                                     \
                   : "+v"(acc), "+v"(v), "+v"(one), "+v"(s1), "+v"(s2), "+s"(sg), "+v"(f1), "+v"(f2) : "v"(ldsa), "v"(gaddr));                  \
    }                                                                                                \
    const unsigned long long c1 = clock64();                                                         \
    if (lane == 0) {                                                                                 \
      out[0] = acc + s1 + s2 + sg + f1 + f2;                                                                   \
      t[0] = c1 - c0;                                                                                \
    }                                                                                                \
  }

KERNEL(k_none, F_NONE)
KERNEL(k_vmulf64, F_VMULF64)
KERNEL(k_vmulf64x2, F_VMULF64X2)
KERNEL(k_vmulf32, F_VMULF32)
KERNEL(k_salu, F_SALU)
KERNEL(k_salu2, F_SALU2)
KERNEL(k_readlane, F_READLANE)
KERNEL(k_vmov, F_VMOV)
KERNEL(k_snop, F_SNOP)
KERNEL(k_dsw, F_DSW)
KERNEL(k_gst, F_GST)
KERNEL(k_gld, F_GLD)

// issue rate of the fillers alone (128 independent ones per iteration, no fold)
#define ALONE(NAME, FILL)                                                                            \
  __global__ __launch_bounds__(64) void NAME(const double* x, double* out, unsigned long long* t,    \
                                             int iters) {                                            \
    const int lane = threadIdx.x;                                                                    \
    double v = x[lane], acc = 0.0, s1 = x[lane + 64], s2 = x[lane + 128];                           \
    double one = 1.0;                                                                                \
    unsigned sg = 0;                                                                                 \
    float f1 = float(x[lane + 1]), f2 = float(x[lane + 2]);                                          \
    __shared__ double lds[64];                                                                       \
    const unsigned ldsa = static_cast<unsigned>(reinterpret_cast<uintptr_t>(&lds[lane]));            \
    double* gaddr = out + 8 + lane;                                                                  \
    const unsigned long long c0 = clock64();                                                         \
    for (int it = 0; it < iters; ++it) {                                                             \
      asm volatile(R128(FILL) : "+v"(acc), "+v"(v), "+v"(one), "+v"(s1), "+v"(s2), "+s"(sg), "+v"(f1), "+v"(f2) : "v"(ldsa), "v"(gaddr));        \
    }                                                                                                \
    const unsigned long long c1 = clock64();                                                         \
    if (lane == 0) {                                                                                 \
      out[0] = acc + s1 + s2 + sg + f1 + f2;                                                                   \
      t[0] = c1 - c0;                                                                                \
    }                                                                                                \
  }
ALONE(a_vmulf64, F_VMULF64)
ALONE(a_vmulf32, F_VMULF32)
ALONE(a_salu, F_SALU)
ALONE(a_readlane, F_READLANE)
ALONE(a_salu2, F_SALU2)

typedef void (*K)(const double*, double*, unsigned long long*, int);

int main() {
  double *x, *out;
  unsigned long long* t;
  hipMalloc(&x, 192 * 8);
  hipMalloc(&out, 1024 * 8);
  hipMalloc(&t, 8);
  double h[192];
  for (int i = 0; i < 192; ++i) h[i] = 1.0 + i * 1e-3;
  hipMemcpy(x, h, sizeof h, hipMemcpyHostToDevice);
  struct {
    const char* name;
    K k;
    int fill;  // filler instructions per fold step
  } ks[] = {{"fold, no filler", k_none, 0},
            {"fold + 1 v_mul_f64 per step", k_vmulf64, 1},
            {"fold + 2 v_mul_f64 per step", k_vmulf64x2, 2},
            {"fold + 1 v_mul_f32 per step", k_vmulf32, 1},
            {"fold + 1 s_movk per step", k_salu, 1},
            {"fold + 2 s_mov per step", k_salu2, 2},
            {"fold + 1 v_readlane per step", k_readlane, 1},
            {"fold + 1 v_mov_b32 per step", k_vmov, 1},
            {"fold + 1 s_nop 0 per step", k_snop, 1},
            {"fold + 1 ds_write_b64 per step", k_dsw, 1},
            {"fold + 1 global_store_dwordx2 per step", k_gst, 1},
            {"fold + 1 global_load_dwordx2 per step", k_gld, 1},
            {"alone: 128 v_mul_f64", a_vmulf64, 0},
            {"alone: 128 v_mul_f32", a_vmulf32, 0},
            {"alone: 128 s_movk", a_salu, 0},
            {"alone: 128 v_readlane", a_readlane, 0},
            {"alone: 256 s_mov", a_salu2, 0}};
  const int iters = 2000;
  for (auto& e : ks) {
    unsigned long long c = 0;
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(e.k, dim3(1), dim3(64), 0, 0, x, out, t, iters);
      hipDeviceSynchronize();
      hipMemcpy(&c, t, 8, hipMemcpyDeviceToHost);
    }
    std::printf("%-32s %8.1f cycles per 128 steps  %6.2f per step\n", e.name, double(c) / iters,
                double(c) / iters / 128);
  }
  return 0;
}
