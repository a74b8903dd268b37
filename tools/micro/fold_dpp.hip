// Sequential-fold microbenchmark and bit-exactness check for seq_fold_dpp (csrc/seq_fold.hpp), the
// deterministic sweep's F2jBLAS.ddot-order fold (DSGDforMF.scala:405) with operands brought to row
// 0 by permlane swaps and read through DPP row_newbcast.  Tools only, not part of libmfhip.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I large-scale-recommendation_amd/csrc fold_dpp.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace mfhip {
namespace {
#include "seq_fold.hpp"
}  // namespace
}  // namespace mfhip
using namespace mfhip;

template <typename T, int KPL, bool DPP>
__global__ __launch_bounds__(64) void k_check(const T* x, T* out, int n) {
  __shared__ __attribute__((aligned(16))) T lds[64 * KPL];
  const int lane = threadIdx.x;
  for (int t = 0; t < n; ++t) {
    T p[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) p[c] = x[t * 64 * KPL + 64 * c + lane];
    T s;
    if constexpr (DPP) s = seq_fold_dpp<T, KPL>(p);
    else s = seq_fold<T, KPL>(p, 64 * KPL, lds, lane);
    if (lane == 0) out[t] = s;
  }
}

template <typename T, int KPL, bool DPP>
__global__ __launch_bounds__(64) void k_time(const T* x, T* out, unsigned long long* t, int iters) {
  __shared__ __attribute__((aligned(16))) T lds[64 * KPL];
  const int lane = threadIdx.x;
  T base[KPL];
#pragma unroll
  for (int c = 0; c < KPL; ++c) base[c] = x[64 * c + lane];
  T acc = T(1);
  const unsigned long long c0 = clock64();
  for (int it = 0; it < iters; ++it) {
    T p[KPL];
#pragma unroll
    for (int c = 0; c < KPL; ++c) p[c] = base[c] * acc;  // the next fold depends on this one
    T s;
    if constexpr (DPP) s = seq_fold_dpp<T, KPL>(p);
    else s = seq_fold<T, KPL>(p, 64 * KPL, lds, lane);
    acc = T(1) + s * T(1e-30);
  }
  const unsigned long long c1 = clock64();
  if (lane == 0) { out[0] = acc; t[0] = c1 - c0; }
}

template <typename T, int KPL>
bool check(const char* name) {
  const int n = 64, len = 64 * KPL;
  std::mt19937_64 g(7 + KPL);
  std::uniform_real_distribution<double> u(-1.0, 1.0), ex(-20.0, 20.0);
  std::vector<T> x(static_cast<size_t>(n) * len);
  for (auto& v : x) v = static_cast<T>(u(g) * std::exp2(ex(g)));
  for (int t = 0; t < 4; ++t) x[static_cast<size_t>(t) * len] = T(-0.0);  // -0 first: the sum starts at +0
  T *dx, *dout;
  (void)hipMalloc(&dx, x.size() * sizeof(T));
  (void)hipMalloc(&dout, 2 * n * sizeof(T));
  (void)hipMemcpy(dx, x.data(), x.size() * sizeof(T), hipMemcpyHostToDevice);
  hipLaunchKernelGGL((k_check<T, KPL, true>), dim3(1), dim3(64), 0, 0, dx, dout, n);
  hipLaunchKernelGGL((k_check<T, KPL, false>), dim3(1), dim3(64), 0, 0, dx, dout + n, n);
  std::vector<T> o(2 * n);
  (void)hipMemcpy(o.data(), dout, o.size() * sizeof(T), hipMemcpyDeviceToHost);
  int bad_dpp = 0, bad_lds = 0;
  for (int t = 0; t < n; ++t) {
    volatile T acc = T(0);
    for (int f = 0; f < len; ++f) acc = acc + x[static_cast<size_t>(t) * len + f];
    const T a = acc;
    bad_dpp += std::memcmp(&a, &o[t], sizeof(T)) != 0;
    bad_lds += std::memcmp(&a, &o[n + t], sizeof(T)) != 0;
  }
  std::printf("%-10s k=%3d  folds %d  mismatches: dpp %d  lds %d\n", name, len, n, bad_dpp, bad_lds);
  (void)hipFree(dx);
  (void)hipFree(dout);
  return bad_dpp == 0 && bad_lds == 0;
}

template <typename T, int KPL, bool DPP>
void timeit(const char* name) {
  const int iters = 512;
  std::vector<T> x(64 * KPL);
  for (int i = 0; i < 64 * KPL; ++i) x[i] = static_cast<T>(1.0 + 1e-3 * i);
  T *dx, *dout;
  unsigned long long* dt;
  (void)hipMalloc(&dx, x.size() * sizeof(T));
  (void)hipMalloc(&dout, sizeof(T));
  (void)hipMalloc(&dt, 8);
  (void)hipMemcpy(dx, x.data(), x.size() * sizeof(T), hipMemcpyHostToDevice);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL((k_time<T, KPL, DPP>), dim3(1), dim3(64), 0, 0, dx, dout, dt, iters);
    (void)hipDeviceSynchronize();
  }
  unsigned long long h = 0;
  (void)hipMemcpy(&h, dt, 8, hipMemcpyDeviceToHost);
  std::printf("%-22s k=%3d  %8.1f clk per chained fold  %5.2f clk per add\n", name, 64 * KPL, double(h) / iters,
              double(h) / iters / (64 * KPL));
  (void)hipFree(dx);
  (void)hipFree(dout);
  (void)hipFree(dt);
}

int main() {
  bool ok = true;
  ok &= check<double, 1>("f64");
  ok &= check<double, 2>("f64");
  ok &= check<double, 4>("f64");
  ok &= check<float, 1>("f32");
  ok &= check<float, 2>("f32");
  ok &= check<float, 4>("f32");
  timeit<double, 2, false>("f64 lds (seq_fold)");
  timeit<double, 2, true>("f64 dpp (seq_fold_dpp)");
  timeit<double, 1, false>("f64 lds (seq_fold)");
  timeit<double, 1, true>("f64 dpp (seq_fold_dpp)");
  timeit<double, 4, false>("f64 lds (seq_fold)");
  timeit<double, 4, true>("f64 dpp (seq_fold_dpp)");
  timeit<float, 2, false>("f32 lds (seq_fold)");
  timeit<float, 2, true>("f32 dpp (seq_fold_dpp)");
  std::printf(ok ? "ALL BITWISE OK\n" : "MISMATCH\n");
  return ok ? 0 : 1;
}
