// Is a CU's vector-memory path paced by lanes (addresses) or by bytes?  Four waves per CU (one
// per SIMD, as in the systolic sweep) each stream 512-B row reads from L2-resident rows in three
// shapes of the same bytes: 64 lanes x 8 B (dwordx2, the k = 128 sweep's rows), 32 lanes x 16 B
// (dwordx4, half the lanes masked off) and 64 lanes x 16 B (two rows per instruction, 1 KB).
// Reports ns per 512 B per wave and the CU's rate (24 loads in flight per wave, 8 waves per CU).  Rows are random within a 16-MB table (L2 / MALL resident).
//
//   hipcc -O3 --offload-arch=gfx950 -o ta_width ta_width.hip && ./ta_width
#include <hip/hip_runtime.h>

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

constexpr int kIters = 4096;
constexpr int kDepth = 24;  // loads in flight per wave (enough to cover the latency: a throughput test)

// MODE 0: 64 lanes x 8 B; MODE 1: 32 lanes x 16 B (lanes 32-63 idle); MODE 2: 64 lanes x 16 B (two rows)
template <int MODE>
__global__ __launch_bounds__(256) void k_rows(const char* __restrict__ base, const unsigned* __restrict__ rows,
                                              unsigned nrows, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, 0x7FFFFFF0u, 0x00020000);
  float acc = 0.f;
  for (int it = 0; it < kIters; it += kDepth) {
    float part[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      const unsigned r = rows[(wave * 7919u + (it + d) * 104729u) % nrows];
      const unsigned off = r * 512u;
      if constexpr (MODE == 0) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8u, off, 0);
        part[d] = __uint_as_float(x[0]) + __uint_as_float(x[1]);
      } else if constexpr (MODE == 1) {
        float v = 0.f;
        if (lane < 32) {
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16u, off, 0);
          v = __uint_as_float(x[0]) + __uint_as_float(x[1]) + __uint_as_float(x[2]) + __uint_as_float(x[3]);
        }
        part[d] = v;
      } else {
        // two rows: lanes 0-31 row r, lanes 32-63 row r+1 (the same bytes per row, half the instructions)
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane & 31) * 16u + (lane >> 5) * 512u, off, 0);
        part[d] = __uint_as_float(x[0]) + __uint_as_float(x[1]) + __uint_as_float(x[2]) + __uint_as_float(x[3]);
      }
    }
#pragma unroll
    for (int d = 0; d < kDepth; ++d) acc += part[d];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const unsigned nrows = (16u << 20) / 512u;  // 16 MB of rows
  char* base;
  unsigned* rows;
  float* out;
  CK(hipMalloc(&base, (size_t)(nrows + 2) * 512));
  CK(hipMemset(base, 0, (size_t)(nrows + 2) * 512));
  std::vector<unsigned> h(nrows);
  for (unsigned i = 0; i < nrows; ++i) h[i] = (i * 2654435761u) % nrows;
  CK(hipMalloc(&rows, nrows * 4));
  CK(hipMemcpy(rows, h.data(), nrows * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = 2 * cus;  // two 256-thread blocks (8 waves) per CU
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[3] = {"64 lanes x 8 B (dwordx2)", "32 lanes x 16 B (dwordx4, half the lanes)",
                          "64 lanes x 16 B (two rows per dwordx4)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      CK(hipEventRecord(a));
      if (m == 0) k_rows<0><<<blocks, 256>>>(base, rows, nrows, out);
      if (m == 1) k_rows<1><<<blocks, 256>>>(base, rows, nrows, out);
      if (m == 2) k_rows<2><<<blocks, 256>>>(base, rows, nrows, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double rows_per_wave = (m == 2 ? 2.0 : 1.0) * kIters;
      const double rows_total = rows_per_wave * blocks * 4;
      std::printf("%-44s %8.3f ms  %6.2f ns per 512-B row per wave (8 waves per CU, %d CUs); %.2f TB/s of rows, "
                  "%.2f ns per instruction per CU\n", names[m], ms, ms * 1e6 / rows_per_wave, cus,
                  rows_total * 512.0 / (ms * 1e-3) / 1e12, ms * 1e6 / (kIters * 8.0));
    }
  return 0;
}
