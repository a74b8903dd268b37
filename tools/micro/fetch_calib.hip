// What FETCH_SIZE / WRITE_SIZE (rocprofv3) count for the sweeps' row accesses: 512-B rows (k = 128
// f32) read as 64 lanes x 8 B (buffer_load_dwordx2, the pair sweep's user-row shape) and written the
// same way, at rows drawn at random from a slab far larger than the 256-MiB MALL (misses go to HBM)
// and from a slab that fits it (hits).  Each kernel moves a known number of bytes; the PMC passes
// (one counter per pass) are compared with it by tools/pmc_calib.py.  MI355X_MICROARCH.md calibrates
// FETCH_SIZE at 1/2 of the bytes for 16-B/lane streaming reads only; this checks the 8-B/lane,
// random-row case the roofline summaries use, with plain and sc1 policies.
//
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip && ./fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ;  rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
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

constexpr int kRowBytes = 512;
constexpr int kPerWave = 256;  // rows per wave
constexpr int kDepth = 16;     // loads in flight per wave

// MODE 0: read (policy POL), MODE 1: write (policy POL), MODE 2: read + write back (the sweep's user rows)
template <int MODE, int POL>
__global__ __launch_bounds__(256) void k_rows(char* __restrict__ base, uint32_t slab_rows, uint32_t seed,
                                              float* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0xFFFFF000u, 0x00020000);
  float acc = 0.f;
  uint32_t h = wave * 2654435761u ^ seed;
  for (int it = 0; it < kPerWave; it += kDepth) {
    uint32_t off[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      h = h * 1664525u + 1013904223u;
      off[d] = (h % slab_rows) * kRowBytes;
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        using u2 = uint32_t __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u2{wave, lane}, rs, lane * 8u, off[d], POL);
      }
    } else {
      uint32_t x[kDepth][2];
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8u, off[d], POL);
        x[d][0] = v[0];
        x[d][1] = v[1];
      }
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        acc += __uint_as_float(x[d][0]) + __uint_as_float(x[d][1]);
        if constexpr (MODE == 2) {
          using u2 = uint32_t __attribute__((ext_vector_type(2)));
          __builtin_amdgcn_raw_buffer_store_b64(u2{x[d][0] + 1u, x[d][1]}, rs, lane * 8u, off[d], POL);
        }
      }
    }
  }
  if (acc == 12345.f) sink[wave] = acc;  // keeps the loads
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t big = 3ull << 30;  // 3 GiB slab: random rows miss the 256-MiB MALL
  const uint64_t small = 64ull << 20;  // 64 MiB: resident in the MALL after the first pass
  char* slab = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&slab, big));
  CK(hipMemset(slab, 0, big));
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU
  CK(hipMalloc(&sink, static_cast<size_t>(blocks) * 4 * 4));
  const double rows = static_cast<double>(blocks) * 4 * kPerWave;
  const double bytes = rows * kRowBytes;
  CK(hipDeviceSynchronize());
  struct Case {
    const char* name;
    void (*k)(char*, uint32_t, uint32_t, float*);
    uint64_t slab;
    double rd, wr;
  } cases[] = {
      {"read_plain_3GiB", k_rows<0, 0>, big, bytes, 0},
      {"read_sc1_3GiB", k_rows<0, 16>, big, bytes, 0},
      {"read_plain_64MiB_warm", k_rows<0, 0>, small, bytes, 0},
      {"write_plain_3GiB", k_rows<1, 0>, big, 0, bytes},
      {"write_sc1_3GiB", k_rows<1, 16>, big, 0, bytes},
      {"rmw_sc1_3GiB", k_rows<2, 16>, big, bytes, bytes},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // dispatch order = the order rocprofv3 lists them (tools/pmc_calib.py pairs them by index)
  std::printf("case,dispatch,rows,read_bytes,write_bytes,ms,GBps\n");
  int disp = 0;
  for (const Case& c : cases) {
    const uint32_t srows = static_cast<uint32_t>(c.slab / kRowBytes);
    if (c.slab == small) {  // warm the MALL with the same rows first (its own dispatch)
      hipLaunchKernelGGL(c.k, dim3(blocks), dim3(256), 0, 0, slab, srows, 7u, sink);
      CK(hipDeviceSynchronize());
      std::printf("%s_warmup,%d,%.0f,%.0f,%.0f,0,0\n", c.name, disp++, rows, c.rd, c.wr);
    }
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(c.k, dim3(blocks), dim3(256), 0, 0, slab, srows, 7u, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%s,%d,%.0f,%.0f,%.0f,%.4f,%.1f\n", c.name, disp++, rows, c.rd, c.wr, ms,
                (c.rd + c.wr) / (ms * 1e-3) / 1e9);
  }
  CK(hipFree(slab));
  CK(hipFree(sink));
  return 0;
}
