// What a buffer load costs the CU's vector-memory path when it moves nothing: in-range loads (L2/L1
// hits), out-of-range offsets (the systolic sweep's "no load"), and loads issued with EXEC = 0.
// 4 waves per CU (one per SIMD), every CU busy; each wave issues 32 independent loads, then waits.
// Build: hipcc -O3 --offload-arch=gfx950 vmem_cost.hip -o vmem_cost
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>  // 0: in range, 1: out of range, 2: EXEC = 0
__global__ __launch_bounds__(256) void k_vmem(const float* __restrict__ buf, float* __restrict__ out, int rounds) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), 0, 1u << 20, 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t voff = (MODE == 1 ? 0xFFFFF000u : 0u) + lane * 4u;
  float acc = 0.f;
  for (int r = 0; r < rounds; r += 4) {  // 32 loads in flight, then one wait: the path's throughput
    float d[32];
    if constexpr (MODE == 2) {
      asm volatile("s_mov_b64 exec, 0\n"
          "buffer_load_dword %0, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %1, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %2, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %3, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %4, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %5, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %6, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %7, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %8, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %9, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %10, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %11, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %12, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %13, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %14, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %15, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %16, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %17, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %18, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %19, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %20, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %21, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %22, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %23, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %24, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %25, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %26, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %27, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %28, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %29, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %30, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %31, %32, %33, 0 offen offset:1792\n"
          "s_mov_b64 exec, -1\n"
          "s_waitcnt vmcnt(0)\n"
          : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]), "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10]), "=&v"(d[11]), "=&v"(d[12]), "=&v"(d[13]), "=&v"(d[14]), "=&v"(d[15]), "=&v"(d[16]), "=&v"(d[17]), "=&v"(d[18]), "=&v"(d[19]), "=&v"(d[20]), "=&v"(d[21]), "=&v"(d[22]), "=&v"(d[23]), "=&v"(d[24]), "=&v"(d[25]), "=&v"(d[26]), "=&v"(d[27]), "=&v"(d[28]), "=&v"(d[29]), "=&v"(d[30]), "=&v"(d[31])
          : "v"(voff), "s"(rs));
    } else {
      asm volatile("buffer_load_dword %0, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %1, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %2, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %3, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %4, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %5, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %6, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %7, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %8, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %9, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %10, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %11, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %12, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %13, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %14, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %15, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %16, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %17, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %18, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %19, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %20, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %21, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %22, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %23, %32, %33, 0 offen offset:1792\n"
          "buffer_load_dword %24, %32, %33, 0 offen offset:0\n"
          "buffer_load_dword %25, %32, %33, 0 offen offset:256\n"
          "buffer_load_dword %26, %32, %33, 0 offen offset:512\n"
          "buffer_load_dword %27, %32, %33, 0 offen offset:768\n"
          "buffer_load_dword %28, %32, %33, 0 offen offset:1024\n"
          "buffer_load_dword %29, %32, %33, 0 offen offset:1280\n"
          "buffer_load_dword %30, %32, %33, 0 offen offset:1536\n"
          "buffer_load_dword %31, %32, %33, 0 offen offset:1792\n"
          "s_waitcnt vmcnt(0)\n"
          : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]), "=&v"(d[8]), "=&v"(d[9]), "=&v"(d[10]), "=&v"(d[11]), "=&v"(d[12]), "=&v"(d[13]), "=&v"(d[14]), "=&v"(d[15]), "=&v"(d[16]), "=&v"(d[17]), "=&v"(d[18]), "=&v"(d[19]), "=&v"(d[20]), "=&v"(d[21]), "=&v"(d[22]), "=&v"(d[23]), "=&v"(d[24]), "=&v"(d[25]), "=&v"(d[26]), "=&v"(d[27]), "=&v"(d[28]), "=&v"(d[29]), "=&v"(d[30]), "=&v"(d[31])
          : "v"(voff), "s"(rs));
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) acc += d[i];
  }
  if (acc == 12345.f) out[threadIdx.x] = acc;  // keeps the loads alive
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float *buf = nullptr, *out = nullptr;
  hipMalloc(&buf, 1 << 20);
  hipMemset(buf, 0, 1 << 20);
  hipMalloc(&out, 1024);
  const int rounds = 20000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[3] = {"in range (L1/L2 hits)", "out of range offset", "EXEC = 0"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
      hipEventRecord(a);
      if (m == 0) k_vmem<0><<<cus, 256>>>(buf, out, rounds);
      if (m == 1) k_vmem<1><<<cus, 256>>>(buf, out, rounds);
      if (m == 2) k_vmem<2><<<cus, 256>>>(buf, out, rounds);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double per = ms * 1e6 / rounds / 8;  // ns per load instruction per wave (4 waves per CU)
      std::printf("%-24s %8.3f ms  %6.2f ns per load per wave  (%5.1f shader cycles at 2.4 GHz)\n", names[m], ms, per,
                  per * 2.4);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
