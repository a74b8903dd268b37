// Known-good and known-bad machine code for tests/test_isa.py: proves that tools/isa_check.py
// finds what it is meant to find.  Built into a throwaway shared library by the test (CPU only,
// never launched).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7FFFFFFF, 0x00020000);
}

// A row store, one load after it, then vmcnt(N) and the flag store.  N = 1: the load may still
// fly, the store has landed (good).  N = 2: the store may still be in flight (bad).
template <int N>
__device__ __forceinline__ void handoff(float* rows, const float* src, int32_t* flag, float* out) {
  const __amdgpu_buffer_rsrc_t r = rsrc(rows), s = rsrc(const_cast<float*>(src));
  const uint32_t v = threadIdx.x * 4u;
  const uint32_t off = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x))) * 256u;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(1.0f + static_cast<float>(threadIdx.x)), r, v, off, 16);
  const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(s, v, off, 16);
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  out[threadIdx.x] = __uint_as_float(x);
}

}  // namespace

__global__ void k_fixture_good_handoff(float* rows, const float* src, int32_t* flag, float* out) {
  handoff<1>(rows, src, flag, out);
}
__global__ void k_fixture_bad_handoff(float* rows, const float* src, int32_t* flag, float* out) {
  handoff<2>(rows, src, flag, out);
}

// A 16-B buffer store with an SGPR offset whose data VGPRs a VALU overwrites at once (bad), or
// after two wait states (good).
#define MF_FIX_STORE(NOPS)                                                                  \
  asm volatile("v_mov_b32 v40, %0\n\tv_mov_b32 v41, %0\n\tv_mov_b32 v42, %0\n\tv_mov_b32 v43, %0\n\t" \
               "s_nop 4\n\t"                                                                \
               "buffer_store_dwordx4 v[40:43], %1, %2, %3 offen\n\t" NOPS                   \
               "v_mov_b32 v40, 0\n\tv_mov_b32 v41, 0\n\tv_mov_b32 v42, 0\n\tv_mov_b32 v43, 0\n\t" ::"v"(1u), \
               "v"(threadIdx.x * 16u), "s"(r), "s"(off)                                      \
               : "v40", "v41", "v42", "v43", "memory")

__global__ void k_fixture_bad_store(float* rows) {
  const __amdgpu_buffer_rsrc_t r = rsrc(rows);
  const uint32_t off = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x))) * 1024u;
  MF_FIX_STORE("");
}
__global__ void k_fixture_good_store(float* rows) {
  const __amdgpu_buffer_rsrc_t r = rsrc(rows);
  const uint32_t off = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x))) * 1024u;
  MF_FIX_STORE("s_nop 1\n\t");
}
