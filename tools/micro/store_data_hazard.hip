// Is a 16-B buffer store's data safe from a VALU write of its data VGPRs issued right after it,
// when the store takes its offset from an SGPR (soffset)?
//
// The gfx9-family hazard table asks for 1 wait state between a >64-bit VMEM store and a VALU
// write of its data VGPRs, and exempts BUFFER_STORE with an SGPR offset; LLVM's hazard recognizer
// (GCNHazardRecognizer::createsVALUHazard) follows the exemption and pads only stores whose
// soffset is not a register.  The round-4 k = 256 lean single-run sweep (MFHIP_EXP_K256_LEAN)
// was the only built code with such a write within 1-2 instructions of a buffer_store_dwordx4
// (tools/isa_store_hazard.py), and the only one that did not repeat itself.
//
// Each wave stores ITER 16-B records per lane (a distinct address each), then overwrites the
// store's data VGPRs with 0xDEADBEEF after N wait states (s_nop N-1; N = 0: the next instruction).
// The host checks every stored word.  Modes:
//   sgpr   buffer_store_dwordx4 v[40:43], voff, rsrc, s_off offen    (the sweep's form)
//   imm0   buffer_store_dwordx4 v[40:43], voff+off, rsrc, 0 offen    (the documented hazard)
//   x2     buffer_store_dwordx2 v[40:41], voff, rsrc, s_off offen    (<= 64 bits: no hazard listed)
//   ldoob  the sgpr store, then a buffer_load_dwordx4 INTO its data VGPRs from an out-of-range
//          offset (returns zeros at once) -- a load, not a VALU, overwriting the store data
//   ldin   the same with an in-range load of a region filled with 0xEF bytes
// each plain and with sc1 (the sweep's user-row policy), on 1 wave (idle chip) and on 4096 waves.
//
//   hipcc -O3 --offload-arch=gfx950 -o store_data_hazard store_data_hazard.hip && ./store_data_hazard
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

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 256;
constexpr uint32_t kBad = 0xDEADBEEFu;

#define NOP0 ""
#define NOP1 "s_nop 0\n\t"
#define NOP2 "s_nop 1\n\t"
#define NOP5 "s_nop 4\n\t"
#define FILL                   \
  "v_mov_b32 v40, %[a]\n\t"    \
  "v_mov_b32 v41, %[b]\n\t"    \
  "v_mov_b32 v42, %[c]\n\t"    \
  "v_mov_b32 v43, %[d]\n\t"    \
  "s_nop 4\n\t"
#define SMASH                  \
  "v_mov_b32 v40, %[bad]\n\t"  \
  "v_mov_b32 v41, %[bad]\n\t"  \
  "v_mov_b32 v42, %[bad]\n\t"  \
  "v_mov_b32 v43, %[bad]\n\t"  \
  "s_nop 4\n\t"
#define LDOOB                                                          \
  "buffer_load_dwordx4 v[40:43], %[vo], %[rs], %[oob] offen\n\t"       \
  "s_waitcnt vmcnt(0)\n\t"
#define LDIN                                                           \
  "buffer_load_dwordx4 v[40:43], %[vo], %[rs], %[tail] offen\n\t"      \
  "s_waitcnt vmcnt(0)\n\t"
#define OPS [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [bad] "v"(kBad), [vo] "v"(vo), [rs] "s"(rs), [so] "s"(so), \
    [oob] "s"(0xFFFFF000u), [tail] "s"(tail)
#define CLOB "v40", "v41", "v42", "v43", "memory"

// MODE 0 = sgpr, 1 = imm0, 2 = x2; N = wait states between the store and the first overwrite; SC1
constexpr uint32_t kTailWords = 16384;  // 64 KB of 0xEF bytes after the records (ldin)
constexpr uint32_t kTailPattern = 0xEFEFEFEFu;

template <int MODE, int N, bool SC1>
__global__ __launch_bounds__(64) void k_store(uint32_t* out, uint32_t tail) {
  const uint32_t lane = threadIdx.x, wave = blockIdx.x;
  const uint64_t base = reinterpret_cast<uint64_t>(out);
  const u4 rs = u4{static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(base))),
                   static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(base >> 32))) & 0xFFFFu,
                   0xFFFFF000u, 0x00020000u};
  for (int i = 0; i < ITER; ++i) {
    const uint32_t a = i, b = lane, c = wave, d = 0x1234u;
    // record (wave, i): 64 lanes x 16 B
    const uint32_t rec = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>((wave * ITER + i) * 1024u)));
    uint32_t vo = lane * 16u;
    uint32_t so = rec;
    if constexpr (MODE == 1) { vo += rec; so = 0; }
#define BODY(STORE, NOPS)                                                           \
  if constexpr (MODE == 3) asm volatile(FILL STORE NOPS LDOOB ::OPS : CLOB);        \
  else if constexpr (MODE == 4) asm volatile(FILL STORE NOPS LDIN ::OPS : CLOB);    \
  else asm volatile(FILL STORE NOPS SMASH ::OPS : CLOB)
#define SEL(STORE)                    \
  if constexpr (N == 0) BODY(STORE, NOP0); \
  else if constexpr (N == 1) BODY(STORE, NOP1); \
  else if constexpr (N == 2) BODY(STORE, NOP2); \
  else BODY(STORE, NOP5);
    if constexpr ((MODE == 0 || MODE >= 3) && !SC1) { SEL("buffer_store_dwordx4 v[40:43], %[vo], %[rs], %[so] offen\n\t") }
    if constexpr ((MODE == 0 || MODE >= 3) && SC1) { SEL("buffer_store_dwordx4 v[40:43], %[vo], %[rs], %[so] offen sc1\n\t") }
    if constexpr (MODE == 1 && !SC1) { SEL("buffer_store_dwordx4 v[40:43], %[vo], %[rs], 0 offen\n\t") }
    if constexpr (MODE == 1 && SC1) { SEL("buffer_store_dwordx4 v[40:43], %[vo], %[rs], 0 offen sc1\n\t") }
    if constexpr (MODE == 2 && !SC1) { SEL("buffer_store_dwordx2 v[40:41], %[vo], %[rs], %[so] offen\n\t") }
    if constexpr (MODE == 2 && SC1) { SEL("buffer_store_dwordx2 v[40:41], %[vo], %[rs], %[so] offen sc1\n\t") }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

template <int MODE, int N, bool SC1>
void run(const char* mode, uint32_t* d, std::vector<uint32_t>& h, int waves) {
  const size_t words = static_cast<size_t>(waves) * ITER * 256;
  const size_t tail = static_cast<size_t>(4096) * ITER * 256;  // the 0xEF region (ldin)
  CK(hipMemset(d, 0, words * 4));
  CK(hipMemset(d + tail, 0xEF, kTailWords * 4));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((k_store<MODE, N, SC1>), dim3(waves), dim3(64), 0, 0, d, static_cast<uint32_t>(tail * 4));
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h.data(), d, words * 4, hipMemcpyDeviceToHost));
  const int nw = MODE == 2 ? 2 : 4;
  size_t bad = 0, smashed = 0, recs_bad = 0;
  for (int w = 0; w < waves; ++w)
    for (int i = 0; i < ITER; ++i)
      for (int l = 0; l < 64; ++l) {
        const uint32_t* p = h.data() + (static_cast<size_t>(w) * ITER + i) * 256 + l * 4;
        const uint32_t want[4] = {static_cast<uint32_t>(i), static_cast<uint32_t>(l), static_cast<uint32_t>(w), 0x1234u};
        bool rb = false;
        for (int j = 0; j < nw; ++j)
          if (p[j] != want[j]) {
            ++bad;
            rb = true;
            smashed += p[j] == kBad || p[j] == kTailPattern || p[j] == 0u;
          }
        recs_bad += rb;
      }
  std::printf("%-5s sc1=%d waves=%4d wait_states=%d: %zu of %zu lane records wrong, %zu words wrong (%zu = the overwriting value)\n",
              mode, SC1 ? 1 : 0, waves, N, recs_bad, static_cast<size_t>(waves) * ITER * 64, bad, smashed);
}

template <int MODE, bool SC1>
void sweep(const char* mode, uint32_t* d, std::vector<uint32_t>& h) {
  for (int waves : {1, 4096}) {
    run<MODE, 0, SC1>(mode, d, h, waves);
    run<MODE, 1, SC1>(mode, d, h, waves);
    run<MODE, 2, SC1>(mode, d, h, waves);
    run<MODE, 5, SC1>(mode, d, h, waves);
  }
}

int main() {
  const size_t words = static_cast<size_t>(4096) * ITER * 256 + kTailWords;
  uint32_t* d = nullptr;
  CK(hipMalloc(&d, words * 4));
  std::vector<uint32_t> h(words);
  sweep<0, false>("sgpr", d, h);
  sweep<0, true>("sgpr", d, h);
  sweep<1, false>("imm0", d, h);
  sweep<1, true>("imm0", d, h);
  sweep<2, false>("x2", d, h);
  sweep<2, true>("x2", d, h);
  sweep<3, true>("ldoob", d, h);
  sweep<4, true>("ldin", d, h);
  CK(hipFree(d));
  return 0;
}
