// Does a synchronous hipMemset / hipMemcpy (legacy null stream) finish before it returns, and is a
// kernel on a hipStreamNonBlocking stream ordered after it?  (mfhip issues prepare-time zeroing
// with hipMemset and sweeps on non-blocking streams.)
//
//   hipcc -O2 --offload-arch=gfx950 -o memset_order memset_order.hip && ./memset_order
#include <hip/hip_runtime.h>

#include <chrono>
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

// reads the last word of the buffer, and how many of 64 sampled words are not zero
__global__ void probe(const unsigned* d, size_t n, unsigned* out) {
  if (threadIdx.x == 0) {
    out[0] = d[n - 1];
    unsigned bad = 0;
    for (int j = 0; j < 64; ++j) bad += d[(n / 64) * j + (n / 64) - 1] != 0u;
    out[1] = bad;
  }
}

int main() {
  const size_t bytes = size_t{4} << 30, n = bytes / 4;
  unsigned *d = nullptr, *out = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(d, 0xFF, bytes));
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    CK(hipMemset(d, 0, bytes));
    auto t1 = std::chrono::steady_clock::now();
    probe<<<1, 64, 0, st>>>(d, n, out);
    CK(hipStreamSynchronize(st));
    unsigned h[2];
    CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
    std::printf("hipMemset 4 GiB returned after %.3f ms; a non-blocking-stream kernel launched right after saw "
                "last word %08x, %u of 64 sampled words not yet zero\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(), h[0], h[1]);
  }
  // pageable H2D
  std::vector<unsigned> host(n / 4, 0u);
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipMemset(d, 0xFF, bytes));
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    CK(hipMemcpy(d + 3 * (n / 4), host.data(), bytes / 4, hipMemcpyHostToDevice));
    auto t1 = std::chrono::steady_clock::now();
    probe<<<1, 64, 0, st>>>(d, n, out);
    CK(hipStreamSynchronize(st));
    unsigned h[2];
    CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
    std::printf("hipMemcpy 1 GiB pageable H2D returned after %.3f ms; the kernel saw last word %08x\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(), h[0]);
  }
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
