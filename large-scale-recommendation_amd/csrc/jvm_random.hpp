// jvm_random.hpp -- bit-exact java.util.Random (JDK 8 spec) and scala.util.Random.shuffle
// (Scala 2.11), the two RNGs the reference's DSGD uses:
//   block ids      DSGDforMF.scala:531-533   new Random(id ^ seed).nextInt(numBlocks)
//   initial rows   DSGDforMF.scala:548-549   k x nextDouble of a fresh Random(id ^ seed)
//   sweep order    DSGDforMF.scala:392-393   Random(iteration ^ ratingBlockId ^ seed).shuffle
//   online init    core/FactorInitializer.scala:33   new Random(id)
#pragma once
#include <cstdint>
#include <cmath>

namespace mfhip {

class JavaRandom {
 public:
  explicit JavaRandom(int64_t seed) : s_((static_cast<uint64_t>(seed) ^ kMult) & kMask) {}

  int32_t next(int bits) {
    s_ = (s_ * kMult + 0xBULL) & kMask;
    return static_cast<int32_t>(static_cast<uint32_t>(s_ >> (48 - bits)));
  }

  // nextInt(bound): power-of-two path, else the int32 rejection loop of JDK 8.
  int32_t nextInt(int32_t bound) {
    int32_t r = next(31);
    const int32_t m = bound - 1;
    if ((bound & m) == 0) return static_cast<int32_t>((static_cast<int64_t>(bound) * r) >> 31);
    for (int32_t u = r;; u = next(31)) {
      r = u % bound;
      const int32_t guard = static_cast<int32_t>(static_cast<uint32_t>(u) - static_cast<uint32_t>(r) +
                                                 static_cast<uint32_t>(m));
      if (guard >= 0) return r;
    }
  }

  double nextDouble() {
    const int64_t hi = next(26);
    const int64_t lo = next(27);
    return static_cast<double>((hi << 27) + lo) * 0x1.0p-53;
  }

 private:
  static constexpr uint64_t kMult = 0x5DEECE66DULL;
  static constexpr uint64_t kMask = (1ULL << 48) - 1;
  uint64_t s_;
};

// scala.util.Random.shuffle on indices 0..len-1: for n = len..2 { k = nextInt(n); swap(n-1,k) }.
template <typename Idx>
inline void scala_shuffle(JavaRandom& rng, Idx* buf, int64_t len) {
  for (int64_t i = 0; i < len; ++i) buf[i] = static_cast<Idx>(i);
  // The draws do not depend on the buffer, so they run kAhead swaps early and the random slot of
  // each swap is prefetched: a block of millions of ratings no longer pays a cache miss per swap
  // (the det host build's bound).  Same draws in the same order, same permutation.
  constexpr int64_t kAhead = 32;
  int32_t ks[kAhead];
  for (int64_t w = 0; w < kAhead && len - w >= 2; ++w) {
    ks[w] = rng.nextInt(static_cast<int32_t>(len - w));
    __builtin_prefetch(buf + ks[w], 1);
  }
  for (int64_t n = len; n >= 2; --n) {
    const int64_t slot = (len - n) % kAhead;
    const int32_t k = ks[slot];
    if (n - kAhead >= 2) {
      ks[slot] = rng.nextInt(static_cast<int32_t>(n - kAhead));
      __builtin_prefetch(buf + ks[slot], 1);
    }
    const Idx t = buf[n - 1];
    buf[n - 1] = buf[k];
    buf[k] = t;
  }
}

// flink-ml 1.3 LearningRateMethod.calculateLearningRate(lr, t, lambda) (DSGDforMF.scala:383-386).
inline double learning_rate(int method, double lr, int32_t t, double lambda, double arg) {
  switch (method) {
    case 1: return lr;                                                    // Constant
    case 2: return 1.0 / (lambda * (arg + static_cast<double>(t) - 1.0)); // Bottou
    case 3: return lr / std::pow(static_cast<double>(t), arg);            // InvScaling
    case 4: return lr * std::pow(1.0 + lambda * lr * static_cast<double>(t), -arg);  // Xu
    default: return lr / std::sqrt(static_cast<double>(t));              // Default
  }
}

}  // namespace mfhip
