// id_index.hpp -- int32 id -> factor row map.  Replaces the reference's joins of ratings
// with (id, idx, blockId) triples (DSGDforMF.scala:301-312) and the online operators'
// mutable.HashMap state (FlinkOnlineMF.scala:62,123; OfflineSpark.scala:33-67).
// Open addressing with linear probing; lookups are read-only and thread-safe.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mfhip {

class IdIndex {
 public:
  void clear() { keys_.clear(); vals_.clear(); size_ = 0; mask_ = 0; }
  int64_t size() const { return size_; }

  void reserve(int64_t n) {
    uint64_t cap = 16;
    while (cap < static_cast<uint64_t>(n) * 2 + 16) cap <<= 1;
    if (cap <= keys_.size()) return;
    rehash(cap);
  }

  // Returns the row for id, or -1.
  int32_t find(int32_t id) const {
    if (keys_.empty()) return -1;
    uint64_t h = hash(id) & mask_;
    while (true) {
      const int32_t v = vals_[h];
      if (v < 0) return -1;
      if (keys_[h] == id) return v;
      h = (h + 1) & mask_;
    }
  }

  // Inserts id -> row if absent; returns the stored row.
  int32_t insert(int32_t id, int32_t row) {
    if (static_cast<uint64_t>(size_ + 1) * 2 > keys_.size()) rehash(keys_.empty() ? 16 : keys_.size() * 2);
    uint64_t h = hash(id) & mask_;
    while (true) {
      if (vals_[h] < 0) { keys_[h] = id; vals_[h] = row; ++size_; return row; }
      if (keys_[h] == id) return vals_[h];
      h = (h + 1) & mask_;
    }
  }

 private:
  static uint64_t hash(int32_t id) {
    uint64_t x = static_cast<uint32_t>(id);
    x ^= x >> 16; x *= 0x7feb352dULL; x ^= x >> 15; x *= 0x846ca68bULL; x ^= x >> 16;
    return x;
  }
  void rehash(uint64_t cap) {
    std::vector<int32_t> ok(std::move(keys_)), ov(std::move(vals_));
    keys_.assign(cap, 0);
    vals_.assign(cap, -1);
    mask_ = cap - 1;
    size_ = 0;
    for (size_t j = 0; j < ov.size(); ++j)
      if (ov[j] >= 0) insert(ok[j], ov[j]);
  }
  std::vector<int32_t> keys_, vals_;
  uint64_t mask_ = 0;
  int64_t size_ = 0;
};

}  // namespace mfhip
