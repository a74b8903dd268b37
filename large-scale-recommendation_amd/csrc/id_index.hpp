// id_index.hpp -- int32 id -> factor row map.  Replaces the reference's joins of ratings
// with (id, idx, blockId) triples (DSGDforMF.scala:301-312) and the online operators'
// mutable.HashMap state (FlinkOnlineMF.scala:62,123; OfflineSpark.scala:33-67).
// Open addressing with linear probing; lookups are read-only and thread-safe.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace mfhip {

class IdIndex {
 public:
  // id and row side by side: a lookup touches one cache line, not two
  struct Slot {
    int32_t id;
    int32_t row;  // -1: empty
  };
  IdIndex() = default;
  // a copy is a table of its own (its own generation): a mirror of the original never takes it
  IdIndex(const IdIndex& o) : slots_(o.slots_), mask_(o.mask_), size_(o.size_), gen_(next_gen()) {}
  IdIndex& operator=(const IdIndex& o) {
    if (this != &o) { slots_ = o.slots_; mask_ = o.mask_; size_ = o.size_; gen_ = next_gen(); log_.clear(); }
    return *this;
  }
  IdIndex(IdIndex&&) = default;
  IdIndex& operator=(IdIndex&&) = default;
  void clear() { slots_.clear(); size_ = 0; mask_ = 0; gen_ = next_gen(); log_.clear(); }
  int64_t size() const { return size_; }

  // The device mirror of the table (mfhip.cpp DevIndex, the online batch's id lookup on the GPU)
  // copies slots() whole when gen() changed (a rehash or clear: every slot may have moved) and
  // otherwise only the slots written since, listed in log() in write order.  gen() is unique
  // across all tables of the process, so a table replaced by another never matches a stale mirror.
  const Slot* slots() const { return slots_.data(); }
  uint64_t capacity() const { return slots_.size(); }
  uint64_t gen() const { return gen_; }
  const std::vector<uint32_t>& log() const { return log_; }
  static uint64_t hash(int32_t id) {
    uint64_t x = static_cast<uint32_t>(id);
    x ^= x >> 16; x *= 0x7feb352dULL; x ^= x >> 15; x *= 0x846ca68bULL; x ^= x >> 16;
    return x;
  }

  void reserve(int64_t n) {
    uint64_t cap = 16;
    while (cap < static_cast<uint64_t>(n) * 2 + 16) cap <<= 1;
    if (cap <= slots_.size()) return;
    rehash(cap);
  }

  // Returns the row for id, or -1.
  int32_t find(int32_t id) const {
    if (slots_.empty()) return -1;
    uint64_t h = hash(id) & mask_;
    while (true) {
      const Slot sl = slots_[h];
      if (sl.row < 0) return -1;
      if (sl.id == id) return sl.row;
      h = (h + 1) & mask_;
    }
  }

  // find() of n ids into rows (-1 as 0xFFFFFFFF), the slot of the id kPrefetch places ahead
  // prefetched: the table is far larger than L2, so independent lookups overlap their misses.
  void find_many(const int32_t* ids, int64_t n, uint32_t* rows) const {
    constexpr int64_t kPrefetch = 16;
    if (slots_.empty()) {
      for (int64_t j = 0; j < n; ++j) rows[j] = 0xFFFFFFFFu;
      return;
    }
    for (int64_t j = 0; j < n && j < kPrefetch; ++j) __builtin_prefetch(&slots_[hash(ids[j]) & mask_]);
    for (int64_t j = 0; j < n; ++j) {
      if (j + kPrefetch < n) __builtin_prefetch(&slots_[hash(ids[j + kPrefetch]) & mask_]);
      rows[j] = static_cast<uint32_t>(find(ids[j]));
    }
  }

  // Inserts id -> row if absent; returns the stored row.
  int32_t insert(int32_t id, int32_t row) {
    if (static_cast<uint64_t>(size_ + 1) * 2 > slots_.size()) rehash(slots_.empty() ? 16 : slots_.size() * 2);
    uint64_t h = hash(id) & mask_;
    while (true) {
      Slot& sl = slots_[h];
      if (sl.row < 0) { sl = Slot{id, row}; ++size_; log_.push_back(static_cast<uint32_t>(h)); return row; }
      if (sl.id == id) return sl.row;
      h = (h + 1) & mask_;
    }
  }

 private:
  static uint64_t next_gen() {
    static std::atomic<uint64_t> g{1};
    return g.fetch_add(1);
  }
  void rehash(uint64_t cap) {
    std::vector<Slot> old(std::move(slots_));
    slots_.assign(cap, Slot{0, -1});
    mask_ = cap - 1;
    size_ = 0;
    for (const Slot& sl : old)
      if (sl.row >= 0) insert(sl.id, sl.row);
    gen_ = next_gen();  // every slot may have moved: a mirror copies the table again
    log_.clear();
  }
  std::vector<Slot> slots_;
  uint64_t mask_ = 0;
  int64_t size_ = 0;
  uint64_t gen_ = next_gen();
  std::vector<uint32_t> log_;  // slots written since the last rehash, in write order
};

}  // namespace mfhip
