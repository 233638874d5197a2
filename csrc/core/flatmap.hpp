// Open-addressing hash map (linear probing, backward-shift deletion, power-of-two size)
// for the persistence hot path: the write-behind worker does a handful of lookups per
// persistent message (persist.cpp), where std::unordered_map's node allocations and
// pointer chasing dominated.  Keys need a sentinel "empty" value that is never stored.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace cmq {

template <class K, class V, class H>
class FlatMap {
 public:
  explicit FlatMap(K empty, size_t hint = 8) : empty_(empty) {
    size_t cap = 16;
    while (cap < 2 * hint) cap *= 2;
    resize(cap);
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }

  V* find(const K& k) {
    size_t i = H()(k) & mask_;
    while (true) {
      Slot& s = t_[i];
      if (s.k == empty_) return nullptr;
      if (s.k == k) return &s.v;
      i = (i + 1) & mask_;
    }
  }
  // the value for k, default-constructed when absent; *fresh says which
  V& get(const K& k, bool* fresh = nullptr) {
    if ((n_ + 1) * 2 > t_.size()) resize(t_.size() * 2);
    size_t i = H()(k) & mask_;
    while (true) {
      Slot& s = t_[i];
      if (s.k == empty_) {
        s.k = k;
        s.v = V();
        ++n_;
        if (fresh) *fresh = true;
        return s.v;
      }
      if (s.k == k) {
        if (fresh) *fresh = false;
        return s.v;
      }
      i = (i + 1) & mask_;
    }
  }
  V& operator[](const K& k) { return get(k); }
  bool erase(const K& k) {
    size_t i = H()(k) & mask_;
    while (true) {
      if (t_[i].k == empty_) return false;
      if (t_[i].k == k) break;
      i = (i + 1) & mask_;
    }
    // backward shift: pull later members of the probe run into the hole
    size_t j = i;
    while (true) {
      j = (j + 1) & mask_;
      if (t_[j].k == empty_) break;
      const size_t home = H()(t_[j].k) & mask_;
      // t_[j] may move to i iff its home is not in the cyclic range (i, j]
      if ((j > i && (home <= i || home > j)) || (j < i && (home <= i && home > j))) {
        t_[i] = std::move(t_[j]);
        i = j;
      }
    }
    t_[i].k = empty_;
    --n_;
    return true;
  }
  void clear() {
    if (n_ == 0) return;
    for (auto& s : t_) s.k = empty_;
    n_ = 0;
  }
  template <class F>
  void for_each(F f) {
    for (auto& s : t_)
      if (!(s.k == empty_)) f(s.k, s.v);
  }

 private:
  struct Slot { K k; V v; };
  void resize(size_t cap) {
    std::vector<Slot> old;
    old.swap(t_);
    t_.resize(cap);
    for (auto& s : t_) s.k = empty_;
    mask_ = cap - 1;
    n_ = 0;
    for (auto& s : old)
      if (!(s.k == empty_)) get(s.k) = std::move(s.v);
  }
  std::vector<Slot> t_;
  size_t mask_ = 0, n_ = 0;
  K empty_;
};

struct HashI64 {
  size_t operator()(int64_t k) const {
    uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull;
    return (size_t)(x ^ (x >> 29));
  }
};

}  // namespace cmq
