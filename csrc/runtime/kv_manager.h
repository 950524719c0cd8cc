// Paged KV-cache block manager (see kv_manager.cpp for the design notes).
#pragma once
#ifndef BFLY_RT_NO_PYTHON   // the sanitizer self-test builds the runtime without Python
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#endif

#include <algorithm>
#include <cstdint>
#include <iterator>
#include <list>
#include <stdexcept>
#include <tuple>
#include <unordered_map>
#include <vector>

#ifndef BFLY_RT_NO_PYTHON
namespace py = pybind11;
#endif

namespace bfly_rt {

// Prefix caching: a FULL page whose tokens are known (a prompt block) is registered under a
// chained 64-bit hash of every token up to its end. When its last owner frees it, the page is
// not returned to the free list but parked in an LRU of cached pages, still counted as free
// capacity; a later request whose prompt starts with the same blocks takes those pages back
// (match_prefix / allocate_prefixed) and only prefills the rest. Pages are evicted from the
// LRU (and unregistered) only when the free list is empty.
inline uint64_t kv_block_hash(uint64_t prev, const int32_t* tok, int n) {
  uint64_t h = prev ^ 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; ++i) {
    uint64_t z = h + (uint64_t)(uint32_t)tok[i] + 0x9E3779B97F4A7C15ull;   // splitmix64 step
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    h = z ^ (z >> 31);
  }
  return h | 1ull;   // 0 = "no hash"
}

class KVBlockManager {
 public:
  KVBlockManager(int num_blocks, int block_size)
      : num_blocks_(num_blocks), block_size_(block_size), refcnt_(num_blocks, 0),
        hash_(num_blocks, 0), lru_pos_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad KV geometry");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  }

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)(free_.size() + lru_.size()); }
  int num_cached_blocks() const { return (int)cached_.size(); }

  // Hashes of the full blocks of `tokens` (block i covers tokens [i*bs, (i+1)*bs)).
  std::vector<uint64_t> block_hashes(const std::vector<int32_t>& tokens) const {
    std::vector<uint64_t> hs;
    uint64_t h = 0;
    for (size_t i = 0; (i + 1) * block_size_ <= tokens.size(); ++i) {
      h = kv_block_hash(h, tokens.data() + i * block_size_, block_size_);
      hs.push_back(h);
    }
    return hs;
  }
  // Leading blocks of `hashes` whose pages are cached (live or parked in the LRU).
  int match_prefix(const std::vector<uint64_t>& hashes, int max_blocks) const {
    int n = 0;
    while (n < max_blocks && n < (int)hashes.size() && cached_.count(hashes[n])) ++n;
    return n;
  }
  // Register a sequence that starts with the cached pages of hashes[0..nblocks) and has
  // `tokens` more tokens to cache; returns the slots of those tokens.
  std::vector<int32_t> allocate_prefixed(int64_t sid, const std::vector<uint64_t>& hashes, int nblocks,
                                         int64_t tokens) {
    if (seqs_.count(sid)) throw std::invalid_argument("sequence already allocated");
    Seq s;
    for (int i = 0; i < nblocks; ++i) {
      const int b = cached_.at(hashes[i]);
      if (refcnt_[b] == 0) lru_.erase(lru_pos_[b]);   // parked page comes back to life
      ++refcnt_[b];
      s.blocks.push_back(b);
    }
    s.len = (int64_t)nblocks * block_size_;
    seqs_.emplace(sid, std::move(s));
    return tokens > 0 ? extend(sid, tokens) : std::vector<int32_t>{};
  }
  // Register the sequence's pages that are now full and whose content is hashes[i].
  void register_blocks(int64_t sid, const std::vector<uint64_t>& hashes) {
    const Seq& s = cget(sid);
    const int full = (int)std::min<int64_t>((int64_t)hashes.size(), s.len / block_size_);
    for (int i = 0; i < full; ++i) {
      const int b = s.blocks[i];
      if (hash_[b] != 0 || cached_.count(hashes[i])) continue;
      hash_[b] = hashes[i];
      cached_[hashes[i]] = b;
    }
  }
  int num_seqs() const { return (int)seqs_.size(); }
  bool has(int64_t sid) const { return seqs_.count(sid) != 0; }

  int blocks_needed(int64_t tokens) const { return (int)((tokens + block_size_ - 1) / block_size_); }
  bool can_allocate(int64_t tokens) const { return blocks_needed(tokens) <= num_free(); }

  // Register a sequence with `tokens` tokens to cache; returns their slots.
  std::vector<int32_t> allocate(int64_t sid, int64_t tokens) {
    if (seqs_.count(sid)) throw std::invalid_argument("sequence already allocated");
    const int nb = blocks_needed(tokens);
    if (nb > num_free()) throw std::runtime_error("KV cache out of blocks");
    Seq s;
    s.blocks.reserve(nb + 4);
    for (int i = 0; i < nb; ++i) s.blocks.push_back(take());
    s.len = tokens;
    std::vector<int32_t> slots(tokens);
    for (int64_t t = 0; t < tokens; ++t) slots[t] = slot_of(s, t);
    seqs_.emplace(sid, std::move(s));
    return slots;
  }

  // Slots for `tokens` more tokens of an existing sequence (chunked prefill: the next chunk of
  // a prompt whose earlier chunks are cached). Its pages are private (a sequence is forked only
  // after its prefill), so no copy-on-write is needed.
  std::vector<int32_t> extend(int64_t sid, int64_t tokens) {
    Seq& s = get(sid);
    if (extend_blocks(sid, tokens) > num_free()) throw std::runtime_error("KV cache out of blocks");
    while ((int64_t)s.blocks.size() * block_size_ < s.len + tokens) s.blocks.push_back(take());
    std::vector<int32_t> slots(tokens);
    for (int64_t t = 0; t < tokens; ++t) slots[t] = slot_of(s, s.len + t);
    s.len += tokens;
    return slots;
  }
  // Fresh pages extend(sid, tokens) would take.
  int extend_blocks(int64_t sid, int64_t tokens) const {
    const Seq& s = cget(sid);
    return blocks_needed(s.len + tokens) - (int)s.blocks.size();
  }

  // Reserve the slot for one more token. Returns (slot, cow_src, cow_dst): when the last page
  // is shared, a fresh page is taken and the caller must copy cow_src -> cow_dst first.
  std::tuple<int32_t, int32_t, int32_t> append_slot(int64_t sid) {
    Seq& s = get(sid);
    int cow_src = -1, cow_dst = -1;
    if (s.len % block_size_ == 0) {
      if (num_free() == 0) throw std::runtime_error("KV cache out of blocks");
      s.blocks.push_back(take());
    } else if (refcnt_[s.blocks.back()] > 1) {
      if (num_free() == 0) throw std::runtime_error("KV cache out of blocks");
      cow_src = s.blocks.back();
      cow_dst = take();
      --refcnt_[cow_src];
      s.blocks.back() = cow_dst;
    }
    const int32_t slot = slot_of(s, s.len);
    ++s.len;
    return {slot, cow_src, cow_dst};
  }

  // Can every sequence in `sids` append one token without running out of pages?
  bool can_append(const std::vector<int64_t>& sids) const {
    int need = 0;
    for (int64_t sid : sids) {
      const Seq& s = cget(sid);
      if (s.len % block_size_ == 0 || refcnt_[s.blocks.back()] > 1) ++need;
    }
    return need <= num_free();
  }

  void fork(int64_t parent, int64_t child) {
    const Seq& p = cget(parent);
    if (seqs_.count(child)) throw std::invalid_argument("child exists");
    Seq c = p;
    for (int b : c.blocks) ++refcnt_[b];
    seqs_.emplace(child, std::move(c));
  }

  void free(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    for (int b : it->second.blocks) release(b);
    seqs_.erase(it);
  }

  std::vector<int32_t> block_table(int64_t sid) const {
    const Seq& s = cget(sid);
    return std::vector<int32_t>(s.blocks.begin(), s.blocks.end());
  }
  int64_t length(int64_t sid) const { return cget(sid).len; }

#ifndef BFLY_RT_NO_PYTHON
  // Decode-step arrays for a batch, written into caller buffers:
  //   tables [B, max_blocks] (row-major, zero padded), ctx_lens [B] = len after append.
  // Call after append_slot for this step.
  void fill_decode_tables(const std::vector<int64_t>& sids,
                          py::array_t<int32_t, py::array::c_style> tables,
                          py::array_t<int32_t, py::array::c_style> ctx_lens) const {
    auto T = tables.mutable_unchecked<2>();
    auto C = ctx_lens.mutable_unchecked<1>();
    const int64_t B = (int64_t)sids.size();
    if (T.shape(0) < B || C.shape(0) < B) throw std::invalid_argument("buffers too small");
    const int64_t mb = T.shape(1);
    for (int64_t i = 0; i < B; ++i) {
      const Seq& s = cget(sids[i]);
      if ((int64_t)s.blocks.size() > mb) throw std::invalid_argument("block table too narrow");
      int64_t j = 0;
      for (; j < (int64_t)s.blocks.size(); ++j) T(i, j) = s.blocks[j];
      for (; j < mb; ++j) T(i, j) = 0;
      C(i) = (int32_t)s.len;
    }
  }
#endif

 private:
  struct Seq {
    std::vector<int> blocks;
    int64_t len = 0;
  };
  int take() {
    int b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {   // evict the least recently parked cached page
      b = lru_.front();
      lru_.pop_front();
      cached_.erase(hash_[b]);
      hash_[b] = 0;
    }
    refcnt_[b] = 1;
    return b;
  }
  void release(int b) {
    if (--refcnt_[b] != 0) return;
    if (hash_[b] != 0) {
      lru_.push_back(b);
      lru_pos_[b] = std::prev(lru_.end());
    } else {
      free_.push_back(b);
    }
  }
  int32_t slot_of(const Seq& s, int64_t t) const {
    return (int32_t)(s.blocks[t / block_size_] * block_size_ + t % block_size_);
  }
  Seq& get(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }
  const Seq& cget(int64_t sid) const {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }

  int num_blocks_, block_size_;
  std::vector<int> free_;
  std::vector<int> refcnt_;
  std::vector<uint64_t> hash_;                        // per page: registered hash (0 = none)
  std::list<int> lru_;                                // parked cached pages, oldest first
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int> cached_;          // hash -> page
  std::unordered_map<int64_t, Seq> seqs_;
};

}  // namespace bfly_rt
