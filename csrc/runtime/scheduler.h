// Continuous-batching scheduler core (host runtime, C++; header-only so the sanitizer
// self-test (selftest.cpp) builds it without Python) — the "Scheduling System" of the
// reference's declared architecture (/root/reference/CLAUDE.md:22).
//
// Policy (one instance per data-parallel replica; deterministic, so PP/TP ranks that run
// replicas of it on identical inputs make identical decisions without messaging):
//   1. prefill first: admit waiting sequences in FIFO order while the batch has room
//      (max_batch), the step's token budget allows (max_prefill_tokens) and the KV pages for
//      the whole (re)prompt plus one decode page are free; a step is either all-prefill or
//      all-decode, so decode steps keep a fixed shape for hipGraph replay;
//   2. otherwise decode every running sequence; if the KV cache cannot hold one more token
//      for each of them, preempt the most recently admitted ones (free their pages, requeue
//      them at the FRONT of the waiting queue for recompute) until it can.
// Mixed mode (`mixed`, chunked prefill + decode in one step): every step decodes all
// decode-ready sequences AND spends the rest of the token budget on prompt chunks — first the
// sequences already being prefilled (in admission order), then new admissions. A prompt longer
// than the budget is prefilled over several steps (its later chunks attend to the cached
// earlier ones), and decoding never stalls behind a long prefill: the prefill rows ride along
// the decode step's weight streaming. kind 3 = mixed step.
// The scheduler owns page allocation (through KVBlockManager) and returns the cache slots
// of every token it schedules.
#pragma once
#include "kv_manager.h"

#include <algorithm>
#include <deque>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace bfly_rt {

struct StepPlan {
  int kind = 0;  // 0 idle, 1 prefill, 2 decode, 3 mixed (decode rows first, then prompt chunks)
  std::vector<int64_t> seq_ids;                     // decode sequences, then prefill sequences
  int num_decode = 0;                               // leading decode rows of seq_ids
  std::vector<std::vector<int32_t>> prefill_slots;  // per prefill sequence, every chunk token
  std::vector<int64_t> prefill_lens;                // chunk lengths
  std::vector<int64_t> prefill_starts;              // position of each chunk's first token
  std::vector<bool> prefill_final;                  // chunk completes the (re)prompt: sample
  std::vector<int32_t> decode_slots;                // per sequence, the new token
  std::vector<int32_t> decode_positions;
  std::vector<std::pair<int32_t, int32_t>> cow;     // page copies to do before the step
  std::vector<int64_t> preempted;
};

class Scheduler {
 public:
  Scheduler(KVBlockManager& kv, int max_batch, int64_t max_prefill_tokens, bool mixed = false,
            bool prefix_cache = false)
      : kv_(kv), max_batch_(max_batch), max_prefill_tokens_(max_prefill_tokens), mixed_(mixed),
        prefix_cache_(mixed && prefix_cache) {}

  // `tokens` (optional): the prompt, for prefix caching (mixed mode: a later chunk, or a
  // request admitted with a cached prefix, attends to the cached pages of earlier tokens).
  void add(int64_t sid, int64_t prompt_len, int64_t max_new_tokens,
           const std::vector<int32_t>& tokens = {}) {
    if (info_.count(sid)) throw std::invalid_argument("duplicate sequence id");
    Info in{prompt_len, 0, max_new_tokens, false, {}};
    if (prefix_cache_ && (int64_t)tokens.size() == prompt_len) in.hashes = kv_.block_hashes(tokens);
    info_[sid] = std::move(in);
    waiting_.push_back(sid);
  }

  int64_t prefix_hit_tokens() const { return prefix_hit_tokens_; }

  // Context-parallel prefill (engine CP across data-parallel replicas): the prompt was run by
  // the replica's CP group outside this scheduler and its K/V arrives in this rank's pages.
  // Allocate them and enter the sequence as running with its prompt fully cached. Returns the
  // slots of the prompt's tokens; empty when it does not fit now (batch or KV pages).
  std::vector<int32_t> admit_prefilled(int64_t sid, int64_t prompt_len, int64_t max_new_tokens) {
    if (info_.count(sid)) throw std::invalid_argument("duplicate sequence id");
    if ((int)running_.size() >= max_batch_ || !can_admit_prefilled(prompt_len)) return {};
    info_[sid] = Info{prompt_len, 0, max_new_tokens, false, {}};
    running_.push_back(sid);
    return kv_.allocate(sid, prompt_len);
  }
  bool can_admit_prefilled(int64_t prompt_len) const {
    return (int)running_.size() < max_batch_ && kv_.blocks_needed(prompt_len + 1) <= kv_.num_free();
  }


  // Record one generated token (after a prefill or decode step produced it).
  void on_token(int64_t sid) { info_.at(sid).generated++; }

  void finish(int64_t sid) {
    auto it = std::find(running_.begin(), running_.end(), sid);
    if (it != running_.end()) running_.erase(it);
    auto wt = std::find(waiting_.begin(), waiting_.end(), sid);
    if (wt != waiting_.end()) waiting_.erase(wt);
    kv_.free(sid);
    info_.erase(sid);
  }

  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  std::vector<int64_t> running() const { return running_; }
  std::vector<int64_t> waiting() const { return std::vector<int64_t>(waiting_.begin(), waiting_.end()); }

  StepPlan schedule() {
    if (mixed_) return schedule_mixed();
    StepPlan plan;
    // --- 1. prefill admission --------------------------------------------------------------
    int64_t budget = max_prefill_tokens_;
    int free_pages = kv_.num_free();
    while (!waiting_.empty() && (int)(running_.size() + plan.seq_ids.size()) < max_batch_) {
      const int64_t sid = waiting_.front();
      const Info& in = info_.at(sid);
      const int64_t len = in.prompt_len + in.generated;   // recompute after preemption
      if (len > budget && !plan.seq_ids.empty()) break;
      const int need = kv_.blocks_needed(len + 1);
      if (need > free_pages) break;
      waiting_.pop_front();
      plan.seq_ids.push_back(sid);
      plan.prefill_lens.push_back(len);
      plan.prefill_starts.push_back(0);
      plan.prefill_final.push_back(true);
      plan.prefill_slots.push_back(kv_.allocate(sid, len));
      free_pages = kv_.num_free();
      budget -= len;
      if (budget <= 0) break;
    }
    if (!plan.seq_ids.empty()) {
      plan.kind = 1;
      for (int64_t sid : plan.seq_ids) running_.push_back(sid);
      return plan;
    }
    if (running_.empty()) return plan;  // idle
    // --- 2. decode (preempt newest until one token per sequence fits) -------------------------
    while (!running_.empty() && !kv_.can_append(running_)) {
      const int64_t victim = running_.back();
      running_.pop_back();
      kv_.free(victim);
      waiting_.push_front(victim);
      plan.preempted.push_back(victim);
    }
    if (running_.empty()) return plan;
    plan.kind = 2;
    plan.seq_ids = running_;
    plan.num_decode = (int)running_.size();
    for (int64_t sid : running_) {
      auto [slot, src, dst] = kv_.append_slot(sid);
      plan.decode_slots.push_back(slot);
      const Info& in = info_.at(sid);
      plan.decode_positions.push_back((int32_t)(in.prompt_len + in.generated - 1));
      if (src >= 0) plan.cow.emplace_back(src, dst);
    }
    return plan;
  }

 private:
  struct Info {
    int64_t prompt_len, generated, max_new;
    bool in_prefill;   // mixed mode: admitted, its (re)prompt not yet fully scheduled
    std::vector<uint64_t> hashes;   // prefix cache: chained hashes of the prompt's full blocks
  };

  StepPlan schedule_mixed() {
    StepPlan plan;
    // --- 1. decode rows: every running sequence whose prompt is fully cached --------------------
    auto decode_ready = [&]() {
      std::vector<int64_t> d;
      for (int64_t sid : running_)
        if (!info_.at(sid).in_prefill) d.push_back(sid);
      return d;
    };
    std::vector<int64_t> dec = decode_ready();
    while (!dec.empty() && !kv_.can_append(dec)) {   // preempt the newest running sequence
      const int64_t victim = running_.back();
      running_.pop_back();
      kv_.free(victim);
      info_.at(victim).in_prefill = false;
      waiting_.push_front(victim);
      plan.preempted.push_back(victim);
      dec = decode_ready();
    }
    for (int64_t sid : dec) {
      auto [slot, src, dst] = kv_.append_slot(sid);
      plan.seq_ids.push_back(sid);
      plan.decode_slots.push_back(slot);
      const Info& in = info_.at(sid);
      plan.decode_positions.push_back((int32_t)(in.prompt_len + in.generated - 1));
      if (src >= 0) plan.cow.emplace_back(src, dst);
    }
    plan.num_decode = (int)dec.size();
    int64_t budget = max_prefill_tokens_ - plan.num_decode;
    // --- 2. next chunks of the prompts being prefilled (admission order) ------------------------
    for (int64_t sid : running_) {
      if (budget <= 0) break;
      Info& in = info_.at(sid);
      if (!in.in_prefill) continue;
      const int64_t target = in.prompt_len + in.generated, cached = kv_.length(sid);
      const int64_t n = std::min(target - cached, budget);
      if (kv_.extend_blocks(sid, n + (n == target - cached ? 1 : 0)) > kv_.num_free()) break;
      plan.seq_ids.push_back(sid);
      plan.prefill_starts.push_back(cached);
      plan.prefill_lens.push_back(n);
      plan.prefill_slots.push_back(kv_.extend(sid, n));
      plan.prefill_final.push_back(cached + n == target);
      if (cached + n == target) in.in_prefill = false;
      budget -= n;
    }
    // --- 3. admit waiting sequences (FIFO) into the remaining budget ----------------------------
    const int bs = kv_.block_size();
    while (budget > 0 && !waiting_.empty() && (int)running_.size() < max_batch_) {
      const int64_t sid = waiting_.front();
      Info& in = info_.at(sid);
      const int64_t target = in.prompt_len + in.generated;   // recompute after preemption
      // cached prefix: whole blocks, and at least one token left to compute (it yields logits)
      const int P = prefix_cache_ ? kv_.match_prefix(in.hashes, (int)((target - 1) / bs)) : 0;
      const int64_t start = (int64_t)P * bs;
      const int64_t n = std::min(target - start, budget);
      const bool fin = start + n == target;
      // fresh pages for the chunk (+ one decode page when it completes the prompt); the
      // matched pages may be parked ones, which also count as free: reserve them too
      if (kv_.blocks_needed(start + n + (fin ? 1 : 0)) > kv_.num_free()) break;
      waiting_.pop_front();
      running_.push_back(sid);
      plan.seq_ids.push_back(sid);
      plan.prefill_starts.push_back(start);
      plan.prefill_lens.push_back(n);
      plan.prefill_slots.push_back(P > 0 ? kv_.allocate_prefixed(sid, in.hashes, P, n) : kv_.allocate(sid, n));
      plan.prefill_final.push_back(fin);
      in.in_prefill = !fin;
      prefix_hit_tokens_ += start;
      budget -= n;
    }
    if (prefix_cache_)   // pages completed by this step's chunks become reusable next step
      for (size_t j = plan.num_decode; j < plan.seq_ids.size(); ++j)
        kv_.register_blocks(plan.seq_ids[j], info_.at(plan.seq_ids[j]).hashes);
    const bool has_prefill = (int)plan.seq_ids.size() > plan.num_decode;
    plan.kind = plan.num_decode > 0 ? (has_prefill ? 3 : 2) : (has_prefill ? 1 : 0);
    return plan;
  }

  KVBlockManager& kv_;
  int max_batch_;
  int64_t max_prefill_tokens_;
  bool mixed_;
  bool prefix_cache_;
  int64_t prefix_hit_tokens_ = 0;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  std::unordered_map<int64_t, Info> info_;
};

}  // namespace bfly_rt
