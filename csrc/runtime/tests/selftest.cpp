// Host-runtime self-test for sanitizer builds ("host ASan/UBSan builds of
// csrc/runtime for the CPU-testable parts"). Built by tests/test_runtime_sanitizers.py with
//   g++ -fsanitize=address,undefined -fno-omit-frame-pointer selftest.cpp  (no Python headers)
// and run as a plain executable (no Python). It drives the paged-KV block manager and the
// continuous-batching scheduler (legacy and mixed/chunked modes) through long randomized
// request streams and checks the invariants the engine relies on:
//   * a cache slot is owned by at most one live (non-forked) sequence at any time;
//   * pages are conserved: free + referenced == total, and everything is free at the end;
//   * every request finishes with exactly max_new tokens, whatever preemption happened;
//   * chunk starts/lengths tile each (re)prompt exactly once.
// Exit code 0 = pass; a failed check prints and aborts (and ASan/UBSan abort on memory / UB).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <unordered_map>
#include <vector>

#define BFLY_RT_NO_PYTHON
#include "../program_sim.h"
#include "../scheduler.h"

using namespace bfly_rt;

#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                            \
    }                                                                          \
  } while (0)

static void test_prefix_cache_pages() {
  KVBlockManager kv(8, 4);
  std::vector<int32_t> t = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
  auto hs = kv.block_hashes(t);                  // 2 full blocks
  CHECK(hs.size() == 2 && hs[0] != hs[1]);
  kv.allocate(1, 10);
  kv.register_blocks(1, hs);
  CHECK(kv.num_cached_blocks() == 2 && kv.match_prefix(hs, 2) == 2);
  kv.free(1);                                    // pages parked, still free capacity
  CHECK(kv.num_free() == 8 && kv.match_prefix(hs, 2) == 2);
  auto slots = kv.allocate_prefixed(2, hs, 2, 3);   // reuse both pages, 3 new tokens
  CHECK(slots.size() == 3 && kv.length(2) == 11 && kv.num_free() == 5);
  kv.free(2);
  // exhaust the free list: parked pages are evicted (and unregistered) last
  kv.allocate(3, 32);
  CHECK(kv.num_free() == 0 && kv.num_cached_blocks() == 0 && kv.match_prefix(hs, 2) == 0);
  kv.free(3);
  CHECK(kv.num_free() == 8);
}

static void test_kv_manager() {
  KVBlockManager kv(16, 4);
  auto a = kv.allocate(1, 6);                // 2 pages
  CHECK(a.size() == 6 && kv.num_free() == 14);
  auto b = kv.extend(1, 3);                  // 9 tokens -> 3 pages
  CHECK(b.size() == 3 && kv.num_free() == 13 && kv.length(1) == 9);
  kv.fork(1, 2);                             // shares 3 pages
  CHECK(kv.num_free() == 13);
  auto [s1, src, dst] = kv.append_slot(2);   // last page shared -> copy-on-write
  CHECK(src >= 0 && dst >= 0 && src != dst && kv.num_free() == 12);
  (void)s1;
  for (int i = 0; i < 3; ++i) kv.append_slot(1);   // 12 tokens: fills page 3 of seq 1
  kv.free(1);
  kv.free(2);
  CHECK(kv.num_free() == 16 && kv.num_seqs() == 0);
  bool threw = false;
  try {
    kv.allocate(3, 100);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw && kv.num_free() == 16);
}

static void run_stream(bool mixed, unsigned seed, bool prefix_cache = false) {
  std::mt19937 rng(seed);
  const int kPages = 48, kBS = 8, kMaxBatch = 6;
  KVBlockManager kv(kPages, kBS);
  Scheduler sch(kv, kMaxBatch, /*max_prefill_tokens=*/mixed ? 24 : 64, mixed, prefix_cache);
  struct Req {
    int64_t prompt, max_new, gen = 0;
    int64_t cached = 0;      // tokens of (prompt + generated) scheduled into the cache
    bool done = false;
  };
  std::unordered_map<int64_t, Req> reqs;
  int64_t next_id = 0;
  int steps = 0;
  // prompts drawn from 3 shared prefixes + a random tail (prefix-cache hits and evictions)
  std::vector<std::vector<int32_t>> heads(3);
  for (auto& h : heads)
    for (int i = 0; i < 24; ++i) h.push_back((int32_t)(rng() % 1000));
  auto add = [&]() {
    Req r{(int64_t)(rng() % 40) + 1, (int64_t)(rng() % 12) + 1};
    std::vector<int32_t> toks;
    const auto& h = heads[rng() % 3];
    for (int64_t i = 0; i < r.prompt; ++i) toks.push_back(i < 24 && rng() % 8 ? h[i] : (int32_t)(rng() % 1000));
    sch.add(next_id, r.prompt, r.max_new, toks);
    reqs[next_id++] = r;
  };
  for (int i = 0; i < 8; ++i) add();
  while (sch.num_waiting() + sch.num_running() > 0 || next_id < 60) {
    if (next_id < 60 && rng() % 3 == 0) add();
    StepPlan p = sch.schedule();
    ++steps;
    CHECK(steps < 100000);
    for (int64_t v : p.preempted) reqs[v].cached = 0;   // pages freed: recompute later
    std::set<int32_t> used;                            // slots written this step
    const int nd = p.num_decode;
    for (int i = 0; i < nd; ++i) {
      Req& r = reqs.at(p.seq_ids[i]);
      CHECK(!r.done && r.gen >= 1);
      CHECK(p.decode_positions[i] == r.prompt + r.gen - 1);
      CHECK(used.insert(p.decode_slots[i]).second);
      r.cached = r.prompt + r.gen;
    }
    std::vector<int64_t> sampled(p.seq_ids.begin(), p.seq_ids.begin() + nd);
    for (size_t j = 0; j + nd < p.seq_ids.size(); ++j) {
      const int64_t sid = p.seq_ids[nd + j];
      Req& r = reqs.at(sid);
      if (r.cached == 0 && p.prefill_starts[j] > 0) {   // admitted with a cached prefix
        CHECK(prefix_cache && p.prefill_starts[j] % kBS == 0 && p.prefill_starts[j] < r.prompt + r.gen);
        r.cached = p.prefill_starts[j];
      }
      CHECK(p.prefill_starts[j] == r.cached);          // chunks tile the (re)prompt in order
      CHECK((int64_t)p.prefill_slots[j].size() == p.prefill_lens[j] && p.prefill_lens[j] > 0);
      for (int32_t s : p.prefill_slots[j]) CHECK(used.insert(s).second);
      r.cached += p.prefill_lens[j];
      CHECK(r.cached <= r.prompt + r.gen);
      CHECK(bool(p.prefill_final[j]) == (r.cached == r.prompt + r.gen));
      if (p.prefill_final[j]) sampled.push_back(sid);
    }
    for (int32_t s : used) CHECK(s >= 0 && s < kPages * kBS);
    // the engine: one token per sampled row, finish at max_new
    for (int64_t sid : sampled) {
      Req& r = reqs.at(sid);
      sch.on_token(sid);
      ++r.gen;
      if (r.gen >= r.max_new) {
        r.done = true;
        sch.finish(sid);
      }
    }
    CHECK(kv.num_free() <= kPages);
  }
  for (auto& kvp : reqs) CHECK(kvp.second.done && kvp.second.gen == kvp.second.max_new);
  CHECK(kv.num_free() == kPages && kv.num_seqs() == 0);
  std::printf("stream mixed=%d prefix_cache=%d seed=%u: %zu requests in %d steps, %lld prefix-hit tokens\n",
              (int)mixed, (int)prefix_cache, seed, reqs.size(), steps, (long long)sch.prefix_hit_tokens());
}

// rank-program simulator: a random pipeline of S stages x M microbatches (recv -> TP
// all-reduce -> send) runs to the end under rendezvous semantics; the same programs with two
// ranks' collective order swapped across groups deadlock
static void test_program_sim() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 50; ++trial) {
    const int S = 2 + (int)(rng() % 4), T = 1 + (int)(rng() % 2), M = 1 + (int)(rng() % 4);
    std::vector<std::vector<SimOp>> progs(S * T);
    for (int m = 0; m < M; ++m)
      for (int s = 0; s < S; ++s)
        for (int t = 0; t < T; ++t) {
          const int r = s * T + t;
          if (s > 0) progs[r].push_back({kSimRecv, "recv", {(s - 1) * T + t, r}, 1000 + m, false});
          if (T > 1) {
            std::vector<int> g;
            for (int u = 0; u < T; ++u) g.push_back(s * T + u);
            progs[r].push_back({kSimCollective, "all_reduce", g, 64, false});
          }
          if (s + 1 < S) progs[r].push_back({kSimSend, "send", {r, (s + 1) * T + t}, 1000 + m, (m & 1) != 0});
        }
    const SimResult ok = simulate_programs(progs, true);
    CHECK(ok.ok && ok.error.empty() && ok.blocked.empty());
  }
  std::vector<std::vector<SimOp>> cyc = {
      {{kSimCollective, "all_reduce", {0, 1}, 8, false}, {kSimCollective, "all_reduce", {0, 2}, 8, false}},
      {{kSimCollective, "all_reduce", {1, 2}, 8, false}, {kSimCollective, "all_reduce", {0, 1}, 8, false}},
      {{kSimCollective, "all_reduce", {0, 2}, 8, false}, {kSimCollective, "all_reduce", {1, 2}, 8, false}}};
  const SimResult dl = simulate_programs(cyc, false);
  CHECK(!dl.ok && dl.error.empty() && dl.blocked.size() == 3);
}

int main() {
  test_program_sim();
  test_kv_manager();
  test_prefix_cache_pages();
  for (unsigned seed = 1; seed <= 20; ++seed) {
    run_stream(false, seed);
    run_stream(true, seed);
    run_stream(true, seed, /*prefix_cache=*/true);
  }
  std::printf("runtime selftest: PASS\n");
  return 0;
}
