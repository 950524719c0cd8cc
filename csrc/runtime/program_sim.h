// Rank-program simulator: executes every rank's communication program of one engine step
// under blocking semantics and reports deadlocks (SURVEY.md §2.7-A A11 "comm scheduler /
// rank program", §5.2 "comm-ordering checker").
//
// partition/schedule.py writes each rank's step down as an ordered list of instructions
// (collectives over a group, point-to-point send / recv, with payload and stream). Its Python
// checker (`check_programs`) compares sequences per group and per pair, which catches a
// mismatched collective or a send without its recv — but not a wait cycle ACROSS groups: rank
// 0 entering group A's all-reduce while rank 1 is still in group C's, whose last member waits
// in group B for rank 0, is consistent per group and still hangs. This simulator runs the
// programs against each other:
//   * a collective completes when every member of its group has reached its next collective
//     on that group (same op and payload, else a mismatch error);
//   * a send on the "send" stream (the engine's side-stream isend of a graph's static output)
//     never blocks; any other send blocks until its receiver is at the matching recv when
//     `rendezvous` is set (RCCL point-to-point on the issuing stream), else it is buffered;
//   * a recv blocks until the pair's next message is there (payloads must match, FIFO).
// The result names every rank still blocked and the instruction it is blocked on, so a hang
// that would show up on the node as a step watchdog is found before any rank starts.
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace bfly_rt {

enum SimKind { kSimCollective = 0, kSimSend = 1, kSimRecv = 2 };

struct SimOp {
  int kind;                   // SimKind
  std::string op;             // all_reduce | all_gather | ... | send | recv
  std::vector<int> group;     // collective: members (sorted); send / recv: {src, dst}
  int64_t nbytes;
  bool nonblocking;           // send on the engine's side stream
};

struct SimBlocked {
  int rank;
  int index;                  // position in the rank's program
  std::string what;
};

struct SimResult {
  bool ok = true;             // every rank ran to the end
  std::string error;          // mismatch (collective op / payload, p2p payload); empty if none
  std::vector<SimBlocked> blocked;
  int64_t completed = 0;      // instructions executed
};

inline std::string sim_describe(const SimOp& o) {
  std::string g;
  for (size_t i = 0; i < o.group.size(); ++i) g += (i ? "," : "") + std::to_string(o.group[i]);
  return o.op + "[" + g + "] " + std::to_string(o.nbytes) + "B";
}

inline SimResult simulate_programs(const std::vector<std::vector<SimOp>>& progs, bool rendezvous) {
  SimResult res;
  const int n = (int)progs.size();
  std::vector<size_t> pc(n, 0);
  std::map<std::pair<int, int>, std::deque<int64_t>> chan;     // (src, dst) -> buffered payloads
  // a collective in progress per group: member -> (op, nbytes) of the instruction it waits on
  std::map<std::vector<int>, std::map<int, std::pair<std::string, int64_t>>> arrived;
  bool progress = true;
  while (progress && res.error.empty()) {
    progress = false;
    for (int r = 0; r < n && res.error.empty(); ++r) {
      while (pc[r] < progs[r].size() && res.error.empty()) {
        const SimOp& o = progs[r][pc[r]];
        if (o.kind == kSimSend) {
          const int dst = o.group.size() > 1 ? o.group[1] : -1;
          if (dst < 0 || dst >= n) {
            res.error = "rank " + std::to_string(r) + ": send to a rank outside the job: " + sim_describe(o);
            break;
          }
          if (rendezvous && !o.nonblocking) {
            // completes with the receiver's matching recv, once the pair's earlier (buffered)
            // messages are consumed: a pair's messages arrive in issue order
            const SimOp* peer = pc[dst] < progs[dst].size() ? &progs[dst][pc[dst]] : nullptr;
            if (!chan[{r, dst}].empty() || !peer || peer->kind != kSimRecv || peer->group != o.group) break;
            if (peer->nbytes != o.nbytes) {
              res.error = "p2p " + std::to_string(r) + "->" + std::to_string(dst) + ": send " +
                          std::to_string(o.nbytes) + "B meets recv " + std::to_string(peer->nbytes) + "B";
              break;
            }
            ++pc[r];
            ++pc[dst];
            res.completed += 2;
            progress = true;
            continue;
          }
          chan[{r, dst}].push_back(o.nbytes);
          ++pc[r];
          ++res.completed;
          progress = true;
        } else if (o.kind == kSimRecv) {
          const int src = o.group.empty() ? -1 : o.group[0];
          auto& q = chan[{src, r}];
          if (q.empty()) break;                  // (a rendezvous sender advances both sides)
          if (q.front() != o.nbytes) {
            res.error = "p2p " + std::to_string(src) + "->" + std::to_string(r) + ": recv " +
                        std::to_string(o.nbytes) + "B, next message " + std::to_string(q.front()) + "B";
            break;
          }
          q.pop_front();
          ++pc[r];
          ++res.completed;
          progress = true;
        } else {
          auto& a = arrived[o.group];
          if (!a.count(r)) {
            a[r] = {o.op, o.nbytes};
            progress = true;
          }
          if (a.size() < o.group.size()) break;  // wait for the other members
          for (const auto& kv : a) {
            if (kv.second.first != o.op || kv.second.second != o.nbytes) {
              res.error = "group " + sim_describe(o) + ": rank " + std::to_string(kv.first) + " is in " +
                          kv.second.first + " " + std::to_string(kv.second.second) + "B";
              break;
            }
          }
          if (!res.error.empty()) break;
          for (const auto& kv : a) ++pc[kv.first];
          res.completed += (int64_t)a.size();
          arrived.erase(o.group);
          progress = true;
        }
      }
    }
  }
  for (int r = 0; r < n; ++r)
    if (pc[r] < progs[r].size()) {
      res.ok = false;
      res.blocked.push_back({r, (int)pc[r], sim_describe(progs[r][pc[r]])});
    }
  if (!res.error.empty()) res.ok = false;
  return res;
}

}  // namespace bfly_rt
