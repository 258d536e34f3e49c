// Randomised operation-sequence test of the native scheduler core, built only for the host
// memory / UB checkers (tests/test_native_sanitizers.py builds it with AddressSanitizer +
// UBSan). The scheduler is single-threaded by contract (the node serialises calls), so the
// checks here are memory safety and resource accounting, not races.
//
// Parity: reference src/ray/raylet/scheduling/cluster_resource_scheduler_test.cc and
// local_task_manager_test.cc drive submit / dependency-ready / dispatch / release / cancel and
// placement-group bundle commit / return sequences and assert resource conservation; this
// fuzzes the same operations on csrc/sched/scheduler.cc:
//   * available never exceeds total and never goes negative, on every node, after every op;
//   * after every held assignment is released, every pending task cancelled and every
//     placement group removed, each node's available resources equal its totals again.
//
// usage: sched_fuzz [iters] [seed]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../sched/scheduler.h"

using rmm::Assignment;
using rmm::Scheduler;

namespace {

struct Held {
  Assignment a;
  std::map<std::string, double> req;  // exactly what the task acquired
  std::string pg;
};

int g_fail = 0;

void CheckNode(Scheduler& s, int64_t n, const char* when) {
  auto tot = s.Total(n);
  auto av = s.Available(n);
  for (auto& kv : av) {
    double t = tot.count(kv.first) ? tot[kv.first] : 0.0;
    if (kv.second < -1e-6 || kv.second > t + 1e-6) {
      if (g_fail++ < 10)
        std::printf("node %ld %s: %s avail %.4f total %.4f\n", (long)n, when, kv.first.c_str(),
                    kv.second, t);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 7;
  std::mt19937_64 rng(seed);
  auto U = [&](int n) { return static_cast<int>(rng() % n); };

  Scheduler s;
  const std::map<std::string, double> node_res[2] = {
      {{"CPU", 8}, {"GPU", 4}, {"memory", 1e9}}, {{"CPU", 4}, {"GPU", 2}, {"custom", 3}}};
  s.AddNode(1, node_res[0]);
  s.AddNode(2, node_res[1]);
  s.SetLocalNode(1);

  std::map<int64_t, std::pair<std::map<std::string, double>, std::string>> pending;  // key -> req, pg
  std::vector<Held> held;
  std::map<std::string, int> pgs;  // pg id -> bundle count
  int64_t next_key = 1;
  int next_obj = 0, next_pg = 0;
  long n_assigned = 0, n_released = 0, n_cancel = 0, n_pg = 0, n_pg_placed = 0;
  const double cpu_amts[] = {0.5, 1, 2}, gpu_amts[] = {0, 0, 0.25, 0.5, 1};

  for (int it = 0; it < iters; it++) {
    int r = U(100);
    if (r < 30) {
      std::map<std::string, double> req{{"CPU", cpu_amts[U(3)]}};
      double g = gpu_amts[U(5)];
      if (g > 0) req["GPU"] = g;
      if (U(10) == 0) req["custom"] = 1;
      int strategy = U(3);  // default / spread / node affinity
      std::string pg;
      int bundle = -1;
      if (!pgs.empty() && U(4) == 0) {
        auto p = pgs.begin();
        std::advance(p, U(static_cast<int>(pgs.size())));
        pg = p->first;
        bundle = U(p->second + 1) - 1;  // -1 = any bundle
        strategy = 3;
        req = {{"CPU", 0.5}};
      }
      std::vector<std::string> deps;
      for (int d = U(3); d > 0; d--) deps.push_back("o" + std::to_string(U(next_obj + 8)));
      int64_t key = next_key++;
      s.Submit(key, req, strategy, 1 + U(2), U(2) == 0, pg, bundle, deps);
      // what the task will hold if dispatched (placement-group tasks hold derived resources)
      std::map<std::string, double> held_req;
      if (strategy == 3) {
        std::string sfx = bundle >= 0 ? "_group_" + std::to_string(bundle) + "_" + pg : "_group_" + pg;
        for (auto& kv : req) held_req[kv.first + sfx] = kv.second;
        held_req["bundle" + sfx] = 0.001;
      } else {
        held_req = req;
      }
      pending[key] = {held_req, pg};
    } else if (r < 42) {
      s.ObjectReady("o" + std::to_string(next_obj++));
    } else if (r < 46 && !pending.empty()) {
      auto p = pending.begin();
      std::advance(p, U(static_cast<int>(pending.size())));
      s.Cancel(p->first);
      pending.erase(p);
      n_cancel++;
    } else if (r < 66) {
      for (auto& a : s.Schedule(1 + U(4))) {
        auto p = pending.find(a.key);
        if (p == pending.end()) {
          if (g_fail++ < 10) std::printf("assignment for unknown key %ld\n", (long)a.key);
          continue;
        }
        held.push_back({a, p->second.first, p->second.second});
        pending.erase(p);
        n_assigned++;
      }
    } else if (r < 82 && !held.empty()) {
      size_t i = static_cast<size_t>(U(static_cast<int>(held.size())));
      s.Release(held[i].a.node, held[i].req, held[i].a.gpu_ids, held[i].a.gpu_amounts);
      held[i] = held.back();
      held.pop_back();
      n_released++;
    } else if (r < 86 && pgs.size() < 4) {
      std::string id = "pg" + std::to_string(next_pg++);
      int nb = 1 + U(3);
      std::vector<std::map<std::string, double>> bundles;
      for (int b = 0; b < nb; b++) {
        std::map<std::string, double> bres{{"CPU", 1}};
        if (U(2)) bres["GPU"] = U(2) ? 0.5 : 1.0;
        bundles.push_back(bres);
      }
      s.CreatePlacementGroup(id, bundles, U(4));
      pgs[id] = nb;
      n_pg++;
    } else if (r < 90) {
      n_pg_placed += static_cast<long>(s.SchedulePlacementGroups().size());
    } else if (r < 93 && !pgs.empty()) {
      // remove a placement group once no running task holds its bundles; its queued tasks are
      // cancelled first (the reference fails a removed group's pending tasks)
      auto p = pgs.begin();
      std::advance(p, U(static_cast<int>(pgs.size())));
      bool busy = false;
      for (auto& h : held) busy |= h.pg == p->first;
      if (!busy) {
        for (auto q = pending.begin(); q != pending.end();) {
          if (q->second.second == p->first) {
            s.Cancel(q->first);
            q = pending.erase(q);
            n_cancel++;
          } else {
            ++q;
          }
        }
        s.RemovePlacementGroup(p->first);
        pgs.erase(p);
      }
    } else {
      (void)s.ResourceDemands();
      (void)s.PendingPlacementGroups();
      (void)s.InfeasibleTasks();
      (void)s.WaitingTasks();
      (void)s.ClusterAvailable();
    }
    CheckNode(s, 1, "during");
    CheckNode(s, 2, "during");
  }

  for (auto& kv : pending) s.Cancel(kv.first);
  for (auto& h : held) s.Release(h.a.node, h.req, h.a.gpu_ids, h.a.gpu_amounts);
  for (auto& kv : pgs) s.RemovePlacementGroup(kv.first);
  for (int n = 1; n <= 2; n++) {
    auto tot = s.Total(n), av = s.Available(n);
    for (auto& kv : node_res[n - 1]) {
      if (std::fabs(av[kv.first] - kv.second) > 1e-6 || std::fabs(tot[kv.first] - kv.second) > 1e-6) {
        if (g_fail++ < 10)
          std::printf("node %d end: %s avail %.4f total %.4f want %.4f\n", n, kv.first.c_str(),
                      av[kv.first], tot[kv.first], kv.second);
      }
    }
  }
  std::printf("assigned=%ld released=%ld cancelled=%ld pgs=%ld placed=%ld pending_left=%zu fails=%d\n",
              n_assigned, n_released, n_cancel, n_pg, n_pg_placed, s.NumPending(), g_fail);
  bool ok = g_fail == 0 && n_assigned > 0 && n_pg_placed > 0 && s.NumPending() == 0;
  std::printf(ok ? "FUZZ OK\n" : "FUZZ FAILED\n");
  return ok ? 0 : 1;
}
