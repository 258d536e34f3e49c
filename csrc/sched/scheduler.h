// Scheduler core: cluster resource view, scheduling policies, placement-group bundle
// placement, dependency-gated per-scheduling-class ready queues.
//
// Parity (behaviour, re-implemented): reference
//   src/ray/raylet/scheduling/cluster_resource_scheduler.cc      (feasible/available checks)
//   src/ray/raylet/scheduling/policy/hybrid_scheduling_policy.cc (local-first, spread threshold,
//                                                                 critical-resource utilisation)
//   src/ray/raylet/scheduling/policy/spread_scheduling_policy.cc (round robin)
//   src/ray/raylet/scheduling/policy/node_affinity_scheduling_policy.cc (hard / soft)
//   src/ray/raylet/scheduling/policy/bundle_scheduling_policy.cc (PACK/SPREAD/STRICT_*)
//   src/ray/raylet/dependency_manager.cc, local_task_manager.cc  (wait for args, dispatch by
//                                                                 scheduling class)
//   src/ray/common/scheduling/resource_instance_set.cc           (GPU unit instances)
// Placement-group bundles are committed as derived resources "<R>_group_<i>_<pg>" and
// "<R>_group_<pg>" (the reference's naming), so bundle tasks go through the same matcher.
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace rmm {

using Fixed = int64_t;  // resource quantity in 1/10000 units
constexpr Fixed kUnit = 10000;

enum class Strategy : int { kDefault = 0, kSpread = 1, kNodeAffinity = 2, kPlacementGroup = 3 };
enum class PgStrategy : int { kPack = 0, kSpread = 1, kStrictPack = 2, kStrictSpread = 3 };

struct ResourceRequest {
  std::vector<std::pair<int, Fixed>> items;  // (resource id, amount) sorted by id
};

struct Node {
  int64_t id = 0;
  bool alive = true;
  std::vector<Fixed> total;
  std::vector<Fixed> avail;
  // unit-instance resources: GPU instances' remaining capacity (each starts at kUnit)
  std::vector<Fixed> gpu_free;
};

struct Task {
  int64_t key = 0;
  ResourceRequest req;
  Strategy strategy = Strategy::kDefault;
  int64_t affinity_node = -1;
  bool affinity_soft = false;
  std::unordered_set<std::string> missing;  // dependency object ids not yet available
  std::string sched_class;
  bool cancelled = false;
  int64_t seq = 0;
};

struct Assignment {
  int64_t key;
  int64_t node;
  std::vector<int> gpu_ids;
  std::vector<Fixed> gpu_amounts;
};

struct PlacementGroup {
  std::string id;
  PgStrategy strategy;
  std::vector<std::vector<std::pair<int, Fixed>>> bundles;
  std::vector<int64_t> placement;  // node per bundle (-1 = unplaced)
  std::vector<std::vector<int>> bundle_gpu_ids;    // GPU instances reserved by each bundle
  std::vector<std::vector<Fixed>> bundle_gpu_amt;
  bool placed = false;
  bool removed = false;
};

class Scheduler {
 public:
  Scheduler();
  int ResourceId(const std::string& name);
  const std::string& ResourceName(int id) const { return names_[id]; }

  void AddNode(int64_t node, const std::map<std::string, double>& resources);
  void RemoveNode(int64_t node);
  void SetLocalNode(int64_t node) { local_node_ = node; }
  void SetSpreadThreshold(double t) { spread_threshold_ = t; }

  ResourceRequest MakeRequest(const std::map<std::string, double>& r);

  // Submit a task. deps: object ids (binary) not yet known to be ready.
  void Submit(int64_t key, const std::map<std::string, double>& req, int strategy,
              int64_t affinity_node, bool affinity_soft, const std::string& pg_id, int bundle_index,
              const std::vector<std::string>& deps);
  void ObjectReady(const std::string& oid);
  bool Cancel(int64_t key);
  // Dispatch ready tasks that fit. Resources are acquired for returned assignments.
  std::vector<Assignment> Schedule(int max_assign);
  // Try to acquire resources for one request right now on node (no queueing).
  bool Acquire(int64_t node, const std::map<std::string, double>& req, bool force,
               Assignment* out);
  void Release(int64_t node, const std::map<std::string, double>& req,
               const std::vector<int>& gpu_ids, const std::vector<Fixed>& gpu_amounts);

  // Placement groups
  void CreatePlacementGroup(const std::string& id, const std::vector<std::map<std::string, double>>& bundles,
                            int strategy);
  // Attempts to place pending placement groups; returns ids newly placed.
  std::vector<std::string> SchedulePlacementGroups();
  bool RemovePlacementGroup(const std::string& id);
  std::vector<int64_t> PlacementGroupNodes(const std::string& id) const;
  bool PlacementGroupPlaced(const std::string& id) const;

  std::map<std::string, double> Total(int64_t node) const;
  std::map<std::string, double> Available(int64_t node) const;
  std::map<std::string, double> ClusterTotal() const;
  std::map<std::string, double> ClusterAvailable() const;
  std::vector<int64_t> Nodes() const;
  size_t NumPending() const { return tasks_.size(); }
  std::vector<int64_t> InfeasibleTasks();
  std::vector<int64_t> WaitingTasks() const;
  // Autoscaler views (reference autoscaler/_private/load_metrics.py resource demand vector):
  // requests of tasks whose deps are ready but that are not placed yet (bundle-targeted
  // requests excluded: bundles are the demand), and bundles of placement groups not placed yet.
  std::vector<std::map<std::string, double>> ResourceDemands() const;
  std::vector<std::pair<int, std::vector<std::map<std::string, double>>>> PendingPlacementGroups() const;

 private:
  Node* GetNode(int64_t id);
  bool Feasible(const Node& n, const ResourceRequest& r) const;
  bool Available(const Node& n, const ResourceRequest& r) const;
  double Utilization(const Node& n) const;
  int64_t PickNode(const Task& t, bool require_available);
  int64_t HybridPick(const ResourceRequest& r, bool require_available, bool* is_available);
  int64_t SpreadPick(const ResourceRequest& r);
  void AcquireOn(Node* n, const ResourceRequest& r, Assignment* out);
  void ReleaseOn(Node* n, const ResourceRequest& r, const std::vector<int>& gpu_ids,
                 const std::vector<Fixed>& gpu_amounts);
  void Grow(Node* n);
  bool TryPlacePG(PlacementGroup* pg);
  void CommitBundle(PlacementGroup* pg, size_t i, int64_t node);
  void ReturnBundle(PlacementGroup* pg, size_t i);
  std::string ClassKey(const Task& t) const;
  void MakeReady(Task* t);

  std::vector<std::string> names_;
  std::unordered_map<std::string, int> ids_;
  int gpu_id_ = -1;
  std::map<int64_t, Node> nodes_;
  int64_t local_node_ = -1;
  double spread_threshold_ = 0.5;
  size_t spread_rr_ = 0;
  int64_t seq_ = 0;
  std::unordered_map<int64_t, Task> tasks_;
  std::unordered_map<std::string, std::vector<int64_t>> waiters_;  // oid -> tasks
  std::map<std::string, std::deque<int64_t>> ready_;               // class -> FIFO
  std::vector<std::string> class_order_;
  std::map<std::string, PlacementGroup> pgs_;
  std::vector<std::string> pending_pgs_;
  // derived "GPU_group_*" resource id -> GPU instance ids reserved by the bundle(s)
  std::unordered_map<int, std::vector<int>> group_gpu_ids_;
  std::unordered_set<std::string> ready_objects_;  // small recent cache (bounded)
  std::deque<std::string> ready_objects_fifo_;
};

}  // namespace rmm
