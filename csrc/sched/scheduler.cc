// Scheduler core implementation. See scheduler.h.
#include "scheduler.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <sstream>
#include <stdexcept>

namespace rmm {

namespace {
inline Fixed ToFixed(double v) { return Fixed(std::llround(v * double(kUnit))); }
inline double FromFixed(Fixed v) { return double(v) / double(kUnit); }
constexpr size_t kReadyCacheCap = 1 << 16;
}  // namespace

Scheduler::Scheduler() {
  for (const char* r : {"CPU", "GPU", "memory", "object_store_memory"}) ResourceId(r);
  gpu_id_ = ids_["GPU"];
}

int Scheduler::ResourceId(const std::string& name) {
  auto it = ids_.find(name);
  if (it != ids_.end()) return it->second;
  int id = int(names_.size());
  names_.push_back(name);
  ids_[name] = id;
  for (auto& kv : nodes_) Grow(&kv.second);
  return id;
}

void Scheduler::Grow(Node* n) {
  if (n->total.size() < names_.size()) {
    n->total.resize(names_.size(), 0);
    n->avail.resize(names_.size(), 0);
  }
}

Node* Scheduler::GetNode(int64_t id) {
  auto it = nodes_.find(id);
  return it == nodes_.end() ? nullptr : &it->second;
}

void Scheduler::AddNode(int64_t node, const std::map<std::string, double>& resources) {
  for (auto& kv : resources) ResourceId(kv.first);
  Node n;
  n.id = node;
  n.total.assign(names_.size(), 0);
  n.avail.assign(names_.size(), 0);
  for (auto& kv : resources) {
    int id = ids_[kv.first];
    n.total[id] = n.avail[id] = ToFixed(kv.second);
  }
  int ngpu = int(std::floor(resources.count("GPU") ? resources.at("GPU") : 0.0));
  n.gpu_free.assign(size_t(ngpu), kUnit);
  nodes_[node] = n;
  if (local_node_ < 0) local_node_ = node;
}

void Scheduler::RemoveNode(int64_t node) {
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return;
  it->second.alive = false;
  // placement groups with bundles on this node become pending again
  for (auto& kv : pgs_) {
    PlacementGroup& pg = kv.second;
    if (pg.removed || !pg.placed) continue;
    bool hit = false;
    for (auto nid : pg.placement) hit |= (nid == node);
    if (hit) {
      for (size_t i = 0; i < pg.bundles.size(); i++)
        if (pg.placement[i] != node) ReturnBundle(&pg, i);
      std::fill(pg.placement.begin(), pg.placement.end(), -1);
      pg.placed = false;
      pending_pgs_.push_back(pg.id);
    }
  }
  nodes_.erase(it);
}

ResourceRequest Scheduler::MakeRequest(const std::map<std::string, double>& r) {
  ResourceRequest rr;
  for (auto& kv : r) {
    if (kv.second <= 0) continue;
    rr.items.push_back({ResourceId(kv.first), ToFixed(kv.second)});
  }
  std::sort(rr.items.begin(), rr.items.end());
  return rr;
}

bool Scheduler::Feasible(const Node& n, const ResourceRequest& r) const {
  if (!n.alive) return false;
  for (auto& it : r.items) {
    if (size_t(it.first) >= n.total.size() || n.total[size_t(it.first)] < it.second) return false;
  }
  return true;
}

bool Scheduler::Available(const Node& n, const ResourceRequest& r) const {
  if (!n.alive) return false;
  for (auto& it : r.items) {
    if (size_t(it.first) >= n.avail.size() || n.avail[size_t(it.first)] < it.second) return false;
    if (it.first == gpu_id_) {
      // instance check: whole GPUs need that many fully free instances; fractional needs one
      // instance with enough room.
      if (it.second >= kUnit) {
        int need = int(it.second / kUnit);
        int freec = 0;
        for (auto f : n.gpu_free) freec += (f == kUnit);
        if (freec < need) return false;
      } else {
        bool ok = false;
        for (auto f : n.gpu_free) ok |= (f >= it.second);
        if (!ok) return false;
      }
    }
  }
  return true;
}

// Critical-resource utilisation: max over resources of used/total (reference scorer).
double Scheduler::Utilization(const Node& n) const {
  double u = 0;
  for (size_t i = 0; i < n.total.size(); i++) {
    if (n.total[i] <= 0) continue;
    const std::string& nm = names_[i];
    if (nm != "CPU" && nm != "GPU" && nm != "memory" && nm != "object_store_memory") continue;
    u = std::max(u, 1.0 - double(n.avail[i]) / double(n.total[i]));
  }
  return u;
}

int64_t Scheduler::HybridPick(const ResourceRequest& r, bool require_available, bool* is_avail) {
  // Traversal: local node first, then the others in id order (globally consistent).
  std::vector<int64_t> order;
  if (nodes_.count(local_node_)) order.push_back(local_node_);
  for (auto& kv : nodes_)
    if (kv.first != local_node_) order.push_back(kv.first);
  int64_t best = -1;
  double best_score = std::numeric_limits<double>::infinity();
  bool best_avail = false;
  for (int64_t nid : order) {
    const Node& n = nodes_.at(nid);
    if (!Feasible(n, r)) continue;
    bool avail = Available(n, r);
    double u = Utilization(n);
    if (u < spread_threshold_) u = 0;
    bool upd = false;
    if (avail) {
      if (!best_avail || u < best_score) upd = true;
    } else if (!best_avail && u < best_score && !require_available) {
      upd = true;
    }
    if (upd) {
      best = nid;
      best_score = u;
      best_avail = avail;
    }
  }
  if (is_avail) *is_avail = best_avail;
  return best;
}

int64_t Scheduler::SpreadPick(const ResourceRequest& r) {
  std::vector<int64_t> order;
  for (auto& kv : nodes_) order.push_back(kv.first);
  if (order.empty()) return -1;
  int64_t feasible = -1;
  for (size_t k = 0; k < order.size(); k++) {
    size_t idx = (spread_rr_ + k) % order.size();
    const Node& n = nodes_.at(order[idx]);
    if (!Feasible(n, r)) continue;
    if (Available(n, r)) {
      spread_rr_ = idx + 1;
      return order[idx];
    }
    if (feasible < 0) feasible = order[idx];
  }
  return feasible;
}

int64_t Scheduler::PickNode(const Task& t, bool require_available) {
  switch (t.strategy) {
    case Strategy::kSpread:
      return SpreadPick(t.req);
    case Strategy::kNodeAffinity: {
      Node* n = GetNode(t.affinity_node);
      if (n && Feasible(*n, t.req)) {
        if (!t.affinity_soft || Available(*n, t.req)) return t.affinity_node;
      }
      if (!t.affinity_soft) return -1;
      bool a;
      return HybridPick(t.req, require_available, &a);
    }
    default: {
      bool a;
      return HybridPick(t.req, require_available, &a);
    }
  }
}

void Scheduler::AcquireOn(Node* n, const ResourceRequest& r, Assignment* out) {
  for (auto& it : r.items) {
    n->avail[size_t(it.first)] -= it.second;
    if (out && it.second > 0) {
      auto gg = group_gpu_ids_.find(it.first);
      if (gg != group_gpu_ids_.end()) {
        // a task inside a placement-group bundle sees the bundle's GPU instances (amount 0:
        // the instances stay reserved by the bundle, not by the task)
        for (int g : gg->second)
          if (std::find(out->gpu_ids.begin(), out->gpu_ids.end(), g) == out->gpu_ids.end()) {
            out->gpu_ids.push_back(g);
            out->gpu_amounts.push_back(0);
          }
      }
    }
    if (it.first == gpu_id_ && out) {
      if (it.second >= kUnit) {
        int need = int(it.second / kUnit);
        for (size_t g = 0; g < n->gpu_free.size() && need > 0; g++) {
          if (n->gpu_free[g] == kUnit) {
            n->gpu_free[g] = 0;
            out->gpu_ids.push_back(int(g));
            out->gpu_amounts.push_back(kUnit);
            need--;
          }
        }
      } else {
        // best fit: the most-used instance that still has room (packs fractional GPUs)
        int bestg = -1;
        for (size_t g = 0; g < n->gpu_free.size(); g++)
          if (n->gpu_free[g] >= it.second && (bestg < 0 || n->gpu_free[g] < n->gpu_free[size_t(bestg)]))
            bestg = int(g);
        if (bestg >= 0) {
          n->gpu_free[size_t(bestg)] -= it.second;
          out->gpu_ids.push_back(bestg);
          out->gpu_amounts.push_back(it.second);
        }
      }
    }
  }
}

void Scheduler::ReleaseOn(Node* n, const ResourceRequest& r, const std::vector<int>& gpu_ids,
                          const std::vector<Fixed>& gpu_amounts) {
  for (auto& it : r.items) {
    if (size_t(it.first) < n->avail.size()) {
      n->avail[size_t(it.first)] += it.second;
      if (n->avail[size_t(it.first)] > n->total[size_t(it.first)])
        n->avail[size_t(it.first)] = n->total[size_t(it.first)];
    }
  }
  for (size_t i = 0; i < gpu_ids.size(); i++) {
    size_t g = size_t(gpu_ids[i]);
    if (g < n->gpu_free.size()) n->gpu_free[g] = std::min(kUnit, n->gpu_free[g] + gpu_amounts[i]);
  }
}

std::string Scheduler::ClassKey(const Task& t) const {
  std::ostringstream os;
  os << int(t.strategy) << ':' << t.affinity_node << ':' << t.affinity_soft;
  for (auto& it : t.req.items) os << '|' << it.first << '=' << it.second;
  return os.str();
}

void Scheduler::MakeReady(Task* t) {
  auto& q = ready_[t->sched_class];
  if (q.empty() && std::find(class_order_.begin(), class_order_.end(), t->sched_class) == class_order_.end())
    class_order_.push_back(t->sched_class);
  q.push_back(t->key);
}

void Scheduler::Submit(int64_t key, const std::map<std::string, double>& req, int strategy,
                       int64_t affinity_node, bool affinity_soft, const std::string& pg_id,
                       int bundle_index, const std::vector<std::string>& deps) {
  Task t;
  t.key = key;
  t.strategy = Strategy(strategy);
  t.affinity_node = affinity_node;
  t.affinity_soft = affinity_soft;
  t.seq = seq_++;
  if (t.strategy == Strategy::kPlacementGroup) {
    // rewrite to the bundle's derived resources
    std::map<std::string, double> r2;
    for (auto& kv : req) {
      if (kv.second <= 0) continue;
      if (bundle_index >= 0)
        r2[kv.first + "_group_" + std::to_string(bundle_index) + "_" + pg_id] = kv.second;
      else
        r2[kv.first + "_group_" + pg_id] = kv.second;
    }
    if (bundle_index >= 0)
      r2["bundle_group_" + std::to_string(bundle_index) + "_" + pg_id] = 0.001;
    else
      r2["bundle_group_" + pg_id] = 0.001;
    t.req = MakeRequest(r2);
    t.strategy = Strategy::kDefault;
  } else {
    t.req = MakeRequest(req);
  }
  t.sched_class = ClassKey(t);
  for (auto& d : deps)
    if (!ready_objects_.count(d)) t.missing.insert(d);
  auto& ref = tasks_[key] = std::move(t);
  if (ref.missing.empty()) {
    MakeReady(&ref);
  } else {
    for (auto& d : ref.missing) waiters_[d].push_back(key);
  }
}

void Scheduler::ObjectReady(const std::string& oid) {
  auto it = waiters_.find(oid);
  if (it == waiters_.end()) {
    if (ready_objects_.insert(oid).second) {
      ready_objects_fifo_.push_back(oid);
      if (ready_objects_fifo_.size() > kReadyCacheCap) {
        ready_objects_.erase(ready_objects_fifo_.front());
        ready_objects_fifo_.pop_front();
      }
    }
    return;
  }
  std::vector<int64_t> keys = std::move(it->second);
  waiters_.erase(it);
  for (int64_t k : keys) {
    auto t = tasks_.find(k);
    if (t == tasks_.end()) continue;
    t->second.missing.erase(oid);
    if (t->second.missing.empty() && !t->second.cancelled) MakeReady(&t->second);
  }
}

bool Scheduler::Cancel(int64_t key) {
  auto it = tasks_.find(key);
  if (it == tasks_.end()) return false;
  for (auto& d : it->second.missing) {
    auto w = waiters_.find(d);
    if (w != waiters_.end()) {
      auto& v = w->second;
      v.erase(std::remove(v.begin(), v.end(), key), v.end());
      if (v.empty()) waiters_.erase(w);
    }
  }
  auto q = ready_.find(it->second.sched_class);
  if (q != ready_.end()) {
    auto& dq = q->second;
    dq.erase(std::remove(dq.begin(), dq.end(), key), dq.end());
  }
  tasks_.erase(it);
  return true;
}

std::vector<Assignment> Scheduler::Schedule(int max_assign) {
  std::vector<Assignment> out;
  std::vector<std::string> next_order;
  for (auto& cls : class_order_) {
    auto qit = ready_.find(cls);
    if (qit == ready_.end()) continue;
    auto& q = qit->second;
    while (!q.empty() && int(out.size()) < max_assign) {
      int64_t key = q.front();
      auto tit = tasks_.find(key);
      if (tit == tasks_.end()) {
        q.pop_front();
        continue;
      }
      Task& t = tit->second;
      int64_t nid = PickNode(t, true);
      Node* n = nid >= 0 ? GetNode(nid) : nullptr;
      if (!n || !Available(*n, t.req)) break;  // head of this class blocked: try next class
      Assignment a;
      a.key = key;
      a.node = nid;
      AcquireOn(n, t.req, &a);
      out.push_back(std::move(a));
      q.pop_front();
      tasks_.erase(tit);
    }
    if (!q.empty()) next_order.push_back(cls);
    else ready_.erase(qit);
  }
  class_order_.swap(next_order);
  return out;
}

bool Scheduler::Acquire(int64_t node, const std::map<std::string, double>& req, bool force,
                        Assignment* out) {
  Node* n = GetNode(node);
  if (!n) return false;
  ResourceRequest r = MakeRequest(req);
  if (!force && !Available(*n, r)) return false;
  AcquireOn(n, r, out);
  return true;
}

void Scheduler::Release(int64_t node, const std::map<std::string, double>& req,
                        const std::vector<int>& gpu_ids, const std::vector<Fixed>& gpu_amounts) {
  Node* n = GetNode(node);
  if (!n) return;
  ReleaseOn(n, MakeRequest(req), gpu_ids, gpu_amounts);
}

std::vector<int64_t> Scheduler::InfeasibleTasks() {
  std::vector<int64_t> r;
  for (auto& kv : tasks_) {
    const Task& t = kv.second;
    bool any = false;
    for (auto& nk : nodes_) any |= Feasible(nk.second, t.req);
    if (!any && t.missing.empty()) r.push_back(kv.first);
  }
  return r;
}

std::vector<int64_t> Scheduler::WaitingTasks() const {
  std::vector<int64_t> r;
  for (auto& kv : tasks_)
    if (!kv.second.missing.empty()) r.push_back(kv.first);
  return r;
}

std::vector<std::map<std::string, double>> Scheduler::ResourceDemands() const {
  std::vector<std::map<std::string, double>> r;
  for (auto& kv : tasks_) {
    const Task& t = kv.second;
    if (t.cancelled || !t.missing.empty()) continue;
    std::map<std::string, double> m;
    bool bundle = false;
    for (auto& it : t.req.items) {
      const std::string& n = names_[size_t(it.first)];
      if (n.find("_group_") != std::string::npos) bundle = true;
      m[n] = FromFixed(it.second);
    }
    if (!bundle) r.push_back(std::move(m));
  }
  return r;
}

std::vector<std::pair<int, std::vector<std::map<std::string, double>>>>
Scheduler::PendingPlacementGroups() const {
  std::vector<std::pair<int, std::vector<std::map<std::string, double>>>> r;
  for (auto& id : pending_pgs_) {
    auto it = pgs_.find(id);
    if (it == pgs_.end() || it->second.placed || it->second.removed) continue;
    std::vector<std::map<std::string, double>> bs;
    for (auto& b : it->second.bundles) {
      std::map<std::string, double> m;
      for (auto& x : b) m[names_[size_t(x.first)]] = FromFixed(x.second);
      bs.push_back(std::move(m));
    }
    r.emplace_back(int(it->second.strategy), std::move(bs));
  }
  return r;
}

// ---------------------------------------------------------------- placement groups

void Scheduler::CreatePlacementGroup(const std::string& id,
                                     const std::vector<std::map<std::string, double>>& bundles,
                                     int strategy) {
  PlacementGroup pg;
  pg.id = id;
  pg.strategy = PgStrategy(strategy);
  for (auto& b : bundles) {
    auto rr = MakeRequest(b);
    pg.bundles.push_back(rr.items);
  }
  pg.placement.assign(bundles.size(), -1);
  pgs_[id] = pg;
  pending_pgs_.push_back(id);
}

void Scheduler::CommitBundle(PlacementGroup* pg, size_t i, int64_t node) {
  Node* n = GetNode(node);
  ResourceRequest r;
  r.items = pg->bundles[i];
  Assignment inst;
  AcquireOn(n, r, &inst);  // reserves concrete GPU instances for the bundle
  if (pg->bundle_gpu_ids.size() < pg->bundles.size()) {
    pg->bundle_gpu_ids.resize(pg->bundles.size());
    pg->bundle_gpu_amt.resize(pg->bundles.size());
  }
  pg->bundle_gpu_ids[i] = inst.gpu_ids;
  pg->bundle_gpu_amt[i] = inst.gpu_amounts;
  std::map<std::string, double> derived;
  for (auto& it : pg->bundles[i]) {
    const std::string nm = names_[size_t(it.first)];
    derived[nm + "_group_" + std::to_string(i) + "_" + pg->id] += FromFixed(it.second);
    derived[nm + "_group_" + pg->id] += FromFixed(it.second);
  }
  derived["bundle_group_" + std::to_string(i) + "_" + pg->id] += 1000;
  derived["bundle_group_" + pg->id] += 1000;
  for (auto& kv : derived) {
    int rid = ResourceId(kv.first);
    n = GetNode(node);
    Grow(n);
    n->total[size_t(rid)] += ToFixed(kv.second);
    n->avail[size_t(rid)] += ToFixed(kv.second);
    if (!inst.gpu_ids.empty() && kv.first.rfind("GPU_group_", 0) == 0) {
      auto& v = group_gpu_ids_[rid];
      for (int g : inst.gpu_ids)
        if (std::find(v.begin(), v.end(), g) == v.end()) v.push_back(g);
    }
  }
  pg->placement[i] = node;
}

void Scheduler::ReturnBundle(PlacementGroup* pg, size_t i) {
  int64_t node = pg->placement[i];
  Node* n = GetNode(node);
  if (!n) return;
  std::map<std::string, double> derived;
  for (auto& it : pg->bundles[i]) {
    const std::string nm = names_[size_t(it.first)];
    derived[nm + "_group_" + std::to_string(i) + "_" + pg->id] += FromFixed(it.second);
    derived[nm + "_group_" + pg->id] += FromFixed(it.second);
  }
  derived["bundle_group_" + std::to_string(i) + "_" + pg->id] += 1000;
  derived["bundle_group_" + pg->id] += 1000;
  for (auto& kv : derived) {
    int rid = ids_[kv.first];
    n->total[size_t(rid)] -= ToFixed(kv.second);
    n->avail[size_t(rid)] -= ToFixed(kv.second);
    if (n->total[size_t(rid)] < 0) n->total[size_t(rid)] = 0;
    group_gpu_ids_.erase(rid);
  }
  ResourceRequest r;
  r.items = pg->bundles[i];
  for (auto& it : r.items) n->avail[size_t(it.first)] += it.second;
  if (i < pg->bundle_gpu_ids.size()) {
    for (size_t k = 0; k < pg->bundle_gpu_ids[i].size(); k++) {
      size_t g = size_t(pg->bundle_gpu_ids[i][k]);
      if (g < n->gpu_free.size()) n->gpu_free[g] = std::min(kUnit, n->gpu_free[g] + pg->bundle_gpu_amt[i][k]);
    }
    pg->bundle_gpu_ids[i].clear();
    pg->bundle_gpu_amt[i].clear();
  }
  pg->placement[i] = -1;
}

bool Scheduler::TryPlacePG(PlacementGroup* pg) {
  // Work on a scratch copy of availability.
  std::map<int64_t, std::vector<Fixed>> avail;
  std::vector<int64_t> order;
  for (auto& kv : nodes_)
    if (kv.second.alive) {
      avail[kv.first] = kv.second.avail;
      order.push_back(kv.first);
    }
  if (order.empty()) return false;
  auto fits = [&](int64_t nid, size_t b) {
    auto& a = avail[nid];
    for (auto& it : pg->bundles[b])
      if (size_t(it.first) >= a.size() || a[size_t(it.first)] < it.second) return false;
    return true;
  };
  auto take = [&](int64_t nid, size_t b) {
    for (auto& it : pg->bundles[b]) avail[nid][size_t(it.first)] -= it.second;
  };
  // least-utilised first ordering (reference bundle policy sorts nodes by score)
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    double ua = Utilization(nodes_.at(a)), ub = Utilization(nodes_.at(b));
    if (ua != ub) return ua < ub;
    return a < b;
  });
  std::vector<int64_t> place(pg->bundles.size(), -1);
  size_t nb = pg->bundles.size();
  switch (pg->strategy) {
    case PgStrategy::kStrictPack: {
      bool done = false;
      for (int64_t nid : order) {
        auto saved = avail[nid];
        bool ok = true;
        for (size_t b = 0; b < nb && ok; b++) {
          if (fits(nid, b)) take(nid, b);
          else ok = false;
        }
        if (ok) {
          std::fill(place.begin(), place.end(), nid);
          done = true;
          break;
        }
        avail[nid] = saved;
      }
      if (!done) return false;
      break;
    }
    case PgStrategy::kPack: {
      // prefer the node that fits the most bundles, fill it, continue with the rest
      for (size_t b = 0; b < nb; b++) {
        int64_t chosen = -1;
        // stick with the node used by the previous bundle when possible
        if (b > 0 && place[b - 1] >= 0 && fits(place[b - 1], b)) chosen = place[b - 1];
        for (size_t k = 0; chosen < 0 && k < order.size(); k++)
          if (fits(order[k], b)) chosen = order[k];
        if (chosen < 0) return false;
        take(chosen, b);
        place[b] = chosen;
      }
      break;
    }
    case PgStrategy::kSpread:
    case PgStrategy::kStrictSpread: {
      std::set<int64_t> used;
      for (size_t b = 0; b < nb; b++) {
        int64_t chosen = -1;
        for (int64_t nid : order)
          if (!used.count(nid) && fits(nid, b)) { chosen = nid; break; }
        if (chosen < 0 && pg->strategy == PgStrategy::kSpread) {
          for (int64_t nid : order)
            if (fits(nid, b)) { chosen = nid; break; }
        }
        if (chosen < 0) return false;
        take(chosen, b);
        used.insert(chosen);
        place[b] = chosen;
      }
      break;
    }
  }
  for (size_t b = 0; b < nb; b++) CommitBundle(pg, b, place[b]);
  pg->placed = true;
  return true;
}

std::vector<std::string> Scheduler::SchedulePlacementGroups() {
  std::vector<std::string> placed, still;
  for (auto& id : pending_pgs_) {
    auto it = pgs_.find(id);
    if (it == pgs_.end() || it->second.removed || it->second.placed) continue;
    if (TryPlacePG(&it->second)) placed.push_back(id);
    else still.push_back(id);
  }
  pending_pgs_.swap(still);
  return placed;
}

bool Scheduler::RemovePlacementGroup(const std::string& id) {
  auto it = pgs_.find(id);
  if (it == pgs_.end()) return false;
  PlacementGroup& pg = it->second;
  if (pg.placed)
    for (size_t i = 0; i < pg.bundles.size(); i++) ReturnBundle(&pg, i);
  pending_pgs_.erase(std::remove(pending_pgs_.begin(), pending_pgs_.end(), id), pending_pgs_.end());
  pgs_.erase(it);
  return true;
}

std::vector<int64_t> Scheduler::PlacementGroupNodes(const std::string& id) const {
  auto it = pgs_.find(id);
  if (it == pgs_.end()) return {};
  return it->second.placement;
}

bool Scheduler::PlacementGroupPlaced(const std::string& id) const {
  auto it = pgs_.find(id);
  return it != pgs_.end() && it->second.placed;
}

// ---------------------------------------------------------------- views

std::map<std::string, double> Scheduler::Total(int64_t node) const {
  std::map<std::string, double> r;
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return r;
  for (size_t i = 0; i < it->second.total.size(); i++)
    if (it->second.total[i] > 0) r[names_[i]] = FromFixed(it->second.total[i]);
  return r;
}

std::map<std::string, double> Scheduler::Available(int64_t node) const {
  std::map<std::string, double> r;
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return r;
  for (size_t i = 0; i < it->second.avail.size(); i++)
    if (it->second.total[i] > 0) r[names_[i]] = FromFixed(std::max<Fixed>(0, it->second.avail[i]));
  return r;
}

std::map<std::string, double> Scheduler::ClusterTotal() const {
  std::map<std::string, double> r;
  for (auto& kv : nodes_)
    for (auto& x : Total(kv.first)) r[x.first] += x.second;
  return r;
}

std::map<std::string, double> Scheduler::ClusterAvailable() const {
  std::map<std::string, double> r;
  for (auto& kv : nodes_)
    for (auto& x : Available(kv.first)) r[x.first] += x.second;
  return r;
}

std::vector<int64_t> Scheduler::Nodes() const {
  std::vector<int64_t> r;
  for (auto& kv : nodes_) r.push_back(kv.first);
  return r;
}

}  // namespace rmm
