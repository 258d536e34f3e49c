// pybind11 bindings for the scheduler core.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "scheduler.h"

namespace py = pybind11;
using namespace rmm;

PYBIND11_MODULE(_sched, m) {
  m.doc() = "Scheduler core (native): resources, policies, placement groups, dependency queue";
  m.attr("DEFAULT") = 0;
  m.attr("SPREAD") = 1;
  m.attr("NODE_AFFINITY") = 2;
  m.attr("PLACEMENT_GROUP") = 3;
  m.attr("PACK") = 0;
  m.attr("PG_SPREAD") = 1;
  m.attr("STRICT_PACK") = 2;
  m.attr("STRICT_SPREAD") = 3;
  m.attr("UNIT") = kUnit;

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<>())
      .def("add_node", &Scheduler::AddNode)
      .def("remove_node", &Scheduler::RemoveNode)
      .def("set_local_node", &Scheduler::SetLocalNode)
      .def("set_spread_threshold", &Scheduler::SetSpreadThreshold)
      .def("submit",
           [](Scheduler& s, int64_t key, const std::map<std::string, double>& req, int strategy,
              int64_t affinity_node, bool soft, const std::string& pg, int bundle,
              const std::vector<py::bytes>& deps) {
             std::vector<std::string> d;
             d.reserve(deps.size());
             for (auto& b : deps) d.push_back(std::string(b));
             s.Submit(key, req, strategy, affinity_node, soft, pg, bundle, d);
           },
           py::arg("key"), py::arg("req"), py::arg("strategy") = 0, py::arg("affinity_node") = -1,
           py::arg("soft") = false, py::arg("pg") = "", py::arg("bundle") = -1,
           py::arg("deps") = std::vector<py::bytes>())
      .def("object_ready", [](Scheduler& s, py::bytes oid) { s.ObjectReady(std::string(oid)); })
      .def("objects_ready",
           [](Scheduler& s, const std::vector<py::bytes>& oids) {
             for (auto& o : oids) s.ObjectReady(std::string(o));
           })
      .def("cancel", &Scheduler::Cancel)
      .def("schedule",
           [](Scheduler& s, int max_assign) {
             py::list out;
             for (auto& a : s.Schedule(max_assign)) {
               std::vector<double> amounts;
               for (auto f : a.gpu_amounts) amounts.push_back(double(f) / double(kUnit));
               out.append(py::make_tuple(a.key, a.node, a.gpu_ids, amounts));
             }
             return out;
           },
           py::arg("max_assign") = 1 << 20)
      .def("acquire",
           [](Scheduler& s, int64_t node, const std::map<std::string, double>& req, bool force) -> py::object {
             Assignment a;
             if (!s.Acquire(node, req, force, &a)) return py::none();
             std::vector<double> amounts;
             for (auto f : a.gpu_amounts) amounts.push_back(double(f) / double(kUnit));
             return py::make_tuple(a.gpu_ids, amounts);
           },
           py::arg("node"), py::arg("req"), py::arg("force") = false)
      .def("release",
           [](Scheduler& s, int64_t node, const std::map<std::string, double>& req,
              const std::vector<int>& gpu_ids, const std::vector<double>& amounts) {
             std::vector<Fixed> f;
             for (double a : amounts) f.push_back(Fixed(a * double(kUnit) + 0.5));
             s.Release(node, req, gpu_ids, f);
           },
           py::arg("node"), py::arg("req"), py::arg("gpu_ids") = std::vector<int>(),
           py::arg("amounts") = std::vector<double>())
      .def("create_placement_group", &Scheduler::CreatePlacementGroup)
      .def("schedule_placement_groups", &Scheduler::SchedulePlacementGroups)
      .def("remove_placement_group", &Scheduler::RemovePlacementGroup)
      .def("placement_group_nodes", &Scheduler::PlacementGroupNodes)
      .def("placement_group_placed", &Scheduler::PlacementGroupPlaced)
      .def("total", &Scheduler::Total)
      .def("available", [](Scheduler& s, int64_t n) { return s.Available(n); })
      .def("cluster_total", &Scheduler::ClusterTotal)
      .def("cluster_available", &Scheduler::ClusterAvailable)
      .def("nodes", &Scheduler::Nodes)
      .def("num_pending", &Scheduler::NumPending)
      .def("infeasible_tasks", &Scheduler::InfeasibleTasks)
      .def("waiting_tasks", &Scheduler::WaitingTasks)
      .def("resource_demands", &Scheduler::ResourceDemands)
      .def("pending_placement_groups", &Scheduler::PendingPlacementGroups);
}
