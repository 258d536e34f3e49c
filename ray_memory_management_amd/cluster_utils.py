"""Virtual multi-node cluster for tests. Parity: reference python/ray/cluster_utils.py (Cluster with
add_node/remove_node). Nodes here are resource pools with their own worker pools served by one head
(one machine, one object store), which is what the scheduling / placement-group tests need."""
from __future__ import annotations

from typing import Dict, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import worker as _w


class NodeHandle:
    def __init__(self, node_id: int, resources: Dict[str, float]):
        self.node_id = node_id
        self.unique_id = node_id
        self.resources = resources

    def __repr__(self):
        return f"Node({self.node_id}, {self.resources})"


class Cluster:
    def __init__(self, initialize_head: bool = False, head_node_args: Optional[dict] = None,
                 connect: bool = False):
        self.head = None
        self.worker_nodes: List[NodeHandle] = []
        if initialize_head:
            self.add_node(**(head_node_args or {}))
            if connect:
                self.connect()

    def add_node(self, num_cpus: float = 1, num_gpus: float = 0, resources: Optional[dict] = None,
                 object_store_memory: int = 256 << 20, **kwargs) -> NodeHandle:
        res = dict(resources or {})
        res["CPU"] = float(num_cpus)
        if num_gpus:
            res["GPU"] = float(num_gpus)
        if self.head is None:
            ray.init(num_cpus=num_cpus, num_gpus=num_gpus, resources=resources,
                     object_store_memory=object_store_memory, **kwargs)
            self.head = NodeHandle(1, res)
            return self.head
        w = _w._require_worker()
        nid = w.request(lambda rid: (P.ADD_NODE, rid, res))
        n = NodeHandle(nid, res)
        self.worker_nodes.append(n)
        return n

    def remove_node(self, node: NodeHandle, allow_graceful: bool = True):
        w = _w._require_worker()
        w.request(lambda rid: (P.REMOVE_NODE, rid, node.node_id))
        if node in self.worker_nodes:
            self.worker_nodes.remove(node)

    def connect(self, namespace=None):
        return None

    def wait_for_nodes(self, timeout=30):
        return None

    @property
    def address(self):
        return _w._session_dir

    def list_all_nodes(self):
        return ([self.head] if self.head else []) + list(self.worker_nodes)

    def shutdown(self):
        ray.shutdown()
        self.head = None
        self.worker_nodes = []


class AutoscalingCluster:
    """A local cluster whose worker nodes are added and removed by the autoscaler.

    Parity: reference python/ray/cluster_utils.py:AutoscalingCluster (fake multi-node provider).
    ``worker_node_types``: {name: {"resources": {...}, "min_workers": m, "max_workers": M}}."""

    def __init__(self, head_resources: dict, worker_node_types: dict, idle_timeout_minutes: float = 0.05,
                 upscaling_speed: float = 1.0, update_interval_s: float = 0.2, max_workers: Optional[int] = None):
        self.head_resources = dict(head_resources)
        types = {k: dict(v) for k, v in worker_node_types.items()}
        for v in types.values():
            v.setdefault("min_workers", 0)
            v.setdefault("max_workers", 1)
        self.config = {"head_node_type": "head", "available_node_types": types,
                       "idle_timeout_minutes": idle_timeout_minutes, "upscaling_speed": upscaling_speed,
                       "update_interval_s": update_interval_s, "provider": {"type": "virtual"}}
        if max_workers is not None:
            self.config["max_workers"] = max_workers

    def start(self, _system_config: Optional[dict] = None, **init_kwargs):
        res = dict(self.head_resources)
        cpus = res.pop("CPU", 0)
        gpus = res.pop("GPU", 0)
        cfg = dict(_system_config or {})
        cfg["autoscaler"] = self.config
        ray.init(num_cpus=cpus, num_gpus=gpus, resources=res or None, _system_config=cfg, **init_kwargs)

    def shutdown(self):
        ray.shutdown()
