"""Placement groups. Parity: reference python/ray/util/placement_group.py (placement_group,
remove_placement_group, get_placement_group, placement_group_table, ready/wait,
get_current_placement_group). Bundle placement itself runs in the native scheduler
(csrc/sched/scheduler.cc TryPlacePG: PACK / SPREAD / STRICT_PACK / STRICT_SPREAD)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import worker as _w
from ray_memory_management_amd._private.ids import PlacementGroupID

VALID_STRATEGIES = ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD")


class PlacementGroup:
    def __init__(self, id: PlacementGroupID, bundle_cache: Optional[List[Dict]] = None):
        self.id = id
        self.bundle_cache = bundle_cache

    @staticmethod
    def empty():
        return PlacementGroup(PlacementGroupID.nil())

    def is_empty(self):
        return self.id.is_nil()

    def ready(self):
        """An ObjectRef that becomes ready when the group is placed (reference semantics)."""
        from ray_memory_management_amd.remote_function import RemoteFunction

        pg = self

        def _ready():
            return True

        rf = RemoteFunction(_ready, {"num_cpus": 0})
        from ray_memory_management_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy

        # a zero-resource task inside the group: schedulable exactly when the bundles exist
        return rf.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg, -1),
                          resources={}).remote()

    def wait(self, timeout_seconds: float = 30) -> bool:
        w = _w._require_worker()
        try:
            return bool(w.request(lambda rid: (P.PG_WAIT, rid, self.id.binary()), timeout=timeout_seconds))
        except Exception:
            return False

    @property
    def bundle_specs(self) -> List[Dict]:
        if self.bundle_cache is None:
            t = placement_group_table(self)
            self.bundle_cache = [t["bundles"][i] for i in sorted(t["bundles"])] if t else []
        return self.bundle_cache

    @property
    def bundle_count(self):
        return len(self.bundle_specs)

    def __eq__(self, o):
        return isinstance(o, PlacementGroup) and o.id == self.id

    def __hash__(self):
        return hash(self.id)

    def __reduce__(self):
        return (PlacementGroup, (self.id, self.bundle_cache))


def placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", name: str = "",
                    lifetime: Optional[str] = None, _max_cpu_fraction_per_node: float = None) -> PlacementGroup:
    if not isinstance(bundles, list) or not bundles:
        raise ValueError("The placement group `bundles` argument must be a non-empty list of dicts.")
    for b in bundles:
        if not isinstance(b, dict) or not b or all(v == 0 for v in b.values()):
            raise ValueError("Bundles cannot be an empty dictionary or resources with only 0 values. "
                             f"Bundles: {bundles}")
        for v in b.values():
            if v < 0:
                raise ValueError("Bundle resources must be non-negative")
    if strategy not in VALID_STRATEGIES:
        raise ValueError(f"Invalid placement group strategy {strategy}. Supported strategies are: {VALID_STRATEGIES}.")
    if lifetime not in (None, "detached"):
        raise ValueError("Placement group `lifetime` argument must be either `None` or 'detached'.")
    w = _w._require_worker()
    pg_id = os.urandom(16)
    r = w.request(lambda rid: (P.PG_CREATE, rid, {"pg_id": pg_id, "bundles": [{k: float(v) for k, v in b.items()} for b in bundles],
                                                  "strategy": strategy, "name": name or None, "namespace": w.namespace,
                                                  "lifetime": lifetime, "job_id": w.job_id}))
    if r[0] == "exists":
        raise ValueError(f"Failed to create placement group '{name}' because name is already taken.")
    return PlacementGroup(PlacementGroupID(pg_id), [dict(b) for b in bundles])


def remove_placement_group(placement_group: PlacementGroup) -> None:
    w = _w._require_worker()
    w.send((P.PG_REMOVE, placement_group.id.binary()))


def get_placement_group(placement_group_name: str) -> PlacementGroup:
    w = _w._require_worker()
    info = w.request(lambda rid: (P.PG_TABLE, rid, (w.namespace, placement_group_name)))
    if info is None:
        raise ValueError(f"Failed to look up placement group with name: {placement_group_name}")
    return PlacementGroup(PlacementGroupID(bytes.fromhex(info["placement_group_id"])))


def placement_group_table(placement_group: Optional[PlacementGroup] = None) -> dict:
    w = _w._require_worker()
    arg = placement_group.id.binary() if placement_group is not None else None
    return w.request(lambda rid: (P.PG_TABLE, rid, arg))


def get_current_placement_group() -> Optional[PlacementGroup]:
    w = _w.global_worker
    if w is None:
        return None
    return w.placement_group_capture


def check_placement_group_index(placement_group, bundle_index):
    if placement_group is None:
        if bundle_index != -1:
            raise ValueError("If placement_group is not set, the value of bundle_index must be -1.")
    elif bundle_index >= placement_group.bundle_count or bundle_index < -1:
        raise ValueError(f"placement_group bundle_index {bundle_index} is invalid.")
