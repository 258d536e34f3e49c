"""Scheduling strategies. Parity: reference python/ray/util/scheduling_strategies.py."""
from __future__ import annotations

from typing import Optional, Union


class PlacementGroupSchedulingStrategy:
    def __init__(self, placement_group, placement_group_bundle_index: int = -1,
                 placement_group_capture_child_tasks: Optional[bool] = None):
        self.placement_group = placement_group
        self.placement_group_bundle_index = placement_group_bundle_index
        self.placement_group_capture_child_tasks = placement_group_capture_child_tasks


class NodeAffinitySchedulingStrategy:
    def __init__(self, node_id: Union[int, str], soft: bool):
        self.node_id = node_id
        self.soft = soft


SchedulingStrategyT = Union[None, str, PlacementGroupSchedulingStrategy, NodeAffinitySchedulingStrategy]

DEFAULT_SCHEDULING_STRATEGY = "DEFAULT"
SPREAD_SCHEDULING_STRATEGY = "SPREAD"
