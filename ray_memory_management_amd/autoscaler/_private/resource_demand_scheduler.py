"""Which nodes to launch for a resource demand.

Parity: reference python/ray/autoscaler/_private/resource_demand_scheduler.py
(``get_nodes_to_launch``, ``_utilization_score``, ``get_bin_pack_residual``, placement-group
strategy handling, ``upscaling_speed`` cap). Re-implemented: demands are first bin-packed onto the
free capacity of running + pending nodes (first-fit, largest demand first); what is left is packed
onto new nodes, choosing each time the node type that the remaining demand uses best (highest
(#demands placed, min utilisation, mean utilisation) score), bounded per type by ``max_workers``
and in total by ``max_workers`` of the cluster.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

Res = Dict[str, float]

# _sched PgStrategy values
PACK, SPREAD, STRICT_PACK, STRICT_SPREAD = 0, 1, 2, 3
_EPS = 1e-9


def _fits(node: Res, req: Res) -> bool:
    return all(node.get(k, 0.0) + _EPS >= v for k, v in req.items() if v > 0)


def _sub(node: Res, req: Res) -> None:
    for k, v in req.items():
        node[k] = node.get(k, 0.0) - v


def _size(req: Res) -> Tuple[float, ...]:
    return (req.get("GPU", 0.0), req.get("CPU", 0.0), sum(req.values()))


def get_bin_pack_residual(node_resources: List[Res], demands: List[Res],
                          strict_spread: bool = False) -> Tuple[List[Res], List[Res]]:
    """Pack `demands` onto copies of `node_resources`; returns (unfulfilled, remaining nodes).
    With strict_spread, each node takes at most one of the demands."""
    nodes = [dict(n) for n in node_resources]
    used = [False] * len(nodes)
    unfulfilled: List[Res] = []
    for d in sorted(demands, key=_size, reverse=True):
        for i, n in enumerate(nodes):
            if strict_spread and used[i]:
                continue
            if _fits(n, d):
                _sub(n, d)
                used[i] = True
                break
        else:
            unfulfilled.append(d)
    return unfulfilled, nodes


def _utilization_score(node: Res, demands: List[Res]) -> Optional[Tuple[float, float, float]]:
    remaining = dict(node)
    placed = 0
    for d in sorted(demands, key=_size, reverse=True):
        if _fits(remaining, d):
            _sub(remaining, d)
            placed += 1
    if placed == 0:
        return None
    utils = [1.0 - remaining.get(k, 0.0) / v for k, v in node.items() if v > 0]
    if not utils:
        return None
    # never launch a GPU node for a CPU-only demand when a CPU node would do (reference rule)
    gpu_penalty = 1.0 if node.get("GPU", 0) > 0 and not any(d.get("GPU", 0) > 0 for d in demands) else 0.0
    return (placed - gpu_penalty * 1e6, min(utils), sum(utils) / len(utils))


def placement_group_demands(pending_pgs: List[Tuple[int, List[Res]]]) -> Tuple[List[Res], List[List[Res]]]:
    """Normal demands + groups of bundles that need distinct nodes (STRICT_SPREAD)."""
    normal: List[Res] = []
    spread_groups: List[List[Res]] = []
    for strategy, bundles in pending_pgs:
        if strategy == STRICT_PACK:
            merged: Res = {}
            for b in bundles:
                for k, v in b.items():
                    merged[k] = merged.get(k, 0.0) + v
            normal.append(merged)
        elif strategy == STRICT_SPREAD:
            spread_groups.append(list(bundles))
        else:
            normal.extend(bundles)
    return normal, spread_groups


def get_nodes_to_launch(node_types: Dict[str, dict], counts: Dict[str, int], node_free: List[Res],
                        node_totals: List[Res], demands: List[Res], pending_pgs: List[Tuple[int, List[Res]]],
                        requested: List[Res], max_workers: int, pending_launches: Dict[str, int],
                        upscaling_speed: float = 1.0) -> Tuple[Dict[str, int], List[Res]]:
    """Returns ({node_type: count to launch}, infeasible demands)."""
    counts = dict(counts)
    for t, n in pending_launches.items():
        counts[t] = counts.get(t, 0) + n
    pending_caps = [dict(node_types[t]["resources"]) for t, n in pending_launches.items() for _ in range(n)]
    to_launch: Dict[str, int] = {}
    total_workers = sum(counts.values())

    def launch_for(unfulfilled: List[Res], strict_spread: bool) -> List[Res]:
        nonlocal total_workers
        left = list(unfulfilled)
        while left:
            best, best_score = None, None
            for name, spec in node_types.items():
                if counts.get(name, 0) >= spec.get("max_workers", 0) or total_workers >= max_workers:
                    continue
                score = _utilization_score(spec["resources"], left[:1] if strict_spread else left)
                if score is not None and (best_score is None or score > best_score):
                    best, best_score = name, score
            if best is None:
                return left
            counts[best] = counts.get(best, 0) + 1
            total_workers += 1
            to_launch[best] = to_launch.get(best, 0) + 1
            left, _ = get_bin_pack_residual([dict(node_types[best]["resources"])], left, strict_spread)
        return []

    infeasible: List[Res] = []
    # 1) request_resources(): the cluster's TOTAL capacity must hold the requested bundles
    if requested:
        caps = [dict(n) for n in node_totals] + [dict(c) for c in pending_caps]
        un, _ = get_bin_pack_residual(caps, requested)
        infeasible += launch_for(un, False)
        pending_caps += [dict(node_types[t]["resources"]) for t, n in to_launch.items() for _ in range(n)]
    # 2) queued tasks/actors + pending placement groups on FREE capacity
    pg_normal, spread_groups = placement_group_demands(pending_pgs)
    free = [dict(n) for n in node_free] + [dict(c) for c in pending_caps]
    un, free = get_bin_pack_residual(free, list(demands) + pg_normal)
    infeasible += launch_for(un, False)
    for group in spread_groups:
        un_g, _ = get_bin_pack_residual(free, group, strict_spread=True)
        infeasible += launch_for(un_g, True)
    # upscaling speed: at most max(5, speed * running) launches per update (reference rule)
    cap = max(5, int(upscaling_speed * max(1, len(node_free))))
    out: Dict[str, int] = {}
    budget = cap
    for t, n in sorted(to_launch.items()):
        k = min(n, budget)
        if k > 0:
            out[t] = k
            budget -= k
    return out, infeasible
