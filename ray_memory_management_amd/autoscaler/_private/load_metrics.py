"""Per-node load as seen by the autoscaler. Parity: reference
python/ray/autoscaler/_private/load_metrics.py (static/dynamic resources per node, last-used
time for idle detection, resource demand vector, pending placement groups)."""
from __future__ import annotations

import time
from typing import Dict, List, Tuple

Res = Dict[str, float]


class LoadMetrics:
    def __init__(self):
        self.static: Dict[str, Res] = {}
        self.dynamic: Dict[str, Res] = {}
        self.last_used: Dict[str, float] = {}
        self.demands: List[Res] = []
        self.pending_pgs: List[Tuple[int, List[Res]]] = []

    def update(self, node_id: str, total: Res, avail: Res, busy: bool) -> None:
        self.static[node_id] = dict(total)
        self.dynamic[node_id] = dict(avail)
        now = time.time()
        used = busy or any(avail.get(k, 0.0) + 1e-9 < v for k, v in total.items()
                           if not k.startswith("node:") and "_group_" not in k)
        if used or node_id not in self.last_used:
            self.last_used[node_id] = now

    def prune(self, alive: List[str]) -> None:
        for d in (self.static, self.dynamic, self.last_used):
            for k in list(d):
                if k not in alive:
                    del d[k]

    def idle_seconds(self, node_id: str) -> float:
        return time.time() - self.last_used.get(node_id, time.time())

    def summary(self) -> dict:
        tot: Res = {}
        av: Res = {}
        for n, r in self.static.items():
            for k, v in r.items():
                if k.startswith("node:") or "_group_" in k:
                    continue
                tot[k] = tot.get(k, 0.0) + v
                av[k] = av.get(k, 0.0) + self.dynamic.get(n, {}).get(k, 0.0)
        return {"total": tot, "used": {k: tot[k] - av.get(k, 0.0) for k in tot},
                "demands": list(self.demands), "pending_placement_groups": len(self.pending_pgs)}
