"""Autoscaler SDK. Parity: reference python/ray/autoscaler/sdk/sdk.py:request_resources — asks the
autoscaler to scale the cluster so that it could hold the given bundles immediately (a standing
minimum, replaced by each call; ``request_resources()`` with no arguments clears it)."""
from __future__ import annotations

import json
from typing import Dict, List, Optional

REQUEST_KEY = b"__autoscaler_resource_request"
STATUS_KEY = b"__autoscaler_status"


def request_resources(num_cpus: Optional[int] = None, bundles: Optional[List[Dict[str, float]]] = None) -> None:
    from ray_memory_management_amd.internal import _internal_kv_put

    req: List[Dict[str, float]] = []
    if num_cpus:
        req += [{"CPU": 1.0}] * int(num_cpus)
    if bundles:
        for b in bundles:
            if not isinstance(b, dict):
                raise TypeError("bundles must be a list of dicts")
            req.append({k: float(v) for k, v in b.items()})
    _internal_kv_put(REQUEST_KEY, json.dumps(req).encode(), True)


def get_status() -> dict:
    """The autoscaler's last update summary (what ``rmm status`` prints)."""
    from ray_memory_management_amd.internal import _internal_kv_get

    v = _internal_kv_get(STATUS_KEY)
    return json.loads(v) if v else {}
