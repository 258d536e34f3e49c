"""Internal APIs. Parity: reference python/ray/_private/internal_api.py (memory_summary, free,
global_gc) and python/ray/experimental/internal_kv.py."""
from __future__ import annotations

from typing import List, Optional

from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import worker as _w
from ray_memory_management_amd._private.internal_api import (free, get_store_stats, global_gc,  # noqa: F401
                                                              memory_summary)


def memory_pressure_stats() -> dict:
    """Counters of the node's memory-pressure machinery (task-arg backpressure, IO-worker spills,
    global GCs, create-request waits / failures, disk-full state)."""
    return _w._state("memory_pressure")


# ---- internal KV (reference python/ray/experimental/internal_kv.py)
def _internal_kv_initialized() -> bool:
    return _w.global_worker is not None


def _internal_kv_put(key, value, overwrite: bool = True, namespace: Optional[str] = None) -> bool:
    w = _w._require_worker()
    k = key.encode() if isinstance(key, str) else key
    v = value.encode() if isinstance(value, str) else value
    ns = (namespace or "").encode()
    return w.request(lambda rid: (P.KV_PUT, rid, ns, k, v, overwrite))


def _internal_kv_get(key, namespace: Optional[str] = None):
    w = _w._require_worker()
    k = key.encode() if isinstance(key, str) else key
    return w.request(lambda rid: (P.KV_GET, rid, (namespace or "").encode(), k))


def _internal_kv_exists(key, namespace: Optional[str] = None) -> bool:
    return _internal_kv_get(key, namespace) is not None


def _internal_kv_del(key, del_by_prefix: bool = False, namespace: Optional[str] = None) -> int:
    w = _w._require_worker()
    k = key.encode() if isinstance(key, str) else key
    return w.request(lambda rid: (P.KV_DEL, rid, (namespace or "").encode(), k, del_by_prefix))


def _internal_kv_list(prefix, namespace: Optional[str] = None) -> List[bytes]:
    w = _w._require_worker()
    p = prefix.encode() if isinstance(prefix, str) else prefix
    return w.request(lambda rid: (P.KV_KEYS, rid, (namespace or "").encode(), p))
