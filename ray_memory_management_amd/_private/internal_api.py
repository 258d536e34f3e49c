"""Reference-path internal API: `from ray._private.internal_api import memory_summary, free, global_gc`
(reference python/ray/_private/internal_api.py:14-216). The reference formats a raylet
FormatGlobalMemoryInfo reply; here the head's store stats and object table are read directly.
`ray_memory_management_amd.internal` re-exports these."""
from __future__ import annotations

from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import worker as _w

__all__ = ["free", "global_gc", "memory_summary", "get_store_stats", "store_stats_summary"]

_UNITS = {"B": 1, "KB": 1 << 10, "MB": 1 << 20, "GB": 1 << 30}


def global_gc():
    """gc.collect() on every worker and driver of the cluster (reference internal_api.py:14)."""
    import gc

    gc.collect()
    w = _w.global_worker
    if w is not None:
        w.send((P.GLOBAL_GC,))


def store_stats_summary(st: dict) -> str:
    """Reference internal_api.py:108 wording, from the head's store stats dict."""
    mib = 1 << 20
    cap = max(1, st.get("capacity", 1))
    s = "--- Aggregate object store stats across all nodes ---\n"
    s += (f"Plasma memory usage {int(st['bytes_in_use'] / mib)} MiB, {st['num_objects']} objects, "
          f"{round(100 * st['bytes_in_use'] / cap, 2)}% full\n")
    if st.get("fallback_bytes_current", 0) > 0:
        s += f"Plasma filesystem mmap usage: {int(st['fallback_bytes_current'] / mib)} MiB\n"
    if st.get("objects_spilled_total", 0) > 0:
        s += f"Spilled {int(st['bytes_spilled_total'] / mib)} MiB, {st['objects_spilled_total']} objects\n"
    if st.get("objects_restored_total", 0) > 0:
        s += f"Restored {int(st['bytes_restored_total'] / mib)} MiB, {st['objects_restored_total']} objects\n"
    return s


def get_store_stats(state=None, node_manager_address=None, node_manager_port=None) -> str:
    return store_stats_summary(_w._state("store_stats"))


def memory_summary(address=None, redis_password=None, group_by="NODE_ADDRESS", sort_by="OBJECT_SIZE",
                   units="B", line_wrap=True, stats_only=False, num_entries=None) -> str:
    """`ray memory`: the object table (largest first, or by reference count with sort_by="REFERENCE_TYPE")
    followed by the aggregate store stats (reference internal_api.py:21)."""
    st = _w._state("store_stats")
    if stats_only:
        return store_stats_summary(st)
    div = _UNITS[units]
    objs = _w._state("objects")
    key = (lambda o: -o["reference_count"]) if sort_by == "REFERENCE_TYPE" else (lambda o: -o["size"])
    objs = sorted(objs, key=key)
    if num_entries is not None:
        objs = objs[:num_entries]
    lines = ["======== Object references status ========",
             f"Grouping by {group_by}; sorting by {sort_by}; units {units}",
             f"{'object_id':42s} {'size':>12s} {'state':>10s} {'pins':>5s} {'refs':>5s}"]
    for o in objs:
        lines.append(f"{o['object_id']:42s} {o['size'] / div:12.3f} {o['state']:>10s} {o['pin_count']:5d} "
                     f"{o['reference_count']:5d}")
    return "\n".join(lines) + "\n" + store_stats_summary(st)


def free(object_refs, local_only: bool = False):
    """Eagerly delete objects from the store even while referenced (reference internal_api.py:170)."""
    from ray_memory_management_amd.object_ref import ObjectRef

    if isinstance(object_refs, ObjectRef):
        object_refs = [object_refs]
    if not isinstance(object_refs, list):
        raise TypeError(f"free() expects a list of ObjectRef, got {type(object_refs)}")
    for r in object_refs:
        if not isinstance(r, ObjectRef):
            raise TypeError(f"Attempting to call `free` on the value {r}, which is not an ray.ObjectRef.")
    if not object_refs:
        return
    w = _w._require_worker()
    w.store.delete([r.binary() for r in object_refs])
