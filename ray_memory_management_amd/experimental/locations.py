"""Object locations. Parity: reference python/ray/experimental/locations.py
(get_object_locations(obj_refs, timeout_ms) → {ref: {"node_ids": [...], "object_size": bytes}}).
Objects live in the node's shared-memory store (one per node) or, for CUDA tensors, in their
owner's HBM arena; the latter additionally report "gpu": the owner device's PCI address."""
from __future__ import annotations

from typing import Dict, List


def get_object_locations(obj_refs: List, timeout_ms: int = -1) -> Dict:
    import ray_memory_management_amd as ray
    from ray_memory_management_amd._private import serialization as ser
    from ray_memory_management_amd._private.worker import global_worker as w

    if w is None:
        raise RuntimeError("ray.init() must be called first")
    if timeout_ms and timeout_ms > 0:
        ray.wait(list(obj_refs), num_returns=len(obj_refs), timeout=timeout_ms / 1000.0)
    node = ray.get_runtime_context().get_node_id()
    sizes = w.store.sizes([r.binary() for r in obj_refs])
    out = {}
    for r, sz in zip(obj_refs, sizes):
        info = {"node_ids": [node] if sz is not None and sz >= 0 else [], "object_size": sz if sz and sz >= 0 else None}
        if sz is not None and sz >= 0:
            try:  # GPU object descriptors: report the HBM payload size and the owner's device
                from ray_memory_management_amd._private import gpu_object_store as gos

                pin, dsize, msize, tag, is_err, flags = w.store.get_raw(r.binary(), 0)
                try:
                    if tag == ser.TAG_GPU:
                        mv = memoryview(pin)
                        f = gos._DESC.unpack_from(mv, 0)
                        del mv
                        info["object_size"] = int(f[1])
                        info["gpu"] = bytes(f[7]).rstrip(b"\0").decode()
                finally:
                    pin.release()
            except Exception:
                pass
        out[r] = info
    return out
