"""Visible-device sharing for GPU collective groups.

Every GPU worker starts with ``HIP_VISIBLE_DEVICES`` set to its own GPU(s) (node.py:_worker_env), so
its GPU is ``cuda:0``. RCCL ranks of one node are faster when each process can see its peers'
devices (peer access over xGMI is set up between visible devices; an isolated process relies on
RCCL's invisible-device path). The reference does the same for Train workers
(python/ray/train/_internal/backend_executor.py `_share_cuda_visible_devices`): every worker of a
node sees the union of the node's GPUs and selects its own as the current device.

``share_node_devices()`` widens this process's visibility to every GPU of its node — only while
HIP is still uninitialised in the process (visibility is read once at HIP init) — and returns the
local index of the worker's own GPU. ``RMM_SHARE_VISIBLE_DEVICES=0`` turns it off.
"""
from __future__ import annotations

import os
from typing import List, Optional


def plan(own: str, node: str) -> Optional[tuple]:
    """(new HIP_VISIBLE_DEVICES, local index of the first own GPU) or None if sharing does not apply."""
    own_ids = [g for g in (own or "").split(",") if g != ""]
    node_ids = [g for g in (node or "").split(",") if g != ""]
    if not own_ids or len(node_ids) <= len(own_ids) or not set(own_ids) <= set(node_ids):
        return None
    return ",".join(node_ids), node_ids.index(own_ids[0])


def _hip_initialized() -> bool:
    import sys

    torch = sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:
        return True


def share_node_devices() -> int:
    """Widen visibility to the node's GPUs (if still possible); returns this worker's device index."""
    if os.environ.get("RMM_SHARE_VISIBLE_DEVICES", "1") == "0":
        return current_own_index()
    p = plan(os.environ.get("RMM_GPU_IDS", ""), os.environ.get("RMM_NODE_GPU_IDS", ""))
    if p is None:
        return current_own_index()
    if _hip_initialized():
        return current_own_index()  # too late to change what HIP enumerates: stay isolated
    vis, idx = p
    os.environ["HIP_VISIBLE_DEVICES"] = vis
    os.environ["CUDA_VISIBLE_DEVICES"] = vis
    os.environ["RMM_SHARED_VISIBLE_DEVICES"] = vis
    return idx


def current_own_index() -> int:
    """Local index of this worker's own GPU under the current visibility."""
    shared = os.environ.get("RMM_SHARED_VISIBLE_DEVICES")
    own = [g for g in os.environ.get("RMM_GPU_IDS", "").split(",") if g != ""]
    if shared and own:
        ids: List[str] = shared.split(",")
        if own[0] in ids:
            return ids.index(own[0])
    return 0
