"""Validation of the reference's `object_spilling_config` (reference python/ray/_private/external_storage.py:
`setup_external_storage` picks the storage class from "type" and constructs it with "params", so an unknown
type raises ValueError and an unknown or mistyped parameter raises from the constructor, all inside
`ray.init` before any process starts).

Spilling itself is native here (csrc/store/shm_store.cc: fused spill files, round-robin over the directories);
the storage types that need it are the local-filesystem ones. Cloud / smart_open targets need network access
and are refused with a clear error rather than silently spilling to local disk."""
from __future__ import annotations

import json
from typing import Any, Dict

# types the reference knows; the filesystem-backed ones work here
FILESYSTEM_TYPES = ("filesystem", "mock_distributed_fs")
KNOWN_TYPES = FILESYSTEM_TYPES + ("ray_storage", "smart_open", "unstable_fs", "slow_fs")
_PARAMS = {"directory_path": (str, list), "buffer_size": (int,)}


def validate_spilling_config(cfg: Any) -> Dict[str, Any]:
    """Parse and check an object_spilling_config (JSON string or dict); returns the dict."""
    if isinstance(cfg, (str, bytes)):
        try:
            cfg = json.loads(cfg)
        except ValueError as e:
            raise ValueError(f"object_spilling_config is not valid JSON: {e}") from None
    if not isinstance(cfg, dict) or "type" not in cfg:
        raise ValueError("object_spilling_config must be a dict with a 'type' key")
    t = cfg["type"]
    if t not in KNOWN_TYPES:
        raise ValueError(f"Unknown external storage type: {t}")
    if t not in FILESYSTEM_TYPES:
        raise ValueError(f"External storage type {t!r} is not available in this runtime (no network / cloud "
                         f"storage); use one of {FILESYSTEM_TYPES}")
    params = cfg.get("params") or {}
    if not isinstance(params, dict):
        raise TypeError("object_spilling_config 'params' must be a dict")
    for k, v in params.items():
        if k not in _PARAMS:
            raise TypeError(f"FileSystemStorage got an unexpected keyword argument '{k}'")
        if not isinstance(v, _PARAMS[k]) or isinstance(v, bool):
            raise TypeError(f"object_spilling_config param {k!r} must be {' or '.join(x.__name__ for x in _PARAMS[k])}, "
                            f"got {type(v).__name__}")
    dp = params.get("directory_path")
    if dp is None:
        raise ValueError("object_spilling_config needs params.directory_path")
    if isinstance(dp, list) and (not dp or not all(isinstance(d, str) for d in dp)):
        raise ValueError("directory_path must be a non-empty string or list of strings")
    return cfg
