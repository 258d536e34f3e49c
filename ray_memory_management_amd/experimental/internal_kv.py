"""Parity: reference python/ray/experimental/internal_kv.py."""
from ray_memory_management_amd.internal import (  # noqa: F401
    _internal_kv_del, _internal_kv_exists, _internal_kv_get, _internal_kv_initialized, _internal_kv_list,
    _internal_kv_put)
