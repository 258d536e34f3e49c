"""Experimental APIs. Parity: reference python/ray/experimental/ (internal_kv, shuffle, state)."""


def __getattr__(name):
    import importlib

    if name in ("internal_kv", "shuffle", "state"):
        return importlib.import_module(f"ray_memory_management_amd.experimental.{name}")
    raise AttributeError(name)
