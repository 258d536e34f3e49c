"""Experimental APIs. Parity: reference python/ray/experimental/ (internal_kv, shuffle, state)."""


def __getattr__(name):
    import importlib

    if name in ("internal_kv", "shuffle", "state", "array", "locations", "dynamic_resources", "gpu_shuffle"):
        return importlib.import_module(f"ray_memory_management_amd.experimental.{name}")
    if name == "get_object_locations":
        return importlib.import_module("ray_memory_management_amd.experimental.locations").get_object_locations
    if name == "set_resource":
        return importlib.import_module("ray_memory_management_amd.experimental.dynamic_resources").set_resource
    if name == "load_package":
        return _load_package
    raise AttributeError(name)


def _load_package(config_path: str):
    """Reference experimental/packaging/load_package.py: load a package (ray_pkg.yaml → runtime_env
    + interface file) onto the cluster. Needs network package staging; not available offline."""
    raise NotImplementedError("load_package stages remote packages; this offline framework supports "
                              "runtime_env working_dir / py_modules instead")
