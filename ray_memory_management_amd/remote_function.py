"""@remote functions. Parity: reference python/ray/remote_function.py and
python/ray/_private/ray_option_utils.py (option validation)."""
from __future__ import annotations

import hashlib
import inspect
import json
from typing import Any, Dict

import cloudpickle

from ray_memory_management_amd._private import worker as _w

_TASK_OPTIONS = {
    "num_returns", "num_cpus", "num_gpus", "memory", "object_store_memory", "resources", "accelerator_type",
    "max_retries", "retry_exceptions", "scheduling_strategy", "placement_group", "placement_group_bundle_index",
    "placement_group_capture_child_tasks", "runtime_env", "name", "max_calls", "_metadata",
}


def _validate(opts: Dict[str, Any], allowed) -> None:
    for k, v in opts.items():
        if k not in allowed:
            raise ValueError(f"Invalid option keyword {k} for remote functions. Valid ones are {sorted(allowed)}.")
    for k in ("num_cpus", "num_gpus", "memory"):
        v = opts.get(k)
        if v is not None and (not isinstance(v, (int, float)) or v < 0):
            raise ValueError(f"The keyword '{k}' only accepts None or a non-negative number")
    nr = opts.get("num_returns")
    if nr is not None and not (isinstance(nr, int) and nr >= 0) and nr != "dynamic":
        raise ValueError("The keyword 'num_returns' only accepts 0, a positive integer or \"dynamic\".")
    res = opts.get("resources")
    if res:
        for r in ("CPU", "GPU"):
            if r in res:
                raise ValueError(f"Use the '{r.lower()}' arguments (num_cpus/num_gpus) instead of resources['{r}'].")


def resources_from_options(opts, default_cpus=1.0):
    res = {}
    c = opts.get("num_cpus")
    res["CPU"] = float(default_cpus if c is None else c)
    g = opts.get("num_gpus")
    if g:
        res["GPU"] = float(g)
    m = opts.get("memory")
    if m:
        res["memory"] = float(m)
    for k, v in (opts.get("resources") or {}).items():
        res[k] = float(v)
    return {k: v for k, v in res.items() if v > 0}


def strategy_from_options(opts, worker=None):
    from ray_memory_management_amd.util.placement_group import PlacementGroup
    from ray_memory_management_amd.util.scheduling_strategies import (
        NodeAffinitySchedulingStrategy, PlacementGroupSchedulingStrategy)

    st = opts.get("scheduling_strategy")
    pg = opts.get("placement_group")
    if st is None and pg is None and (worker is None or worker.placement_group_capture is None):
        return None  # hot path: default strategy, no captured placement group
    if pg is not None and pg != "default" and st is None:
        st = PlacementGroupSchedulingStrategy(pg, opts.get("placement_group_bundle_index", -1),
                                              opts.get("placement_group_capture_child_tasks"))
    if st is None or st == "DEFAULT":
        cap = getattr(worker, "placement_group_capture", None) if worker else None
        if cap is not None and pg != "default":
            return {"type": "PLACEMENT_GROUP", "pg_id": cap.id.binary(), "bundle_index": -1, "capture": True}
        return None
    if st == "SPREAD":
        return {"type": "SPREAD"}
    if isinstance(st, PlacementGroupSchedulingStrategy):
        if st.placement_group is None:
            return None
        return {"type": "PLACEMENT_GROUP", "pg_id": st.placement_group.id.binary(),
                "bundle_index": st.placement_group_bundle_index,
                "capture": bool(st.placement_group_capture_child_tasks)}
    if isinstance(st, NodeAffinitySchedulingStrategy):
        nid = st.node_id
        if isinstance(nid, str):
            nid = int(nid, 16) if not nid.isdigit() else int(nid)
        return {"type": "NODE_AFFINITY", "node_id": int(nid), "soft": st.soft}
    if isinstance(st, PlacementGroup):
        return {"type": "PLACEMENT_GROUP", "pg_id": st.id.binary(), "bundle_index": -1}
    raise ValueError(f"invalid scheduling_strategy {st!r}")


def env_key_of(runtime_env) -> str:
    if not runtime_env:
        return ""
    return hashlib.sha1(json.dumps(runtime_env, sort_keys=True, default=str).encode()).hexdigest()[:16]


class RemoteFunction:
    def __init__(self, function, options: Dict[str, Any]):
        _validate(options, _TASK_OPTIONS)
        self._function = function
        self._options = dict(options)
        self._name = getattr(function, "__qualname__", getattr(function, "__name__", "fn"))
        self._module = getattr(function, "__module__", "")
        self._blob = None
        self._fid = None
        self._res_cache = None  # (opts dict, resources, runtime_env key) for the default options
        self._is_generator = inspect.isgeneratorfunction(function)
        self.__doc__ = function.__doc__
        self.__name__ = getattr(function, "__name__", "remote_function")
        self.__wrapped__ = function

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Remote functions cannot be called directly. Instead of running '{self._name}()', "
                        f"try '{self._name}.remote()'.")

    def _ensure_pickled(self):
        if self._blob is None:
            self._blob = cloudpickle.dumps(self._function)
            self._fid = hashlib.sha1(self._blob).digest()
        return self._fid, self._blob

    def options(self, **opts):
        _validate(opts, _TASK_OPTIONS)
        parent = self
        merged = {**self._options, **opts}

        class _Opt:
            def remote(self_inner, *args, **kwargs):
                return parent._remote(args, kwargs, merged)

            def bind(self_inner, *args, **kwargs):
                from ray_memory_management_amd.dag import FunctionNode

                return FunctionNode(parent, args, kwargs, merged)

        return _Opt()

    def remote(self, *args, **kwargs):
        return self._remote(args, kwargs, self._options)

    def bind(self, *args, **kwargs):
        from ray_memory_management_amd.dag import FunctionNode

        return FunctionNode(self, args, kwargs, self._options)

    def _remote(self, args, kwargs, opts):
        if _w._client is not None:  # Ray Client: the server submits it
            return _w._client.submit_task(self._function, args, kwargs, opts)
        if _w._local_mode:
            from ray_memory_management_amd._private import local_mode as lm

            return lm.submit_function(self, args, kwargs, opts)
        w = _w._require_worker()
        fid, blob = self._ensure_pickled()
        ea, ek, arg_refs, keep = w.prepare_args(args, kwargs)
        nr = opts.get("num_returns", 1)
        if self._is_generator and nr == 1 and "num_returns" not in opts:
            nr = 1
        runtime_env = opts.get("runtime_env") or getattr(w, "job_runtime_env", None)
        rc = self._res_cache
        if rc is not None and rc[0] is opts and rc[3] is runtime_env:
            res, env_key = dict(rc[1]), rc[2]
        else:
            res, env_key = resources_from_options(opts), env_key_of(runtime_env)
            if opts is self._options:
                self._res_cache = (opts, dict(res), env_key, runtime_env)
        spec = {
            "fn_id": fid, "name": self._name, "args": ea, "kwargs": ek, "arg_refs": arg_refs,
            "num_returns": nr, "resources": res,
            "max_retries": opts.get("max_retries", 3 if w.config.get("task_max_retries") is None
                                    else w.config.get("task_max_retries")),
            "retry_exceptions": opts.get("retry_exceptions", False), "strategy": strategy_from_options(opts, w),
            "runtime_env": runtime_env, "env_key": env_key, "max_calls": opts.get("max_calls", 0),
        }
        b = w.export(fid, blob)
        if b is not None:
            spec["fn_blob"] = b
        refs = w.submit_task(spec, keep, blob)
        if nr == "dynamic":
            return refs[0]
        if nr == 0:
            return None
        if nr == 1:
            return refs[0]
        return refs
