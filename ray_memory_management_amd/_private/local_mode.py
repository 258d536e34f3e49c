"""local_mode=True: run tasks and actor methods synchronously in the driver (debugging aid).

Parity: reference python/ray/_private/worker.py LOCAL_MODE (tasks execute eagerly in-process,
objects live in an in-process dict)."""
from __future__ import annotations

import copy
import os
import threading

from ray_memory_management_amd import exceptions as exc
from ray_memory_management_amd.object_ref import ObjectRef

_objects = {}
_state = {"res": {}}
_lock = threading.Lock()


class _FakeWorker:
    job_id = b"\x00\x00\x00\x01"
    node_id = 1
    current_task_id = None
    current_actor_id = None
    worker_id = b"\x00" * 16
    namespace = "local"
    actor_handle_for_self = None
    placement_group_capture = None
    gpu_ids = []
    head_socket = None


def fake_worker():
    return _FakeWorker()


def start(num_cpus=None, num_gpus=None, resources=None):
    res = dict(resources or {})
    res["CPU"] = float(num_cpus or os.cpu_count() or 1)
    if num_gpus:
        res["GPU"] = float(num_gpus)
    _state["res"] = res


def stop():
    _objects.clear()


def resources():
    return dict(_state["res"])


def _new_ref(value=None, error=None):
    oid = os.urandom(20)
    _objects[oid] = (value, error)
    return ObjectRef(oid, _add_ref=False)


def put(value):
    if isinstance(value, ObjectRef):
        raise TypeError("Calling 'put' on an ObjectRef is not allowed.")
    return _new_ref(copy.deepcopy(value) if not hasattr(value, "__array__") else value)


def _resolve(v):
    if isinstance(v, ObjectRef):
        return get(v)
    return v


def get(refs, timeout=None):
    single = isinstance(refs, ObjectRef)
    lst = [refs] if single else list(refs)
    out = []
    for r in lst:
        value, err = _objects[r.binary()]
        if err is not None:
            raise err
        out.append(value)
    return out[0] if single else out


def wait(refs, num_returns=1, timeout=None):
    refs = list(refs)
    return refs[:num_returns], refs[num_returns:]


def _run(fn, args, kwargs, num_returns, name):
    args = [_resolve(a) for a in args]
    kwargs = {k: _resolve(v) for k, v in kwargs.items()}
    try:
        result = fn(*args, **kwargs)
        if num_returns == 1:
            return _new_ref(result)
        if num_returns == 0:
            return None
        return [_new_ref(v) for v in result]
    except Exception as e:  # noqa: BLE001
        err = exc.RayTaskError.from_exception(e, name).as_instanceof_cause()
        if num_returns in (0, 1):
            return _new_ref(error=err)
        return [_new_ref(error=err) for _ in range(num_returns)]


def submit_function(rf, args, kwargs, opts):
    return _run(rf._function, args, kwargs, opts.get("num_returns", 1), rf._name)


class _LocalActorHandle:
    def __init__(self, inst, cls_name):
        self._inst = inst
        self._cls_name = cls_name

    def __getattr__(self, item):
        m = getattr(self._inst, item)
        handle = self

        class _M:
            def remote(self_inner, *a, **k):
                return _run(m, a, k, getattr(m, "__ray_num_returns__", 1), f"{handle._cls_name}.{item}")

            def options(self_inner, **o):
                return self_inner

        return _M()


def create_actor(ac, args, kwargs, opts):
    args = [_resolve(a) for a in args]
    kwargs = {k: _resolve(v) for k, v in kwargs.items()}
    return _LocalActorHandle(ac._cls(*args, **kwargs), ac._cls.__name__)


def submit_actor_method(handle, name, args, kwargs, num_returns):
    raise RuntimeError("unexpected")
