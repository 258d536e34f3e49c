"""ActorGroup: N copies of one actor class driven together. Parity: reference
python/ray/util/actor_group.py (ActorGroup(actor_cls, num_actors, num_cpus_per_actor,
num_gpus_per_actor, resources_per_actor, init_args, init_kwargs); ``group.method.remote(...)``
calls the method on every actor and returns the refs; ``execute(func)`` / ``execute_async`` run a
function against every actor instance; ``execute_single`` on one; ``start`` / ``shutdown``)."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Type

import ray_memory_management_amd as ray


def _wrap(actor_cls):
    class _Wrapped(actor_cls):
        def _actor_group_execute(self, func, *args, **kwargs):
            return func(self, *args, **kwargs)

    _Wrapped.__name__ = actor_cls.__name__
    _Wrapped.__qualname__ = getattr(actor_cls, "__qualname__", actor_cls.__name__)
    return _Wrapped


class ActorGroupMethod:
    def __init__(self, group: "ActorGroup", name: str):
        self._group, self._name = group, name

    def remote(self, *args, **kwargs) -> List[ray.ObjectRef]:
        return [getattr(a, self._name).remote(*args, **kwargs) for a in self._group.actors]


class ActorGroup:
    def __init__(self, actor_cls: Type, num_actors: int = 1, num_cpus_per_actor: float = 1,
                 num_gpus_per_actor: float = 0, resources_per_actor: Optional[Dict[str, float]] = None,
                 init_args: Optional[tuple] = None, init_kwargs: Optional[Dict[str, Any]] = None):
        if num_actors <= 0:
            raise ValueError("num_actors must be >= 1")
        self.actor_cls = actor_cls
        self.num_actors = num_actors
        self.opts = {"num_cpus": num_cpus_per_actor, "num_gpus": num_gpus_per_actor,
                     "resources": dict(resources_per_actor or {})}
        self.init_args = tuple(init_args or ())
        self.init_kwargs = dict(init_kwargs or {})
        self.actors: List = []
        self.start()

    def start(self):
        if self.actors:
            raise RuntimeError("the actor group is already started")
        cls = ray.remote(_wrap(self.actor_cls)).options(**self.opts)
        self.actors = [cls.remote(*self.init_args, **self.init_kwargs) for _ in range(self.num_actors)]
        ray.get([a.__ray_ready__.remote() for a in self.actors])

    def shutdown(self, patience_s: float = 5):
        for a in self.actors:
            try:
                ray.kill(a)
            except Exception:
                pass
        self.actors = []

    def execute_async(self, func: Callable, *args, **kwargs) -> List[ray.ObjectRef]:
        return [a._actor_group_execute.remote(func, *args, **kwargs) for a in self.actors]

    def execute(self, func: Callable, *args, **kwargs) -> List[Any]:
        return ray.get(self.execute_async(func, *args, **kwargs))

    def execute_single_async(self, actor_index: int, func: Callable, *args, **kwargs) -> ray.ObjectRef:
        return self.actors[actor_index]._actor_group_execute.remote(func, *args, **kwargs)

    def execute_single(self, actor_index: int, func: Callable, *args, **kwargs) -> Any:
        return ray.get(self.execute_single_async(actor_index, func, *args, **kwargs))

    def __len__(self):
        return len(self.actors)

    def __getitem__(self, i):
        return self.actors[i]

    def __getattr__(self, item):
        if item.startswith("_") or item in ("actors", "actor_cls", "num_actors", "opts", "init_args", "init_kwargs"):
            raise AttributeError(item)
        if not hasattr(self.actor_cls, item):
            raise AttributeError(f"{self.actor_cls.__name__} has no method {item!r}")
        return ActorGroupMethod(self, item)
