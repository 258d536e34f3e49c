"""Trainables. Parity: reference python/ray/tune/trainable/{trainable.py (Trainable: setup /
step / save_checkpoint / load_checkpoint / reset_config / cleanup; train() auto-fills
training_iteration, time_this_iter_s, time_total_s, timestamp, done), function_trainable.py
(function API run in a thread, lock-step with session.report / tune.report), util.py
(with_parameters), tune.with_resources}.
"""
from __future__ import annotations

import inspect
import os
import shutil
import tempfile
import threading
import time
import uuid
from typing import Any, Callable, Dict, Optional

from ray_memory_management_amd.air.checkpoint import Checkpoint

RESULT_DUPLICATE = "__duplicate__"


class Trainable:
    """Class API: subclass and implement setup/step (+ save/load_checkpoint for pause/PBT)."""

    def __init__(self, config: Optional[Dict] = None, logger_creator=None, remote_checkpoint_dir=None):
        self.config = dict(config or {})
        self._iteration = 0
        self._time_total = 0.0
        self._timesteps_total = None
        self._episodes_total = None
        self._start = time.time()
        self._logdir = tempfile.mkdtemp(prefix="rmm_trainable_")
        self._trial_info = getattr(self, "_trial_info", None)  # set by the trial actor before __init__
        self.setup(copy_config(self.config))

    # user hooks -------------------------------------------------------
    def setup(self, config: Dict):
        pass

    def step(self) -> Dict:
        raise NotImplementedError

    def save_checkpoint(self, checkpoint_dir: str):
        return None

    def load_checkpoint(self, checkpoint):
        pass

    def reset_config(self, new_config: Dict) -> bool:
        return False

    def cleanup(self):
        pass

    # framework --------------------------------------------------------
    @property
    def iteration(self):
        return self._iteration

    @property
    def training_iteration(self):
        return self._iteration

    @property
    def logdir(self):
        return self._logdir

    @property
    def trial_id(self):
        return (self._trial_info or {}).get("trial_id", "default")

    @property
    def trial_name(self):
        return (self._trial_info or {}).get("trial_name", "default")

    @property
    def trial_resources(self) -> Dict:
        """The resources this trial currently holds (changes under ResourceChangingScheduler)."""
        return dict((self._trial_info or {}).get("resources") or {})

    def get_config(self):
        return self.config

    def train(self) -> Dict:
        t0 = time.time()
        result = self.step()
        if not isinstance(result, dict):
            raise ValueError(f"step() needs to return a dict, got {type(result)}")
        dt = time.time() - t0
        self._iteration += 1
        self._time_total += dt
        result = dict(result)
        result.setdefault("done", False)
        result["training_iteration"] = self._iteration
        result["time_this_iter_s"] = dt
        result["time_total_s"] = self._time_total
        result.setdefault("timestamp", int(time.time()))
        result.setdefault("pid", os.getpid())
        return result

    def save(self, checkpoint_dir: Optional[str] = None):
        """Checkpoint (as a dict-backed Checkpoint, transportable through the object store). With
        `checkpoint_dir` (reference Trainable.save(checkpoint_dir)) it is also written there and
        the directory path is returned; restore() accepts either form."""
        ck = self._save_checkpoint_obj()
        if checkpoint_dir is None:
            return ck
        os.makedirs(checkpoint_dir, exist_ok=True)
        return ck.to_directory(checkpoint_dir)

    def _save_checkpoint_obj(self) -> Checkpoint:
        d = tempfile.mkdtemp(prefix="rmm_ckpt_")
        try:
            out = self.save_checkpoint(d)
            meta = {"_iteration": self._iteration, "_time_total": self._time_total}
            if isinstance(out, dict):
                return Checkpoint.from_dict({"__data__": out, **meta})
            path = out if isinstance(out, str) else d
            ck = Checkpoint.from_directory(path).to_dict()
            ck.update(meta)
            ck["__dir__"] = True
            return Checkpoint.from_dict(ck)
        finally:
            shutil.rmtree(d, ignore_errors=True)

    def restore(self, checkpoint):
        if isinstance(checkpoint, str):
            checkpoint = Checkpoint.from_directory(checkpoint)
        data = checkpoint.to_dict()
        self._iteration = data.pop("_iteration", self._iteration)
        self._time_total = data.pop("_time_total", self._time_total)
        if "__data__" in data:
            self.load_checkpoint(data["__data__"])
        else:
            data.pop("__dir__", None)
            d = tempfile.mkdtemp(prefix="rmm_restore_")
            Checkpoint.from_dict(data).to_directory(d)
            self.load_checkpoint(d)

    def stop(self):
        self.cleanup()


def copy_config(cfg):
    import copy

    return copy.deepcopy(cfg)


class _FunctionTrainable(Trainable):
    """Runs a function trainable in a thread; each train() returns the next reported result."""

    _fn: Callable = None

    def setup(self, config):
        from ray_memory_management_amd.air import session as S

        self._sess = S._Session(trial_name=(self._trial_info or {}).get("trial_name"),
                                trial_id=(self._trial_info or {}).get("trial_id"), config=config)
        self._thread = None
        self._last = {}
        self._restored: Optional[Checkpoint] = None
        self._last_ckpt: Optional[Checkpoint] = None
        self._error = None
        self._finished = False

    def _run(self):
        from ray_memory_management_amd.air import session as S

        S._set_session(self._sess)
        _set_tune_session(self._sess)
        try:
            fn = self._fn
            params = inspect.signature(fn).parameters
            args = [copy_config(self.config)] if len(params) >= 1 else []
            if "checkpoint_dir" in params:
                ckdir = None
                if self._restored is not None:
                    ckdir = tempfile.mkdtemp(prefix="rmm_fn_ckpt_")
                    self._restored.to_directory(ckdir)
                fn(*args, checkpoint_dir=ckdir)
            else:
                fn(*args)
        except SystemExit:
            pass
        except BaseException as e:  # noqa: B902 - forwarded to the driver
            self._error = e
        finally:
            self._sess.results.put(("done", None, None))

    def step(self):
        if self._finished:
            return {"done": True, RESULT_DUPLICATE: True}
        if self._thread is None:
            self._sess.checkpoint = self._restored
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        else:
            self._sess.continue_event.set()
        kind, metrics, ckpt = self._sess.results.get()
        if kind == "done":
            self._finished = True
            if self._error is not None:
                raise self._error
            r = dict(self._last)
            r["done"] = True
            r[RESULT_DUPLICATE] = True
            return r
        if ckpt is not None:
            self._last_ckpt = ckpt
        m = dict(metrics)
        m.pop("training_iteration", None)  # the framework counts iterations
        self._last = m
        return m

    def save(self) -> Optional[Checkpoint]:
        if self._last_ckpt is None:
            return Checkpoint.from_dict({"_iteration": self._iteration, "_time_total": self._time_total})
        d = self._last_ckpt.to_dict()
        d.update({"_iteration": self._iteration, "_time_total": self._time_total, "__fn__": True})
        return Checkpoint.from_dict(d)

    def restore(self, checkpoint: Checkpoint):
        d = checkpoint.to_dict()
        self._iteration = d.pop("_iteration", 0)
        self._time_total = d.pop("_time_total", 0.0)
        if d.pop("__fn__", False):
            self._restored = Checkpoint.from_dict(d)
            self._last_ckpt = self._restored

    def stop(self):
        if self._thread is not None and self._thread.is_alive():
            self._sess.stop_requested = True
            self._sess.continue_event.set()
            self._thread.join(timeout=5)


def wrap_function(fn: Callable) -> type:
    if isinstance(fn, type) and issubclass(fn, Trainable):
        return fn
    cls = type(getattr(fn, "__name__", "func"), (_FunctionTrainable,), {"_fn": staticmethod(fn)})
    cls._resources = getattr(fn, "_resources", None)
    return cls


# ---- legacy function API: tune.report / tune.checkpoint_dir
_tune_session = threading.local()


def _set_tune_session(s):
    _tune_session.s = s


def report(_metric=None, **kwargs):
    """Legacy `tune.report(**metrics)` (reference function_trainable.py)."""
    from ray_memory_management_amd.air import session as S

    if _metric is not None:
        kwargs["_metric"] = _metric
    s = getattr(_tune_session, "s", None) or S._get_session()
    if s is None:
        raise ValueError("tune.report() called outside of a Tune trial")
    ck = getattr(s, "_pending_ckpt", None)
    s._pending_ckpt = None
    s.report(kwargs, ck)


class checkpoint_dir:
    """`with tune.checkpoint_dir(step) as d:` — files written to d become the next report's
    checkpoint."""

    def __init__(self, step: int):
        self.step = step

    def __enter__(self):
        self.dir = tempfile.mkdtemp(prefix=f"rmm_ckpt_{self.step}_")
        return self.dir

    def __exit__(self, *exc):
        from ray_memory_management_amd.air import session as S

        s = getattr(_tune_session, "s", None) or S._get_session()
        if s is not None:
            s._pending_ckpt = Checkpoint.from_dict(Checkpoint.from_directory(self.dir).to_dict())
        shutil.rmtree(self.dir, ignore_errors=True)


def with_parameters(trainable, **kwargs):
    """Put large objects in the object store once; the trial fetches them (reference util.py)."""
    import ray_memory_management_amd as ray

    refs = {k: ray.put(v) for k, v in kwargs.items()}
    if isinstance(trainable, type) and issubclass(trainable, Trainable):
        base = trainable

        class _WithParams(base):
            def setup(self, config):
                extra = {k: ray.get(r) for k, r in refs.items()}
                return base.setup(self, config, **extra)

        _WithParams.__name__ = base.__name__
        return _WithParams

    def inner(config, checkpoint_dir=None):
        extra = {k: ray.get(r) for k, r in refs.items()}
        if "checkpoint_dir" in inspect.signature(trainable).parameters:
            return trainable(config, checkpoint_dir=checkpoint_dir, **extra)
        return trainable(config, **extra)

    inner.__name__ = getattr(trainable, "__name__", "with_parameters")
    inner._resources = getattr(trainable, "_resources", None)
    if "checkpoint_dir" not in inspect.signature(trainable).parameters:
        def inner2(config):
            return trainable(config, **{k: ray.get(r) for k, r in refs.items()})
        inner2.__name__ = inner.__name__
        inner2._resources = inner._resources
        return inner2
    return inner


class PlacementGroupFactory:
    """Per-trial resource request as bundles; bundle 0 hosts the trainable (reference
    tune/execution/placement_groups.py)."""

    def __init__(self, bundles, strategy: str = "PACK"):
        self.bundles = [dict(b) for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle(self):
        return self.bundles[0] if self.bundles else {}

    def required_resources(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0) + v
        return out

    def __eq__(self, o):
        return isinstance(o, PlacementGroupFactory) and o.bundles == self.bundles and o.strategy == self.strategy

    def __repr__(self):
        return f"PlacementGroupFactory({self.bundles}, {self.strategy!r})"


def resources_to_pgf(res) -> PlacementGroupFactory:
    if res is None:
        return PlacementGroupFactory([{"CPU": 1}])
    if isinstance(res, PlacementGroupFactory):
        return res
    if callable(res):
        return resources_to_pgf(res({}))
    r = dict(res)
    head = {"CPU": float(r.pop("cpu", r.pop("CPU", 1)))}
    gpu = float(r.pop("gpu", r.pop("GPU", 0)))
    if gpu:
        head["GPU"] = gpu
    extra_cpu = r.pop("extra_cpu", 0)
    extra_gpu = r.pop("extra_gpu", 0)
    r.pop("memory", None)
    custom = r.pop("custom_resources", {}) or {}
    head.update({k: float(v) for k, v in {**r, **custom}.items() if v})
    bundles = [head]
    if extra_cpu or extra_gpu:
        bundles.append({k: v for k, v in (("CPU", extra_cpu), ("GPU", extra_gpu)) if v})
    return PlacementGroupFactory(bundles)


def with_resources(trainable, resources):
    """Attach a per-trial resource request (dict, PlacementGroupFactory or fn(config))."""
    if isinstance(trainable, type):
        trainable = type(trainable.__name__, (trainable,), {})
        trainable._resources = resources
        return trainable

    def inner(*a, **k):
        return trainable(*a, **k)

    inner.__name__ = getattr(trainable, "__name__", "trainable")
    try:
        inner.__signature__ = inspect.signature(trainable)
    except (TypeError, ValueError):
        pass
    inner._resources = resources
    return inner
