"""Training worker actors + the driver-side loop that runs them in lock-step.

Parity: reference python/ray/train/_internal/{worker_group,backend_executor}.py and
python/ray/train/data_parallel_trainer.py. Each worker is an actor placed in one bundle of a
placement group (one GPU per worker on MI355X); ``Backend.on_start`` initialises the process group
(RCCL for GPUs), the user loop runs in a thread and ``session.report`` hands results to the driver.
"""
from __future__ import annotations

import os
import threading
import time
import traceback
from typing import Any, Callable, Dict, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.air import session as air_session
from ray_memory_management_amd.air.checkpoint import Checkpoint


@ray.remote(num_cpus=0)
class TrainWorker:
    def __init__(self):
        self.session = None
        self.thread = None
        self.done = None
        self.error = None

    def node_and_gpus(self):
        return ray.get_runtime_context().get_node_id(), ray.get_gpu_ids(), os.getpid()

    def execute(self, fn: Callable, *args, **kwargs):
        return fn(*args, **kwargs)

    def start(self, train_fn, config, rank, world_size, local_rank, local_world_size, node_rank, checkpoint,
              shards, trial_info):
        s = air_session._Session(rank, world_size, local_rank, local_world_size, node_rank, checkpoint, shards,
                                 **(trial_info or {}), config=config)
        air_session._set_session(s)
        self.session = s
        self.done = None

        def run():
            try:
                import inspect

                dev = os.environ.get("RMM_TRAIN_DEVICE_INDEX")
                if dev is not None:  # the CUDA current device is per thread: select this worker's GPU
                    import torch

                    torch.cuda.set_device(int(dev))
                    from ray_memory_management_amd._private.numa import pin_to_gpu

                    pin_to_gpu(int(dev))  # this worker (and its data-loader children) on the GPU's socket

                nparams = len(inspect.signature(train_fn).parameters)
                out = train_fn(config) if nparams >= 1 else train_fn()
                s.results.put(("done", out, None))
            except SystemExit:
                s.results.put(("done", None, None))
            except BaseException as e:  # noqa: BLE001
                s.results.put(("error", e, traceback.format_exc()))

        self.thread = threading.Thread(target=run, daemon=True)
        self.thread.start()
        return True

    def next_result(self):
        s = self.session
        kind, a, b = s.results.get()
        return kind, a, b

    def resume(self, stop: bool = False):
        s = self.session
        s.stop_requested = stop
        s.continue_event.set()
        return True

    def shutdown_backend(self, backend):
        try:
            backend.on_shutdown()
        except Exception:
            pass
        return True


class WorkerGroup:
    def __init__(self, num_workers: int, resources_per_worker: Dict[str, float], placement_strategy: str = "PACK"):
        from ray_memory_management_amd.util.placement_group import placement_group
        from ray_memory_management_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy

        self.num_workers = num_workers
        self.pg = placement_group([dict(resources_per_worker) for _ in range(num_workers)],
                                  strategy=placement_strategy)
        if not self.pg.wait(120):
            raise RuntimeError(f"could not place {num_workers} training workers with {resources_per_worker}")
        opts = {"num_cpus": resources_per_worker.get("CPU", 0), "num_gpus": resources_per_worker.get("GPU", 0)}
        extra = {k: v for k, v in resources_per_worker.items() if k not in ("CPU", "GPU")}
        if extra:
            opts["resources"] = extra
        self.workers = [TrainWorker.options(
            scheduling_strategy=PlacementGroupSchedulingStrategy(self.pg, i), **opts).remote()
            for i in range(num_workers)]
        info = ray.get([w.node_and_gpus.remote() for w in self.workers])
        self.node_ids = [i[0] for i in info]
        self.gpu_ids = [i[1] for i in info]
        # ranks ordered by node so local ranks are contiguous (reference sorts workers by node ip)
        order = sorted(range(num_workers), key=lambda i: (self.node_ids[i], i))
        self.workers = [self.workers[i] for i in order]
        self.node_ids = [self.node_ids[i] for i in order]
        self.gpu_ids = [self.gpu_ids[i] for i in order]

    def local_ranks(self):
        out, seen, node_rank = [], {}, {}
        for n in self.node_ids:
            out.append(seen.get(n, 0))
            seen[n] = seen.get(n, 0) + 1
            node_rank.setdefault(n, len(node_rank))
        return out, [seen[n] for n in self.node_ids], [node_rank[n] for n in self.node_ids]

    def execute(self, fn, *args, **kwargs):
        return ray.get([w.execute.remote(fn, *args, **kwargs) for w in self.workers])

    def shutdown(self):
        from ray_memory_management_amd.util.placement_group import remove_placement_group

        for w in self.workers:
            try:
                ray.kill(w)
            except Exception:
                pass
        remove_placement_group(self.pg)


class TrainingFailedError(RuntimeError):
    pass


def run_training(train_fn, config, backend, scaling, checkpoint: Optional[Checkpoint], datasets: dict,
                 on_report: Callable[[Dict[str, Any], Optional[Checkpoint]], None], trial_info=None,
                 max_failures: int = 0):
    """Start the group, run train_fn on every worker, feed rank-0 reports to `on_report`."""
    attempt = 0
    latest = checkpoint
    while True:
        group = WorkerGroup(scaling.num_workers or 1, scaling._resources_per_worker_not_none,
                            scaling.placement_strategy)
        try:
            backend.on_start(group)
            local, local_world, node_rank = group.local_ranks()
            n = group.num_workers
            shards = _split_datasets(datasets, n)
            ray.get([w.start.remote(train_fn, config, r, n, local[r], local_world[r], node_rank[r], latest,
                                    shards[r], trial_info) for r, w in enumerate(group.workers)])
            while True:
                outs = ray.get([w.next_result.remote() for w in group.workers])
                kinds = {o[0] for o in outs}
                if "error" in kinds:
                    err = next(o for o in outs if o[0] == "error")
                    raise TrainingFailedError(f"training function failed:\n{err[2]}") from err[1]
                if kinds == {"done"}:
                    ray.get([w.shutdown_backend.remote(backend) for w in group.workers])
                    return [o[1] for o in outs]
                if "done" in kinds:
                    raise TrainingFailedError("some workers finished while others reported: report() must be "
                                              "called the same number of times on every worker")
                metrics, ckpt = outs[0][1], outs[0][2]
                if ckpt is not None:
                    latest = ckpt
                stop = bool(on_report(metrics, ckpt))
                ray.get([w.resume.remote(stop) for w in group.workers])
        except ray.exceptions.RayActorError as e:
            attempt += 1
            if max_failures >= 0 and attempt > max_failures:
                raise TrainingFailedError(f"a training worker died ({e}); max_failures={max_failures} reached") from e
            time.sleep(0.5)
        finally:
            group.shutdown()


def _split_datasets(datasets: dict, n: int):
    out = [dict() for _ in range(n)]
    for name, ds in (datasets or {}).items():
        if hasattr(ds, "split"):
            parts = ds.split(n, equal=True)
        else:
            parts = [ds] * n
        for i in range(n):
            out[i][name] = parts[i]
    return out
