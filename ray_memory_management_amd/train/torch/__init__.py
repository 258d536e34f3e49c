"""Torch data-parallel training. Parity: reference python/ray/train/torch/{config,torch_trainer,
train_loop_utils}.py (TorchTrainer, TorchConfig, prepare_model, prepare_data_loader, get_device,
accelerate/backward helpers, TorchCheckpoint).

MI355X design: one worker per GPU, process group over RCCL (backend "nccl" on ROCm) through a
file rendezvous in the session dir; DDP uses large gradient buckets (default 256 MB — a 7-link xGMI
ring is per-link bandwidth bound, so fewer, bigger all-reduces overlap better with backward) and
gradient_as_bucket_view to avoid a copy per step.
"""
from __future__ import annotations

import dataclasses
import os
from datetime import timedelta
from typing import Any, Dict, Optional

import torch

from ray_memory_management_amd.air.checkpoint import Checkpoint
from ray_memory_management_amd.air import session
from ray_memory_management_amd.train.base_trainer import Backend, DataParallelTrainer


@dataclasses.dataclass
class TorchConfig:
    backend: Optional[str] = None   # "nccl" (RCCL) for GPU workers, "gloo" for CPU
    init_method: str = "file"
    timeout_s: int = 1800
    ddp_bucket_cap_mb: int = 256


def _init_pg(rank, world, backend, path, timeout_s, device_index):
    import torch.distributed as dist

    if backend == "nccl" and world > 1:
        # every worker of the node sees the node's GPUs and selects its own (reference
        # backend_executor._share_cuda_visible_devices): RCCL peers get direct xGMI peer access
        from ray_memory_management_amd._private.gpu_visibility import share_node_devices

        device_index = share_node_devices()
    if torch.cuda.is_available() and backend == "nccl":
        torch.cuda.set_device(device_index)
        os.environ["RMM_TRAIN_DEVICE_INDEX"] = str(device_index)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(session.get_local_rank() if session._session else 0)
    if not dist.is_initialized():
        dist.init_process_group(backend, init_method=f"file://{path}", rank=rank, world_size=world,
                                timeout=timedelta(seconds=timeout_s))
    return True


def _destroy_pg():
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
    return True


class _TorchBackend(Backend):
    def __init__(self, cfg: TorchConfig):
        self.cfg = cfg

    def on_start(self, worker_group):
        import ray_memory_management_amd as ray
        from ray_memory_management_amd._private import worker as _w

        use_gpu = any(worker_group.gpu_ids)
        backend = self.cfg.backend or ("nccl" if use_gpu else "gloo")
        d = os.path.join(_w.global_worker.session_dir, "train")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"pg-{os.urandom(6).hex()}")
        n = worker_group.num_workers
        ray.get([w.execute.remote(_init_pg, r, n, backend, path, self.cfg.timeout_s, 0)
                 for r, w in enumerate(worker_group.workers)])

    def on_shutdown(self):
        _destroy_pg()


class TorchTrainer(DataParallelTrainer):
    def __init__(self, train_loop_per_worker, *, train_loop_config=None, torch_config: Optional[TorchConfig] = None,
                 scaling_config=None, run_config=None, datasets=None, preprocessor=None,
                 resume_from_checkpoint=None, dataset_config=None):
        super().__init__(train_loop_per_worker, train_loop_config=train_loop_config,
                         backend_config=torch_config or TorchConfig(), scaling_config=scaling_config,
                         run_config=run_config, datasets=datasets, preprocessor=preprocessor,
                         resume_from_checkpoint=resume_from_checkpoint)

    def _backend(self):
        return _TorchBackend(self.backend_config)


def get_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device(f"cuda:{torch.cuda.current_device()}")
    return torch.device("cpu")


def prepare_model(model: torch.nn.Module, move_to_device: bool = True, parallel_strategy: Optional[str] = "ddp",
                  parallel_strategy_kwargs: Optional[Dict[str, Any]] = None) -> torch.nn.Module:
    import torch.distributed as dist

    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    if _ACCEL["amp"]:
        model = _AutocastForward(model)
    if parallel_strategy and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        kw = {"bucket_cap_mb": 256, "gradient_as_bucket_view": True}
        kw.update(parallel_strategy_kwargs or {})
        if parallel_strategy == "bucketed":
            # our own overlapped bucketed all-reduce (ray_memory_management_amd.parallel)
            from ray_memory_management_amd.parallel import BucketedAllReduce

            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0)
            model._rmm_grad_sync = BucketedAllReduce(model.parameters(),
                                                     bucket_cap_mb=(parallel_strategy_kwargs or {}).get("bucket_cap_mb"))
            return model
        if parallel_strategy == "fsdp":
            from torch.distributed.fsdp import FullyShardedDataParallel

            return FullyShardedDataParallel(model, **(parallel_strategy_kwargs or {}))
        if dev.type == "cuda":
            kw["device_ids"] = [dev.index]
        model = torch.nn.parallel.DistributedDataParallel(model, **kw)
    return model


class _DeviceLoader:
    def __init__(self, loader, device):
        self.loader = loader
        self.device = device

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield _to(batch, self.device)


def _to(x, dev):
    if torch.is_tensor(x):
        return x.to(dev, non_blocking=True)
    if isinstance(x, (list, tuple)):
        return type(x)(_to(v, dev) for v in x)
    if isinstance(x, dict):
        return {k: _to(v, dev) for k, v in x.items()}
    return x


def prepare_data_loader(data_loader, add_dist_sampler: bool = True, move_to_device: bool = True):
    import torch.distributed as dist
    from torch.utils.data import DataLoader, DistributedSampler

    if add_dist_sampler and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        shuffle = not isinstance(data_loader.sampler, torch.utils.data.SequentialSampler)
        data_loader = DataLoader(data_loader.dataset, batch_size=data_loader.batch_size,
                                 sampler=DistributedSampler(data_loader.dataset, shuffle=shuffle),
                                 num_workers=data_loader.num_workers, collate_fn=data_loader.collate_fn,
                                 pin_memory=data_loader.pin_memory, drop_last=data_loader.drop_last)
    if move_to_device:
        return _DeviceLoader(data_loader, get_device())
    return data_loader


def backward(tensor):
    tensor.backward()


# --- accelerate / reproducibility / profiling (reference train/torch/train_loop_utils.py) ---------
_ACCEL = {"amp": False}


def accelerate(amp: bool = False) -> None:
    """Enable mixed precision for models / optimizers prepared after this call. On MI355X AMP means
    bf16 autocast (MFMA-native, same exponent range as fp32, so no loss scaler is needed)."""
    _ACCEL["amp"] = bool(amp)


class _AutocastForward(torch.nn.Module):
    def __init__(self, module: torch.nn.Module):
        super().__init__()
        self.module = module

    def forward(self, *a, **kw):
        dev = get_device().type
        with torch.autocast(device_type=dev, dtype=torch.bfloat16):
            out = self.module(*a, **kw)
        return _to_float(out)


def _to_float(x):
    if torch.is_tensor(x) and x.is_floating_point():
        return x.float()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_float(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_float(v) for k, v in x.items()}
    return x


class _AMPOptimizer:
    """Optimizer wrapper handed out by prepare_optimizer under accelerate(amp=True): bf16 needs no
    loss scaling, so step / zero_grad pass through; state_dict round-trips the inner optimizer."""

    def __init__(self, optimizer):
        self.optimizer = optimizer

    def __getattr__(self, name):
        return getattr(self.optimizer, name)

    def step(self, closure=None):
        return self.optimizer.step(closure)

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)


def prepare_optimizer(optimizer):
    return _AMPOptimizer(optimizer) if _ACCEL["amp"] else optimizer


def enable_reproducibility(seed: int = 0) -> None:
    """Seed every RNG and switch torch to deterministic algorithms (reference
    train.torch.enable_reproducibility); call at the top of the training function."""
    import os
    import random

    import numpy as np

    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True


class TorchWorkerProfiler:
    """torch.profiler inside a training worker (reference train/torch/train_loop_utils.py
    TorchWorkerProfiler): use `trace_handler` as the profiler's on_trace_ready and report
    `get_and_clear_profile_traces()` through the session; the driver-side callback writes them."""

    def __init__(self, trace_dir: Optional[str] = None):
        import tempfile

        self.trace_dir = trace_dir or tempfile.mkdtemp(prefix="rmm_torch_prof_")
        self.profiler_trace_filenames = []

    def trace_handler(self, p) -> None:
        import os

        from ray_memory_management_amd.air import session

        rank = session.get_world_rank() if session._get_session(warn=False) else 0
        name = os.path.join(self.trace_dir, f"worker_{rank}_epoch_{len(self.profiler_trace_filenames)}.pt.trace.json")
        p.export_chrome_trace(name)
        self.profiler_trace_filenames.append(name)

    def get_and_clear_profile_traces(self) -> Dict[str, Any]:
        out = {}
        for fn in self.profiler_trace_filenames:
            with open(fn) as f:
                out[fn.rsplit("/", 1)[-1]] = f.read()
        self.profiler_trace_filenames = []
        return {"_train_torch_profiler_traces": out}


class TorchCheckpoint(Checkpoint):
    @classmethod
    def from_state_dict(cls, state_dict):
        return cls.from_dict({"model": state_dict})

    @classmethod
    def from_model(cls, model, *, preprocessor=None):
        if hasattr(model, "module"):
            model = model.module
        return cls.from_dict({"model": model.state_dict(), "preprocessor": preprocessor})

    def get_model(self, model: Optional[torch.nn.Module] = None):
        d = self.to_dict()
        m = d["model"]
        if model is not None and isinstance(m, dict):
            model.load_state_dict(m)
            return model
        return m


from ray_memory_management_amd.train.predictor import TorchPredictor  # noqa: E402,F401
