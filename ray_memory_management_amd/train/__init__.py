"""Distributed training. Parity: reference python/ray/train/ (Trainer API of Ray AIR)."""
from ray_memory_management_amd.air.checkpoint import Checkpoint  # noqa: F401
from ray_memory_management_amd.air.config import (CheckpointConfig, FailureConfig, RunConfig,  # noqa: F401
                                                  ScalingConfig)
from ray_memory_management_amd.air.result import Result  # noqa: F401
from ray_memory_management_amd.air import session  # noqa: F401
from ray_memory_management_amd.train.base_trainer import BaseTrainer, DataParallelTrainer  # noqa: F401
from ray_memory_management_amd.train.batch_predictor import BatchPredictor  # noqa: F401
from ray_memory_management_amd.train.predictor import Predictor  # noqa: F401
from ray_memory_management_amd.train.trainer import (  # noqa: F401  (v1 API)
    TRAIN_DATASET_KEY, BackendConfig, CheckpointStrategy, Trainer, TrainingCallback, TrainingIterator,
    get_dataset_shard, load_checkpoint, local_rank, report, save_checkpoint, world_rank, world_size)


def __getattr__(name):
    import importlib

    if name in ("torch",):
        return importlib.import_module("ray_memory_management_amd.train.torch")
    if name == "TorchTrainer":
        return importlib.import_module("ray_memory_management_amd.train.torch").TorchTrainer
    if name == "TorchPredictor":
        return importlib.import_module("ray_memory_management_amd.train.predictor").TorchPredictor
    if name in ("sklearn", "rl"):
        return importlib.import_module(f"ray_memory_management_amd.train.{name}")
    raise AttributeError(name)
