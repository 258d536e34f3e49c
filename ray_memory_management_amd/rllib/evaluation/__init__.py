"""Evaluation: rollout workers, samplers, sample-batch builders, episodes, metrics and
trajectory postprocessing. Parity: reference rllib/evaluation/__init__.py."""
from ray_memory_management_amd.rllib.algorithms.callbacks import Episode  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.metrics import collect_metrics  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.postprocessing import compute_advantages  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.rollout_worker import RolloutWorker  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.sample_batch_builder import (  # noqa: F401
    MultiAgentSampleBatchBuilder, SampleBatchBuilder)
from ray_memory_management_amd.rllib.evaluation.sampler import AsyncSampler, SyncSampler  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.worker_set import WorkerSet  # noqa: F401
from ray_memory_management_amd.rllib.sample_batch import MultiAgentBatch, SampleBatch  # noqa: F401

MultiAgentEpisode = Episode  # reference keeps the old name as an alias of Episode

__all__ = ["Episode", "MultiAgentEpisode", "RolloutWorker", "WorkerSet", "SampleBatch", "MultiAgentBatch",
           "SampleBatchBuilder", "MultiAgentSampleBatchBuilder", "SyncSampler", "AsyncSampler", "compute_advantages",
           "collect_metrics"]
