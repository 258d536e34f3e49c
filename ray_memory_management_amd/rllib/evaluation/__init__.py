from ray_memory_management_amd.rllib.evaluation.rollout_worker import RolloutWorker  # noqa: F401
from ray_memory_management_amd.rllib.evaluation.worker_set import WorkerSet  # noqa: F401
