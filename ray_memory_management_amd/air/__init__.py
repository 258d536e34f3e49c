"""AIR common types. Parity: reference python/ray/air/{checkpoint,config,result,session}.py."""
from ray_memory_management_amd.air.checkpoint import Checkpoint  # noqa: F401
from ray_memory_management_amd.air.config import (CheckpointConfig, DatasetConfig, FailureConfig,  # noqa: F401
                                                  RunConfig, ScalingConfig)
from ray_memory_management_amd.air.result import Result  # noqa: F401
from ray_memory_management_amd.air import session  # noqa: F401
