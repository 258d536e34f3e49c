"""AIR common types. Parity: reference python/ray/air/{checkpoint,config,result,session}.py."""
from ray_memory_management_amd.air.checkpoint import Checkpoint  # noqa: F401
from ray_memory_management_amd.air.config import (CheckpointConfig, DatasetConfig, FailureConfig,  # noqa: F401
                                                  RunConfig, ScalingConfig)
from ray_memory_management_amd.air.result import Result  # noqa: F401
from ray_memory_management_amd.air import session  # noqa: F401

from typing import Dict as _Dict, Union as _Union  # noqa: E402

import numpy as _np  # noqa: E402

# reference air/data_batch_type.py: the batch formats predictors / preprocessors accept
DataBatchType = _Union[_np.ndarray, "pandas.DataFrame", "pyarrow.Table", _Dict[str, _np.ndarray]]
