"""Tensor extension types for pandas and Arrow (reference python/ray/air/util/tensor_extensions)."""
from ray_memory_management_amd.air.util.tensor_extensions.arrow import ArrowTensorArray, ArrowTensorType  # noqa: F401
from ray_memory_management_amd.air.util.tensor_extensions.pandas import (  # noqa: F401
    TensorArray, TensorArrayElement, TensorDtype, column_needs_tensor_extension)
