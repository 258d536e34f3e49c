"""``data.extensions`` (reference python/ray/data/extensions/__init__.py): tensor columns for
pandas / Arrow blocks."""
from ray_memory_management_amd.air.util.tensor_extensions import (  # noqa: F401
    ArrowTensorArray, ArrowTensorType, TensorArray, TensorArrayElement, TensorDtype)

__all__ = ["TensorDtype", "TensorArray", "TensorArrayElement", "ArrowTensorType", "ArrowTensorArray"]
