"""AIR utilities. Parity: reference python/ray/air/util/ (data_batch_conversion: convert a batch
between pandas / numpy / dict-of-numpy formats; check_ingest)."""
from ray_memory_management_amd.air.util.data_batch_conversion import (  # noqa: F401
    DataType, convert_batch_type_to_pandas, convert_pandas_to_batch_type)
