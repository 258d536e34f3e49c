"""Distributed datasets. Parity: reference python/ray/data/__init__.py."""
from ray_memory_management_amd.data._internal import ActorPoolStrategy  # noqa: F401
from ray_memory_management_amd.data.aggregate import AggregateFn, Count, Max, Mean, Min, Std, Sum  # noqa: F401
from ray_memory_management_amd.data.block import BlockAccessor, BlockMetadata  # noqa: F401
from ray_memory_management_amd.data.context import DatasetContext  # noqa: F401
from ray_memory_management_amd.data.dataset import Dataset  # noqa: F401
from ray_memory_management_amd.data.dataset_pipeline import DatasetPipeline  # noqa: F401
from ray_memory_management_amd.data.datasource import Datasource, ReadTask  # noqa: F401
from ray_memory_management_amd.data.grouped_dataset import GroupedDataset  # noqa: F401
from ray_memory_management_amd.data.preprocessor import Preprocessor  # noqa: F401
from ray_memory_management_amd.data.read_api import (  # noqa: F401
    from_arrow, from_arrow_refs, from_dask, from_huggingface, from_items, from_mars, from_modin, from_numpy,
    from_numpy_refs, from_pandas, from_spark,
    from_pandas_refs, range, range_arrow, range_table, range_tensor, read_binary_files, read_csv, read_datasource,
    read_images,
    read_json, read_numpy, read_parquet, read_parquet_bulk, read_text)


def set_progress_bars(enabled: bool) -> bool:
    return False


__all__ = [
    "ActorPoolStrategy", "Dataset", "DatasetPipeline", "Datasource", "ReadTask", "from_items", "from_arrow",
    "from_arrow_refs", "from_numpy", "from_numpy_refs", "from_pandas", "from_pandas_refs", "from_huggingface",
    "range", "range_table", "range_arrow", "range_tensor", "read_text", "read_binary_files", "read_csv", "read_images",
    "read_datasource", "read_json", "read_numpy", "read_parquet", "read_parquet_bulk", "set_progress_bars",
    "from_dask", "from_modin", "from_mars", "from_spark",
    "Preprocessor", "DatasetContext", "GroupedDataset", "AggregateFn", "Count", "Sum", "Min", "Max", "Mean", "Std",
]
