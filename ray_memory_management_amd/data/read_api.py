"""Dataset constructors. Parity: reference python/ray/data/read_api.py (from_items, range,
range_table, range_tensor, from_numpy(_refs), from_pandas(_refs), from_arrow(_refs),
from_huggingface, read_datasource, read_csv/json/parquet/numpy/text/binary_files)."""
from __future__ import annotations

import builtins
from typing import Any, List, Optional, Union

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.data.block import TENSOR_COL, BlockAccessor, BlockMetadata, NumpyBlock
from ray_memory_management_amd.data.context import DatasetContext
from ray_memory_management_amd.data.dataset import Dataset, ExecutionPlan
from ray_memory_management_amd.data import datasource as D


def _ensure_init():
    if not ray.is_initialized():
        ray.init()


def _from_blocks(blocks: List[Any], stage: str = "read") -> Dataset:
    refs = [ray.put(b) for b in blocks]
    metas = [BlockAccessor.for_block(b).get_metadata() for b in blocks]
    return Dataset(ExecutionPlan(refs, metas))


def _default_parallelism(n_items: Optional[int] = None) -> int:
    ctx = DatasetContext.get_current()
    cpus = int(ray.cluster_resources().get("CPU", 1))
    p = max(ctx.min_parallelism, 2 * cpus)
    p = min(p, ctx.default_parallelism)
    if n_items is not None:
        p = min(p, max(n_items, 1))
    return p


def from_items(items: List[Any], *, parallelism: int = -1) -> Dataset:
    _ensure_init()
    if parallelism <= 0:
        parallelism = _default_parallelism(len(items))
    n = len(items)
    per = max(-(-n // max(parallelism, 1)), 1)
    blocks = []
    is_dict = bool(items) and isinstance(items[0], dict)
    for s in builtins.range(0, n, per):
        chunk = items[s:s + per]
        if is_dict:
            import pyarrow as pa

            blocks.append(pa.Table.from_pylist(chunk))
        else:
            blocks.append(list(chunk))
    if not blocks:
        blocks = [[]]
    return _from_blocks(blocks, "from_items")


def read_datasource(datasource: D.Datasource, *, parallelism: int = -1, ray_remote_args=None,
                    **read_args) -> Dataset:
    _ensure_init()
    if parallelism <= 0:
        parallelism = _default_parallelism()
    tasks = datasource.prepare_read(parallelism, **read_args)
    remote_args = dict(ray_remote_args or {})

    @ray.remote
    def _read(task):
        from ray_memory_management_amd.data.block import concat_blocks

        blocks = list(task())
        b = concat_blocks(blocks) if blocks else []
        meta = BlockAccessor.for_block(b).get_metadata(input_files=task.get_metadata().input_files)
        return b, meta

    out_b, out_m = [], []
    for t in tasks:
        rb, rm = _read.options(num_returns=2, **remote_args).remote(t)
        out_b.append(rb)
        out_m.append(rm)
    if not out_b:
        return _from_blocks([[]])
    plan = ExecutionPlan(out_b, out_m)
    plan.source = (datasource, parallelism, ray_remote_args, dict(read_args))
    return Dataset(plan)


def range(n: int, *, parallelism: int = -1) -> Dataset:  # noqa: A001 - reference API name
    return read_datasource(D.RangeDatasource(), parallelism=parallelism if parallelism > 0 else
                           _default_parallelism(n), n=n, block_format="list")


def range_table(n: int, *, parallelism: int = -1) -> Dataset:
    return read_datasource(D.RangeDatasource(), parallelism=parallelism if parallelism > 0 else
                           _default_parallelism(n), n=n, block_format="arrow")


range_arrow = range_table


def range_tensor(n: int, *, shape=(1,), parallelism: int = -1) -> Dataset:
    return read_datasource(D.RangeDatasource(), parallelism=parallelism if parallelism > 0 else
                           _default_parallelism(n), n=n, block_format="tensor", tensor_shape=tuple(shape))


def from_numpy(ndarrays: Union[np.ndarray, List[np.ndarray]]) -> Dataset:
    _ensure_init()
    if isinstance(ndarrays, np.ndarray):
        ndarrays = [ndarrays]
    return _from_blocks([NumpyBlock({TENSOR_COL: a}) for a in ndarrays])


def from_numpy_refs(ndarrays) -> Dataset:
    _ensure_init()
    if isinstance(ndarrays, ray.ObjectRef):
        ndarrays = [ndarrays]

    @ray.remote
    def conv(a):
        b = NumpyBlock({TENSOR_COL: a})
        return b, BlockAccessor.for_block(b).get_metadata()

    pairs = [conv.options(num_returns=2).remote(r) for r in ndarrays]
    return Dataset(ExecutionPlan([p[0] for p in pairs], [p[1] for p in pairs]))


def from_pandas(dfs) -> Dataset:
    _ensure_init()
    import pandas as pd
    import pyarrow as pa

    if isinstance(dfs, pd.DataFrame):
        dfs = [dfs]
    return _from_blocks([pa.Table.from_pandas(df, preserve_index=False) for df in dfs])


def from_pandas_refs(dfs) -> Dataset:
    _ensure_init()
    if isinstance(dfs, ray.ObjectRef):
        dfs = [dfs]

    @ray.remote
    def conv(df):
        import pyarrow as pa

        b = pa.Table.from_pandas(df, preserve_index=False)
        return b, BlockAccessor.for_block(b).get_metadata()

    pairs = [conv.options(num_returns=2).remote(r) for r in dfs]
    return Dataset(ExecutionPlan([p[0] for p in pairs], [p[1] for p in pairs]))


def from_arrow(tables) -> Dataset:
    _ensure_init()
    import pyarrow as pa

    if isinstance(tables, (pa.Table, bytes)):
        tables = [tables]
    return _from_blocks(list(tables))


def from_arrow_refs(tables) -> Dataset:
    _ensure_init()
    if isinstance(tables, ray.ObjectRef):
        tables = [tables]

    @ray.remote
    def meta(t):
        return BlockAccessor.for_block(t).get_metadata()

    return Dataset(ExecutionPlan(list(tables), [meta.remote(t) for t in tables]))


def from_huggingface(dataset) -> Dataset:
    """A (local, already loaded) HuggingFace `datasets.Dataset` → Dataset via its Arrow table."""
    table = dataset.data.table if hasattr(dataset.data, "table") else dataset.data
    return from_arrow(table)


def read_csv(paths, *, parallelism: int = -1, ray_remote_args=None, **arrow_csv_args) -> Dataset:
    return read_datasource(D.CSVDatasource(), parallelism=parallelism, paths=paths, ray_remote_args=ray_remote_args,
                           **arrow_csv_args)


def read_json(paths, *, parallelism: int = -1, ray_remote_args=None, **arrow_json_args) -> Dataset:
    return read_datasource(D.JSONDatasource(), parallelism=parallelism, paths=paths,
                           ray_remote_args=ray_remote_args, **arrow_json_args)


def read_parquet(paths, *, columns: Optional[List[str]] = None, parallelism: int = -1, ray_remote_args=None,
                 **arrow_parquet_args) -> Dataset:
    return read_datasource(D.ParquetDatasource(), parallelism=parallelism, paths=paths, columns=columns,
                           ray_remote_args=ray_remote_args, **arrow_parquet_args)


read_parquet_bulk = read_parquet


def read_numpy(paths, *, parallelism: int = -1, **numpy_load_args) -> Dataset:
    return read_datasource(D.NumpyDatasource(), parallelism=parallelism, paths=paths, **numpy_load_args)


def read_text(paths, *, encoding: str = "utf-8", errors: Optional[str] = None, drop_empty_lines: bool = True,
              parallelism: int = -1, ray_remote_args=None) -> Dataset:
    return read_datasource(D.TextDatasource(), parallelism=parallelism, paths=paths, encoding=encoding,
                           errors=errors, drop_empty_lines=drop_empty_lines, ray_remote_args=ray_remote_args)


def read_binary_files(paths, *, include_paths: bool = False, parallelism: int = -1,
                      ray_remote_args=None) -> Dataset:
    return read_datasource(D.BinaryDatasource(), parallelism=parallelism, paths=paths, include_paths=include_paths,
                           ray_remote_args=ray_remote_args)


def read_images(paths, *, size=None, mode: Optional[str] = None, include_paths: bool = False, parallelism: int = -1,
                ray_remote_args=None) -> Dataset:
    """Image-folder dataset (reference ImageFolderDatasource via read_datasource): rows of
    {"image": HxWxC uint8 array, "label": class-directory name}."""
    return read_datasource(D.ImageFolderDatasource(), parallelism=parallelism, paths=paths, size=size, mode=mode,
                           include_paths=include_paths, ray_remote_args=ray_remote_args)


# --- integrations with other dataframe engines (reference read_api.py from_dask / from_modin /
# from_mars / from_spark): each converts the engine's partitions to pandas blocks. The engines are
# not installed in this image, so the import gate is what runs here; with the package present the
# partitions become one block each.
def _require(module: str, fn: str):
    import importlib

    try:
        return importlib.import_module(module)
    except ImportError as e:
        raise ImportError(f"{fn} needs the `{module}` package, which is not installed") from e


def from_dask(df) -> Dataset:
    _require("dask", "from_dask")
    return from_pandas([p.compute() for p in df.to_delayed()])


def from_modin(df) -> Dataset:
    _require("modin", "from_modin")
    from modin.distributed.dataframe.pandas.partitions import unwrap_partitions

    return from_pandas([ray.get(p) if isinstance(p, ray.ObjectRef) else p
                        for p in unwrap_partitions(df, axis=0)])


def from_mars(df) -> Dataset:
    _require("mars", "from_mars")
    return from_pandas(df.to_pandas())


def from_spark(df, *, parallelism: Optional[int] = None) -> Dataset:
    _require("pyspark", "from_spark")
    pdf = df.toPandas()
    n = parallelism or _default_parallelism(len(pdf))
    step = max(1, -(-len(pdf) // n))
    return from_pandas([pdf.iloc[i:i + step] for i in builtins.range(0, len(pdf), step)])
