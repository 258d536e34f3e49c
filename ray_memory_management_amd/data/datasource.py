"""Datasources: parallel reads as ReadTasks, parallel writes as per-block write tasks.

Parity: reference python/ray/data/datasource/{datasource.py (Datasource, ReadTask, Reader,
RangeDatasource, DummyOutputDatasource), file_based_datasource.py (path expansion, one read task
per file group, block write naming {dataset_uuid}_{block_index:06}.{ext}), csv_datasource.py,
json_datasource.py, parquet_datasource.py, numpy_datasource.py, binary_datasource.py,
text via read_text}.
"""
from __future__ import annotations

import io
import os
from typing import Any, Callable, Iterable, List, Optional

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.data.block import TENSOR_COL, BlockAccessor, BlockMetadata, NumpyBlock


class ReadTask:
    """A callable producing an iterable of blocks, plus the metadata known before reading."""

    def __init__(self, read_fn: Callable[[], Iterable[Any]], metadata: BlockMetadata):
        self._read_fn = read_fn
        self._metadata = metadata

    def get_metadata(self) -> BlockMetadata:
        return self._metadata

    def __call__(self) -> Iterable[Any]:
        return self._read_fn()


class Datasource:
    """Subclass and implement prepare_read (reads) and/or do_write (writes)."""

    def prepare_read(self, parallelism: int, **read_args) -> List[ReadTask]:
        raise NotImplementedError

    def create_reader(self, **read_args):
        ds = self

        class _Reader:
            def estimate_inmemory_data_size(self):
                return None

            def get_read_tasks(self, parallelism):
                return ds.prepare_read(parallelism, **read_args)

        return _Reader()

    def do_write(self, blocks: List[Any], metadata: List[BlockMetadata], **write_args) -> List[Any]:
        raise NotImplementedError

    def on_write_complete(self, write_results: List[Any], **kwargs) -> None:
        pass

    def on_write_failed(self, write_results: List[Any], error: Exception, **kwargs) -> None:
        pass


class RangeDatasource(Datasource):
    def prepare_read(self, parallelism: int, n: int, block_format: str = "list", tensor_shape=(1,),
                     column_name: Optional[str] = None):
        tasks = []
        parallelism = max(1, min(parallelism, n)) if n > 0 else 1
        per = -(-n // parallelism) if n else 0
        for start in range(0, max(n, 1), max(per, 1)):
            if n == 0:
                break
            count = min(per, n - start)

            def make(start=start, count=count):
                if block_format == "arrow":
                    import pyarrow as pa

                    return [pa.table({column_name or "value": np.arange(start, start + count)})]
                if block_format == "tensor":
                    v = np.arange(start, start + count).reshape((count,) + (1,) * len(tensor_shape))
                    v = np.ones((count,) + tuple(tensor_shape), dtype=np.int64) * v
                    return [NumpyBlock({column_name or TENSOR_COL: v})]
                return [list(range(start, start + count))]

            tasks.append(ReadTask(make, BlockMetadata(count, 8 * count, None)))
        return tasks


class DummyOutputDatasource(Datasource):
    """Counts written rows (reference test helper)."""

    def __init__(self):
        self.num_ok = 0
        self.num_failed = 0
        self.rows_written = 0

    def do_write(self, blocks, metadata, **kw):
        @ray.remote
        def count(b):
            return BlockAccessor.for_block(b).num_rows()

        return [count.remote(b) for b in blocks]

    def on_write_complete(self, write_results, **kw):
        self.num_ok += 1
        self.rows_written += sum(ray.get(write_results))

    def on_write_failed(self, write_results, error, **kw):
        self.num_failed += 1


# ---------------------------------------------------------------------- file based
def _expand_paths(paths, exts: Optional[List[str]] = None) -> List[str]:
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        p = os.path.expanduser(p)
        if p.startswith("local://"):
            p = p[len("local://"):]
        if os.path.isdir(p):
            for root, _, files in sorted(os.walk(p)):
                for f in sorted(files):
                    if f.startswith(".") or f.startswith("_"):
                        continue
                    if exts and not any(f.endswith(e) for e in exts):
                        continue
                    out.append(os.path.join(root, f))
        elif os.path.exists(p):
            out.append(p)
        else:
            raise FileNotFoundError(p)
    return out


class FileBasedDatasource(Datasource):
    _FILE_EXTENSIONS: Optional[List[str]] = None
    _WRITE_EXT = "bin"

    def _read_file(self, path: str, **reader_args) -> Any:
        raise NotImplementedError

    def prepare_read(self, parallelism: int, paths, filesystem=None, partition_filter=None,
                     meta_provider=None, **reader_args):
        files = _expand_paths(paths, self._FILE_EXTENSIONS if partition_filter is None else None)
        if partition_filter is not None:
            files = [f for f in files if partition_filter(f)]
        n = max(1, min(parallelism, len(files))) if files else 0
        groups = [files[i::n] for i in range(n)] if n else []
        tasks = []
        for g in groups:
            size = sum(os.path.getsize(f) for f in g)

            def make(g=g):
                return [self._read_file(f, **reader_args) for f in g]

            tasks.append(ReadTask(make, BlockMetadata(None, size, None, input_files=list(g))))
        return tasks

    def _write_block(self, f, block, **writer_args):
        raise NotImplementedError

    def do_write(self, blocks, metadata, path: str, dataset_uuid: str, filesystem=None, try_create_dir=True,
                 block_path_provider=None, **writer_args):
        if try_create_dir:
            os.makedirs(path, exist_ok=True)
        ds = self

        @ray.remote
        def write(block, i):
            if block_path_provider is not None:
                fname = block_path_provider(path, dataset_uuid=dataset_uuid, block=block, block_index=i,
                                            file_format=ds._WRITE_EXT)
                os.makedirs(os.path.dirname(fname) or ".", exist_ok=True)
            else:
                fname = os.path.join(path, f"{dataset_uuid}_{i:06}.{ds._WRITE_EXT}")
            ds._write_block_path(fname, block, **writer_args)
            return fname

        return [write.remote(b, i) for i, b in enumerate(blocks)]

    def _write_block_path(self, fname, block, **writer_args):
        with open(fname, "wb") as f:
            self._write_block(f, block, **writer_args)


class CSVDatasource(FileBasedDatasource):
    _WRITE_EXT = "csv"

    def _read_file(self, path, **reader_args):
        import pyarrow.csv as pcsv

        return pcsv.read_csv(path, **reader_args)

    def _write_block(self, f, block, **writer_args):
        BlockAccessor.for_block(block).to_pandas().to_csv(f, index=False, **writer_args)


class JSONDatasource(FileBasedDatasource):
    _WRITE_EXT = "json"

    def _read_file(self, path, **reader_args):
        import pyarrow.json as pjson

        return pjson.read_json(path, **reader_args)

    def _write_block(self, f, block, **writer_args):
        df = BlockAccessor.for_block(block).to_pandas()
        writer_args.setdefault("orient", "records")
        writer_args.setdefault("lines", True)
        f.write(df.to_json(**writer_args).encode())


class ParquetDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = None
    _WRITE_EXT = "parquet"

    def _read_file(self, path, columns=None, **reader_args):
        import pyarrow.parquet as pq

        return pq.read_table(path, columns=columns, **reader_args)

    def _write_block_path(self, fname, block, **writer_args):
        import pyarrow.parquet as pq

        pq.write_table(BlockAccessor.for_block(block).to_arrow(), fname, **writer_args)


class NumpyDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = [".npy"]
    _WRITE_EXT = "npy"

    def _read_file(self, path, **reader_args):
        return NumpyBlock({TENSOR_COL: np.load(path, allow_pickle=False)})

    def _write_block(self, f, block, column=TENSOR_COL, **writer_args):
        np.save(f, BlockAccessor.for_block(block).to_numpy(column), allow_pickle=False)


class TextDatasource(FileBasedDatasource):
    def _read_file(self, path, encoding="utf-8", errors=None, drop_empty_lines=True):
        with open(path, "rb") as f:
            lines = f.read().decode(encoding, errors or "strict").split("\n")
        return [ln for ln in lines if ln] if drop_empty_lines else lines


class BinaryDatasource(FileBasedDatasource):
    def _read_file(self, path, include_paths=False):
        with open(path, "rb") as f:
            data = f.read()
        return [(path, data)] if include_paths else [data]


class ImageFolderDatasource(FileBasedDatasource):
    """``root/<label>/<image>`` trees (reference data/datasource/image_folder_datasource.py):
    one row per image with an ``image`` array (H, W, C uint8; optionally resized / mode-converted
    with PIL) and its ``label`` (the sub-directory name)."""

    _FILE_EXTENSIONS = [".png", ".jpg", ".jpeg", ".bmp", ".gif", ".tif", ".tiff"]

    def prepare_read(self, parallelism: int, paths, filesystem=None, partition_filter=None, meta_provider=None,
                     **reader_args):
        roots = [paths] if isinstance(paths, str) else list(paths)
        for r in roots:
            if not os.path.isdir(r):
                raise ValueError(f"ImageFolderDatasource expects directories of class folders, got {r!r}")
        return super().prepare_read(parallelism, roots, filesystem, partition_filter, meta_provider, **reader_args)

    def _read_file(self, path, size=None, mode=None, include_paths=False, **kw):
        from PIL import Image

        with Image.open(path) as im:
            if mode is not None:
                im = im.convert(mode)
            if size is not None:
                im = im.resize((int(size[1]), int(size[0])))
            arr = np.asarray(im)
        label = os.path.basename(os.path.dirname(path))
        if size is None:  # shapes may differ: simple rows
            row = {"image": arr, "label": label}
            if include_paths:
                row["path"] = path
            return [row]
        cols = {"image": arr[None], "label": np.asarray([label])}
        if include_paths:
            cols["path"] = np.asarray([path])
        return NumpyBlock(cols)  # fixed shape: columnar tensor block


# --- remaining reference datasource names -------------------------------------------------------
class RandomIntRowDatasource(Datasource):
    """n rows x num_columns of random int64 (reference datasource.py RandomIntRowDatasource)."""

    def prepare_read(self, parallelism: int, n: int, num_columns: int):
        import numpy as np

        from ray_memory_management_amd.data.block import BlockMetadata

        tasks, k = [], max(1, min(parallelism, n))
        per = -(-n // k)
        for i in range(0, n, per):
            cnt = min(per, n - i)

            def make(cnt=cnt, seed=i):
                import pandas as pd

                rng = np.random.default_rng(seed)
                return [pd.DataFrame({f"c_{j}": rng.integers(0, 2 ** 62, cnt) for j in range(num_columns)})]

            tasks.append(ReadTask(make, BlockMetadata(cnt, 8 * cnt * num_columns, None)))
        return tasks


class SimpleTorchDatasource(Datasource):
    """Rows of a map-style torch Dataset (reference simple_torch_datasource.py); the factory is
    called inside each read task."""

    def prepare_read(self, parallelism: int, dataset_factory):
        from ray_memory_management_amd.data.block import BlockMetadata

        ds = dataset_factory()
        n = len(ds)
        k = max(1, min(parallelism, n))
        per = -(-n // k)
        tasks = []
        for lo in range(0, n, per):
            hi = min(n, lo + per)

            def make(lo=lo, hi=hi):
                d = dataset_factory()
                return [[d[i] for i in range(lo, hi)]]

            tasks.append(ReadTask(make, BlockMetadata(hi - lo, None, None)))
        return tasks


class Reader:
    """Reference datasource.Reader (lazy read planning): here prepare_read returns the tasks directly."""

    def estimate_inmemory_data_size(self):
        return None

    def get_read_tasks(self, parallelism: int):
        raise NotImplementedError


WriteResult = Any  # what do_write's tasks return (reference datasource.py WriteResult)
ParquetBaseDatasource = ParquetDatasource

from ray_memory_management_amd.data.partitioning import (  # noqa: E402,F401
    BaseFileMetadataProvider, BlockWritePathProvider, DefaultBlockWritePathProvider, DefaultFileMetadataProvider,
    DefaultParquetMetadataProvider, FastFileMetadataProvider, FileExtensionFilter, FileMetadataProvider,
    ParquetMetadataProvider, Partitioning, PartitionStyle, PathPartitionEncoder, PathPartitionFilter,
    PathPartitionParser)

