"""Sort kernels of the benchmark: key-range partitioning and merging of 100-byte records.

Parity: reference python/ray/experimental/raysort/sortlib.py (which delegates to a C++ extension).
Records are a uint8 ndarray [n, 100]. Partition r of R receives the keys whose big-endian 8-byte
prefix p satisfies floor(p·R / 2^64) == r — the same rule K11's "range" mode computes on the GPU
(csrc/hip/shuffle_kernels.hip), so host and device mappers produce identical partitions. Ordering
within a block is by the full 10-byte key (prefix, then the 2 trailing bytes).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ray_memory_management_amd.experimental.raysort.constants import KEY_SIZE, PREFIX_SIZE, RECORD_SIZE
from ray_memory_management_amd.experimental.raysort.types import BlockInfo


def key_prefix(records: np.ndarray) -> np.ndarray:
    """Big-endian u64 of each record's first 8 key bytes."""
    r = np.ascontiguousarray(records.reshape(-1, RECORD_SIZE)[:, :PREFIX_SIZE])
    return r.view(">u8").reshape(-1).astype(np.uint64)


def key_suffix(records: np.ndarray) -> np.ndarray:
    r = np.ascontiguousarray(records.reshape(-1, RECORD_SIZE)[:, PREFIX_SIZE:KEY_SIZE])
    return r.view(">u2").reshape(-1).astype(np.uint16)


def get_boundaries(num_parts: int) -> List[int]:
    """Lowest key prefix of each of `num_parts` equal ranges of the u64 prefix space."""
    return [(-(-(r << 64) // num_parts)) for r in range(num_parts)]


def range_of(prefix: np.ndarray, num_parts: int) -> np.ndarray:
    """floor(prefix · R / 2^64) without 128-bit arithmetic (R <= 2^31)."""
    R = np.uint64(num_parts)
    hi, lo = prefix >> np.uint64(32), prefix & np.uint64(0xFFFFFFFF)
    return ((hi * R + ((lo * R) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def sort_records(records: np.ndarray) -> np.ndarray:
    order = np.lexsort((key_suffix(records), key_prefix(records)))
    return records.reshape(-1, RECORD_SIZE)[order]


def sort_and_partition(part: np.ndarray, num_parts: int) -> List[BlockInfo]:
    """Sort `part` in place by key and return the (offset, size) in records of each key range."""
    recs = part.reshape(-1, RECORD_SIZE)
    recs[:] = sort_records(recs)
    dest = range_of(key_prefix(recs), num_parts)
    bounds = np.searchsorted(dest, np.arange(num_parts + 1), side="left")
    return [BlockInfo(int(bounds[r]), int(bounds[r + 1] - bounds[r])) for r in range(num_parts)]


def merge_partitions(blocks: Sequence[np.ndarray]) -> np.ndarray:
    """Merge sorted record blocks into one sorted block."""
    blocks = [b.reshape(-1, RECORD_SIZE) for b in blocks if len(b)]
    if not blocks:
        return np.empty((0, RECORD_SIZE), dtype=np.uint8)
    return sort_records(np.concatenate(blocks))


def checksum(records: np.ndarray) -> int:
    """Order-independent checksum: sum over records of a 64-bit mix of the record bytes."""
    recs = np.ascontiguousarray(records.reshape(-1, RECORD_SIZE))
    if not len(recs):
        return 0
    padded = np.zeros((len(recs), 104), dtype=np.uint8)
    padded[:, :RECORD_SIZE] = recs
    w = padded.view("<u8")  # 13 words per record
    with np.errstate(over="ignore"):
        h = np.full(len(recs), np.uint64(0x9E3779B97F4A7C15))
        for j in range(w.shape[1]):
            h ^= w[:, j]
            h *= np.uint64(0xBF58476D1CE4E5B9)
            h ^= h >> np.uint64(31)
        return int(h.sum(dtype=np.uint64))
