"""multiprocessing.Pool drop-in running on actors. Parity: reference
python/ray/util/multiprocessing/{__init__,pool}.py (Pool, TimeoutError, JoinableQueue — the
reference re-exports the stdlib's; so does this package)."""
from multiprocessing import JoinableQueue  # noqa: F401

from ray_memory_management_amd.util.multiprocessing.pool import AsyncResult, Pool, TimeoutError  # noqa: F401

__all__ = ["Pool", "AsyncResult", "TimeoutError", "JoinableQueue"]
