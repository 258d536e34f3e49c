"""Deprecated location of the multiprocessing Pool (reference python/ray/experimental/multiprocessing);
use ``util.multiprocessing``."""
from ray_memory_management_amd.util.multiprocessing import Pool  # noqa: F401

__all__ = ["Pool"]
