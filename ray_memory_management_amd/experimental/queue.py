"""Deprecated location of the actor-backed queue (reference python/ray/experimental/queue.py); use
``util.queue``."""
from ray_memory_management_amd.util.queue import Empty, Full, Queue  # noqa: F401

__all__ = ["Empty", "Full", "Queue"]
