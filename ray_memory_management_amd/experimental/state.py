"""Parity: reference python/ray/experimental/state/api.py (re-exported from util.state)."""
from ray_memory_management_amd.util.state import *  # noqa: F401,F403
