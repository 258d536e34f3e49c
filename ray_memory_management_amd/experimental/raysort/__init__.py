"""Distributed sort benchmark (reference python/ray/experimental/raysort): see main.py
(``python -m ray_memory_management_amd.experimental.raysort.main``)."""
