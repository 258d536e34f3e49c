"""Numpy routines as remote tasks (reference experimental/array/remote/core.py + linalg.py)."""
from __future__ import annotations

import numpy as np

import ray_memory_management_amd as ray


@ray.remote
def zeros(shape, dtype_name="float64"):
    return np.zeros(shape, dtype=np.dtype(dtype_name))


@ray.remote
def ones(shape, dtype_name="float64"):
    return np.ones(shape, dtype=np.dtype(dtype_name))


@ray.remote
def eye(n, m=None, dtype_name="float64"):
    return np.eye(n, m, dtype=np.dtype(dtype_name))


@ray.remote
def dot(a, b):
    return np.dot(a, b)


@ray.remote
def add(a, b):
    return np.add(a, b)


@ray.remote
def subtract(a, b):
    return np.subtract(a, b)


@ray.remote
def transpose(a):
    return np.transpose(a).copy()


@ray.remote
def sum(a, axis=None):  # noqa: A001 - numpy name
    return np.sum(a, axis=axis)


@ray.remote(num_returns=2)
def qr(a):
    q, r = np.linalg.qr(a)
    return q, r
