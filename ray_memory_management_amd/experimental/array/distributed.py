"""DistArray: a blocked matrix whose blocks are objects in the store (reference
experimental/array/distributed/core.py). Blocks are numpy arrays, or CUDA tensors with
device="cuda" (HBM object store; GEMMs on the GPU)."""
from __future__ import annotations

import itertools
from typing import List, Optional, Sequence

import numpy as np

import ray_memory_management_amd as ray

BLOCK_SIZE = 256


def _lib(device):
    if device == "cuda":
        import torch

        return torch
    return np


class DistArray:
    def __init__(self, shape: Sequence[int], object_refs=None, block_size: int = BLOCK_SIZE, device: str = "cpu"):
        self.shape = tuple(int(s) for s in shape)
        self.block_size = int(block_size)
        self.device = device
        self.num_blocks = [int(np.ceil(s / self.block_size)) for s in self.shape]
        self.object_refs = (np.empty(self.num_blocks, dtype=object) if object_refs is None
                            else np.asarray(object_refs, dtype=object))
        if self.object_refs.shape != tuple(self.num_blocks):
            raise ValueError(f"block grid {self.object_refs.shape} does not match {self.num_blocks}")

    @property
    def ndim(self):
        return len(self.shape)

    def block_shape(self, index):
        return tuple(min(self.block_size, s - i * self.block_size) for i, s in zip(index, self.shape))

    def assemble(self):
        """The whole array in this process (numpy, or a CUDA tensor for device="cuda")."""
        blocks = ray.get(list(self.object_refs.flat))
        grid = np.empty(self.num_blocks, dtype=object)
        for idx, b in zip(itertools.product(*[range(n) for n in self.num_blocks]), blocks):
            grid[idx] = b
        if self.device == "cuda":
            import torch

            if self.ndim == 1:
                return torch.cat(list(grid))
            return torch.cat([torch.cat(list(row), dim=1) for row in grid], dim=0)
        return np.block(grid.tolist()) if self.ndim > 1 else np.concatenate(list(grid))

    def __getitem__(self, idx):
        return self.object_refs[idx]


@ray.remote
def _fill(shape, kind, value, dtype_name, device, seed):
    if device == "cuda":
        import torch

        dt = getattr(torch, dtype_name)
        if kind == "normal":
            g = torch.Generator(device="cuda").manual_seed(int(seed))
            return torch.randn(shape, dtype=dt, device="cuda", generator=g)
        if kind == "eye":
            return torch.eye(shape[0], shape[1], dtype=dt, device="cuda") * value
        return torch.full(shape, float(value), dtype=dt, device="cuda")
    if kind == "normal":
        return np.random.default_rng(int(seed)).standard_normal(shape).astype(dtype_name)
    if kind == "eye":
        return (np.eye(shape[0], shape[1]) * value).astype(dtype_name)
    return np.full(shape, value, dtype=np.dtype(dtype_name))


def _make(shape, kind, value=0.0, dtype_name="float64", block_size=BLOCK_SIZE, device="cpu", seed=0):
    a = DistArray(shape, block_size=block_size, device=device)
    opts = {"num_gpus": 0.01} if device == "cuda" else {}
    for k, idx in enumerate(itertools.product(*[range(n) for n in a.num_blocks])):
        kd = kind
        if kind == "eye" and (len(idx) != 2 or idx[0] != idx[1]):
            kd = "full"
        a.object_refs[idx] = _fill.options(**opts).remote(a.block_shape(idx), kd, value if kd != "full" or kind != "eye"
                                                          else 0.0, dtype_name, device, seed * 1000003 + k)
    return a


def zeros(shape, dtype_name="float64", block_size=BLOCK_SIZE, device="cpu"):
    return _make(shape, "full", 0.0, dtype_name, block_size, device)


def ones(shape, dtype_name="float64", block_size=BLOCK_SIZE, device="cpu"):
    return _make(shape, "full", 1.0, dtype_name, block_size, device)


def eye(n, dtype_name="float64", block_size=BLOCK_SIZE, device="cpu"):
    return _make((n, n), "eye", 1.0, dtype_name, block_size, device)


class random:  # noqa: N801 - reference module name
    @staticmethod
    def normal(shape, dtype_name="float64", block_size=BLOCK_SIZE, device="cpu", seed=0):
        return _make(shape, "normal", 0.0, dtype_name, block_size, device, seed)


def numpy_to_dist(a, block_size=BLOCK_SIZE, device="cpu") -> DistArray:
    """Split a local array into blocks put into the store (CUDA tensors stay on the GPU)."""
    d = DistArray(tuple(a.shape), block_size=block_size, device=device)
    for idx in itertools.product(*[range(n) for n in d.num_blocks]):
        sl = tuple(slice(i * block_size, (i + 1) * block_size) for i in idx)
        blk = a[sl]
        d.object_refs[idx] = ray.put(blk.contiguous() if device == "cuda" else np.ascontiguousarray(blk))
    return d


@ray.remote
def _binary(op, a, b):
    return {"add": lambda: a + b, "subtract": lambda: a - b, "multiply": lambda: a * b}[op]()


@ray.remote
def _transpose_block(a):
    return a.T.contiguous() if hasattr(a, "contiguous") else np.ascontiguousarray(a.T)


@ray.remote
def _dot_sum(*pairs):
    """sum_k A_ik @ B_kj for the block row / column pairs handed in (all resolved by the runtime)."""
    half = len(pairs) // 2
    acc = None
    for a, b in zip(pairs[:half], pairs[half:]):
        p = a @ b
        acc = p if acc is None else acc + p
    return acc


def _elementwise(op, x: DistArray, y: DistArray) -> DistArray:
    if x.shape != y.shape or x.block_size != y.block_size:
        raise ValueError("elementwise ops need equal shapes and block sizes")
    out = DistArray(x.shape, block_size=x.block_size, device=x.device)
    opts = {"num_gpus": 0.01} if x.device == "cuda" else {}
    for idx in itertools.product(*[range(n) for n in x.num_blocks]):
        out.object_refs[idx] = _binary.options(**opts).remote(op, x.object_refs[idx], y.object_refs[idx])
    return out


def add(x, y):
    return _elementwise("add", x, y)


def subtract(x, y):
    return _elementwise("subtract", x, y)


def multiply(x, y):
    return _elementwise("multiply", x, y)


def transpose(x: DistArray) -> DistArray:
    if x.ndim != 2:
        raise ValueError("transpose needs a matrix")
    out = DistArray((x.shape[1], x.shape[0]), block_size=x.block_size, device=x.device)
    opts = {"num_gpus": 0.01} if x.device == "cuda" else {}
    for i, j in itertools.product(range(x.num_blocks[0]), range(x.num_blocks[1])):
        out.object_refs[j, i] = _transpose_block.options(**opts).remote(x.object_refs[i, j])
    return out


def dot(x: DistArray, y: DistArray) -> DistArray:
    """Blocked matrix product: one task per output block C_ij = Σ_k A_ik B_kj."""
    if x.ndim != 2 or y.ndim != 2 or x.shape[1] != y.shape[0] or x.block_size != y.block_size:
        raise ValueError(f"dot: incompatible {x.shape} @ {y.shape} (block sizes {x.block_size}, {y.block_size})")
    out = DistArray((x.shape[0], y.shape[1]), block_size=x.block_size, device=x.device)
    opts = {"num_gpus": 0.01} if x.device == "cuda" else {}
    K = x.num_blocks[1]
    for i, j in itertools.product(range(out.num_blocks[0]), range(out.num_blocks[1])):
        refs = [x.object_refs[i, k] for k in range(K)] + [y.object_refs[k, j] for k in range(K)]
        out.object_refs[i, j] = _dot_sum.options(**opts).remote(*refs)
    return out
