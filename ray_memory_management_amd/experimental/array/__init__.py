"""Distributed arrays. Parity: reference python/ray/experimental/array/{remote,distributed}
(remote: numpy routines as tasks — zeros / ones / eye / dot / add / subtract / transpose / sum;
distributed: DistArray = a grid of block ObjectRefs (BLOCK_SIZE per side), numpy_to_dist /
assemble, elementwise ops and blocked dot as one task per output block, random.normal).

MI355X design: ``device="cuda"`` keeps every block a CUDA tensor, so blocks live in the HBM object
store (hipIPC between processes) and blocked GEMMs run on the tasks' GPU (hipBLASLt) with the
partial products summed on the device — a distributed matmul that never stages through host RAM.
"""
from ray_memory_management_amd.experimental.array import distributed, remote  # noqa: F401
