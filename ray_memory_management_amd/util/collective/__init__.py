"""Collective communication between actors/tasks. Parity: reference python/ray/util/collective/
collective.py (init_collective_group, create_collective_group, allreduce, allgather, reducescatter,
broadcast, reduce, send/recv, barrier, destroy_collective_group), plus alltoall.

MI355X design: every named group is an independent torch.distributed process-group OBJECT
(``ProcessGroupNCCL`` = RCCL over xGMI for GPU tensors, ``ProcessGroupGloo`` for CPU tensors) built
directly on a rendezvous store — no global default group, so an actor can be in many groups. The
store is a FileStore in the session directory (node-local); ranks find it by group name.
"""
from ray_memory_management_amd.util.collective.collective import (  # noqa: F401
    Backend, ReduceOp, allgather, alltoall, allreduce_async, allgather_multigpu, allreduce, allreduce_multigpu, barrier, broadcast,
    broadcast_multigpu, create_collective_group, destroy_collective_group, get_collective_group_size,
    get_group_handle, get_rank, init_collective_group, is_group_initialized, nccl_available, gloo_available,
    recv, recv_multigpu, reduce, reduce_multigpu, reducescatter, reducescatter_multigpu, send, send_multigpu)
