"""A minimal communicator handle for learners: all-reduce / broadcast on either the default
``torch.distributed`` group (torchrun ranks) or a ``util.collective`` group (learner actors whose
RCCL group was rendezvoused through the runtime).

Parity: the reference's multi-GPU learner averages tower gradients in-process
(rllib/execution/multi_gpu_learner_thread.py) and DD-PPO all-reduces with torch.distributed
(rllib/algorithms/ddppo/ddppo.py:_sample_and_train_torch_distributed). Here one object hides which
process group carries the collective so the fused PPO learner code is the same in both cases.

``allreduce(t, stream=...)`` can run the collective on a dedicated comm stream: the caller records
an event on its compute stream, the comm stream waits for it, and RCCL launches there — compute
that does not depend on the reduced buffer keeps running (the overlap the PPO learner uses to hide
the dense-bucket all-reduce behind the trunk backward).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


class _Done:
    def wait(self):
        return True


class Comm:
    world: int = 1
    rank: int = 0

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> None:
        raise NotImplementedError

    def allreduce_async(self, t: torch.Tensor, op: str = "sum"):
        """Start an all-reduce; returns a handle whose wait() orders the caller's current stream
        (RCCL) or host (gloo) after it. Compute issued before wait() overlaps the collective."""
        self.allreduce(t, op)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        pass


class LocalComm(Comm):
    """World of one: every collective is the identity."""

    def allreduce(self, t, op="sum"):
        return None

    def broadcast(self, t, src=0):
        return None


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchDistComm(Comm):
    """The default (or a registered) torch.distributed group."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def allreduce(self, t, op="sum"):
        dist.all_reduce(t, op=_OPS[op], group=self.group)

    def allreduce_async(self, t, op="sum"):
        return dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=True)

    def broadcast(self, t, src=0):
        g = dist.get_global_rank(self.group, src) if self.group is not None else src
        dist.broadcast(t, src=g, group=self.group)

    def barrier(self):
        dist.barrier(group=self.group)


class GroupComm(Comm):
    """A util.collective group (a bare ProcessGroup object: RCCL for GPU tensors, its gloo side
    channel for CPU tensors). Works identically in actors and plain processes."""

    def __init__(self, group_name: str):
        from ray_memory_management_amd.util.collective import collective as col

        self.name = group_name
        self._g = col.get_group_handle(group_name)
        self.world = self._g.world_size
        self.rank = self._g.rank

    def allreduce(self, t, op="sum"):
        from ray_memory_management_amd.util.collective import collective as col

        col.allreduce(t, self.name, {"sum": col.ReduceOp.SUM, "max": col.ReduceOp.MAX,
                                     "min": col.ReduceOp.MIN}[op])

    def allreduce_async(self, t, op="sum"):
        from ray_memory_management_amd.util.collective import collective as col

        return col.allreduce_async(t, self.name, {"sum": col.ReduceOp.SUM, "max": col.ReduceOp.MAX,
                                                  "min": col.ReduceOp.MIN}[op])

    def broadcast(self, t, src=0):
        from ray_memory_management_amd.util.collective import collective as col

        col.broadcast(t, src, self.name)

    def barrier(self):
        from ray_memory_management_amd.util.collective import collective as col

        col.barrier(self.name)


def default_comm(process_group=None) -> Comm:
    """torch.distributed when it is initialised (torchrun ranks), else a world of one."""
    if dist.is_available() and dist.is_initialized():
        c = TorchDistComm(process_group)
        if c.world > 1:
            return c
    return LocalComm()


def as_comm(x: Optional[object]) -> Comm:
    if x is None:
        return default_comm()
    if isinstance(x, Comm):
        return x
    if isinstance(x, str):
        return GroupComm(x)
    return default_comm(x)  # a torch.distributed ProcessGroup
