"""Collective groups over torch.distributed process-group objects (RCCL / gloo).

Parity: reference python/ray/util/collective/collective.py and collective_group/{nccl,gloo}_
collective_group.py. See the package docstring for the design."""
from __future__ import annotations

import enum
import os
import threading
import time
from datetime import timedelta
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class Backend(str, enum.Enum):
    NCCL = "nccl"   # RCCL on ROCm
    GLOO = "gloo"
    AUTO = "auto"


class ReduceOp(enum.Enum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3


_TORCH_OP = {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.PRODUCT: dist.ReduceOp.PRODUCT,
             ReduceOp.MIN: dist.ReduceOp.MIN, ReduceOp.MAX: dist.ReduceOp.MAX}


def nccl_available() -> bool:
    return hasattr(dist, "ProcessGroupNCCL") and torch.cuda.is_available()


def gloo_available() -> bool:
    return hasattr(dist, "ProcessGroupGloo")


class _Group:
    def __init__(self, name, world_size, rank, backend, pg, store):
        self.name = name
        self.world_size = world_size
        self.rank = rank
        self.backend = backend
        self.pg = pg
        self.store = store
        self.gloo_pg = None  # lazily-built CPU side channel for a GPU group (barrier / object ops)


_groups: Dict[str, _Group] = {}
_lock = threading.Lock()


def _store_path(group_name: str) -> str:
    from ray_memory_management_amd._private import worker as _w

    base = _w.global_worker.session_dir if _w.global_worker is not None else os.environ.get(
        "RMM_SESSION_DIR", "/tmp/rmm")
    d = os.path.join(base, "collective")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"group-{group_name}")


def _make_pg(backend, store, rank, world_size, timeout_s):
    if backend == Backend.NCCL:
        opts = dist.ProcessGroupNCCL.Options()
        opts._timeout = timedelta(seconds=timeout_s)
        return dist.ProcessGroupNCCL(store, rank, world_size, opts)
    return _gloo_pg(store, rank, world_size, timeout_s)


def _gloo_pg(store, rank, world_size, timeout_s):
    """A gloo group on the loopback interface: every rank of a util.collective group rendezvouses
    through a FileStore in the local session directory, i.e. lives on this host, and gloo's default
    (hostname-resolved) interface was measured 30-45x slower than loopback on the GPU boxes.
    GLOO_SOCKET_IFNAME overrides the choice."""
    iface = os.environ.get("GLOO_SOCKET_IFNAME") or "lo"
    try:
        opts = dist.ProcessGroupGloo._Options()
        opts._timeout = timedelta(seconds=timeout_s)
        opts._devices = [dist.ProcessGroupGloo.create_device(interface=iface)]
        return dist.ProcessGroupGloo(store, rank, world_size, opts)
    except Exception:  # interface missing / older torch: gloo's default device selection
        return dist.ProcessGroupGloo(store, rank, world_size, timedelta(seconds=timeout_s))


def init_collective_group(world_size: int, rank: int, backend=Backend.NCCL, group_name: str = "default",
                          timeout_s: float = 300.0) -> None:
    """Join a named group from inside an actor/task (every rank calls this)."""
    backend = Backend(backend) if not isinstance(backend, Backend) else backend
    if backend == Backend.AUTO:
        backend = Backend.NCCL if nccl_available() else Backend.GLOO
    if backend == Backend.NCCL and not nccl_available():
        raise RuntimeError("NCCL(RCCL) backend requested but no GPU is available; use backend='gloo'")
    if not (0 <= rank < world_size):
        raise ValueError(f"invalid rank {rank} for world_size {world_size}")
    with _lock:
        if group_name in _groups:
            raise RuntimeError(f"Trying to initialize a group twice: {group_name}")
    path = _store_path(group_name)
    store = dist.FileStore(path, world_size)
    if backend == Backend.NCCL and torch.cuda.is_available():
        torch.cuda.set_device(torch.cuda.current_device())
        from ray_memory_management_amd.parallel.comm import rehearsal_host_id

        rehearsal_host_id(group_name, rank)  # no-op unless RMM_RCCL_SAME_DEVICE=1 (1-GPU rehearsal)
    pg = _make_pg(backend, store, rank, world_size, timeout_s)
    with _lock:
        _groups[group_name] = _Group(group_name, world_size, rank, backend, pg, store)


def create_collective_group(actors: list, world_size: int, ranks: List[int], backend=Backend.NCCL,
                            group_name: str = "default") -> None:
    """Declare a group from the driver: each actor joins it via its ``__ray_init_collective__``-style
    hook — here by remotely calling ``init_collective_group`` through a helper method injected with
    `_collective_init` (the actor class must expose a method that calls init_collective_group)."""
    import ray_memory_management_amd as ray

    if len(actors) != len(ranks):
        raise ValueError("actors and ranks must have the same length")
    refs = []
    for a, r in zip(actors, ranks):
        if not hasattr(a, "_collective_init"):
            raise ValueError("actors passed to create_collective_group must define a "
                             "`_collective_init(world_size, rank, backend, group_name)` method")
        refs.append(a._collective_init.remote(world_size, r, str(Backend(backend).value), group_name))
    ray.get(refs)


def is_group_initialized(group_name: str = "default") -> bool:
    return group_name in _groups


def get_group_handle(group_name: str = "default") -> _Group:
    g = _groups.get(group_name)
    if g is None:
        raise RuntimeError(f"The collective group '{group_name}' is not initialized in the process.")
    return g


def destroy_collective_group(group_name: str = "default") -> None:
    with _lock:
        g = _groups.pop(group_name, None)
    if g is None:
        return
    try:
        if hasattr(g.pg, "shutdown"):
            g.pg.shutdown()
    except Exception:
        pass
    if g.rank == 0:
        try:
            os.unlink(_store_path(group_name))
        except OSError:
            pass


def get_rank(group_name: str = "default") -> int:
    g = _groups.get(group_name)
    return g.rank if g else -1


def get_collective_group_size(group_name: str = "default") -> int:
    g = _groups.get(group_name)
    return g.world_size if g else -1


def _opts(cls, **kw):
    o = cls()
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _pg_for(g: _Group, tensor):
    if g.backend == Backend.NCCL and not tensor.is_cuda:
        if g.gloo_pg is None:
            g.gloo_pg = _gloo_pg(dist.PrefixStore("gloo", g.store), g.rank, g.world_size, 300.0)
        return g.gloo_pg
    return g.pg


def allreduce(tensor, group_name: str = "default", op=ReduceOp.SUM):
    g = get_group_handle(group_name)
    _pg_for(g, tensor).allreduce([tensor], _opts(dist.AllreduceOptions, reduceOp=_TORCH_OP[op])).wait()
    return tensor


def allreduce_async(tensor, group_name: str = "default", op=ReduceOp.SUM):
    """Non-blocking all-reduce: returns the work handle (``.wait()``). On an RCCL group the
    collective runs on RCCL's stream after the caller's current stream; work issued before
    ``wait()`` overlaps it (used by the learners to hide gradient buckets behind backward)."""
    g = get_group_handle(group_name)
    return _pg_for(g, tensor).allreduce([tensor], _opts(dist.AllreduceOptions, reduceOp=_TORCH_OP[op]))


def allreduce_multigpu(tensor_list, group_name: str = "default", op=ReduceOp.SUM):
    for t in tensor_list:
        allreduce(t, group_name, op)
    return tensor_list


def barrier(group_name: str = "default"):
    g = get_group_handle(group_name)
    t = torch.zeros(1, device="cuda" if g.backend == Backend.NCCL else "cpu")
    allreduce(t, group_name)
    if t.is_cuda:
        torch.cuda.synchronize()


def reduce(tensor, dst_rank: int = 0, group_name: str = "default", op=ReduceOp.SUM):
    g = get_group_handle(group_name)
    _pg_for(g, tensor).reduce([tensor], _opts(dist.ReduceOptions, reduceOp=_TORCH_OP[op], rootRank=dst_rank,
                                              rootTensor=0)).wait()
    return tensor


def broadcast(tensor, src_rank: int = 0, group_name: str = "default"):
    g = get_group_handle(group_name)
    _pg_for(g, tensor).broadcast([tensor], _opts(dist.BroadcastOptions, rootRank=src_rank, rootTensor=0)).wait()
    return tensor


def broadcast_multigpu(tensor_list, src_rank: int = 0, src_tensor: int = 0, group_name: str = "default"):
    for t in tensor_list:
        broadcast(t, src_rank, group_name)
    return tensor_list


def allgather(tensor_list: list, tensor, group_name: str = "default"):
    g = get_group_handle(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("allgather: tensor_list length must equal the world size")
    _pg_for(g, tensor).allgather([tensor_list], [tensor]).wait()
    return tensor_list


def allgather_multigpu(output_tensor_lists, input_tensor_list, group_name: str = "default"):
    for out, inp in zip(output_tensor_lists, input_tensor_list):
        allgather(out, inp, group_name)
    return output_tensor_lists


def reducescatter(tensor, tensor_list: list, group_name: str = "default", op=ReduceOp.SUM):
    g = get_group_handle(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("reducescatter: tensor_list length must equal the world size")
    pg = _pg_for(g, tensor)
    if g.backend == Backend.NCCL and tensor.is_cuda:
        pg.reduce_scatter([tensor], [tensor_list], _opts(dist.ReduceScatterOptions, reduceOp=_TORCH_OP[op])).wait()
    else:
        # gloo has no reduce_scatter: all-reduce a concatenation, keep this rank's slice
        flat = torch.cat([t.reshape(-1) for t in tensor_list])
        pg.allreduce([flat], _opts(dist.AllreduceOptions, reduceOp=_TORCH_OP[op])).wait()
        n = tensor.numel()
        tensor.copy_(flat[g.rank * n:(g.rank + 1) * n].view_as(tensor))
    return tensor


def send(tensor, dst_rank: int, group_name: str = "default", tag: int = 0):
    g = get_group_handle(group_name)
    if dst_rank == g.rank:
        raise RuntimeError("The destination rank is the current rank.")
    _pg_for(g, tensor).send([tensor], dst_rank, tag).wait()


def recv(tensor, src_rank: int, group_name: str = "default", tag: int = 0):
    g = get_group_handle(group_name)
    if src_rank == g.rank:
        raise RuntimeError("The source rank is the current rank.")
    _pg_for(g, tensor).recv([tensor], src_rank, tag).wait()
    return tensor


def alltoall(output, input, output_split_sizes=None, input_split_sizes=None, group_name: str = "default"):
    """All-to-all along dim 0 (split sizes in rows; None = equal splits). RCCL on GPU groups: every
    pair of ranks exchanges its slice directly over xGMI. Parity: extends the reference's
    util.collective API (torch.distributed.all_to_all_single semantics)."""
    g = get_group_handle(group_name)
    pg = _pg_for(g, input)
    outs = list(output_split_sizes) if output_split_sizes is not None else []
    ins = list(input_split_sizes) if input_split_sizes is not None else []
    pg.alltoall_base(output, input, outs, ins, dist.AllToAllOptions()).wait()
    return output


# *_multigpu: the reference drives several GPUs from ONE process (NCCL group calls); here every GPU
# has its own process, so a rank holds one tensor per call and the list variants apply the
# single-tensor collective to each entry (one process per GPU is the supported layout).
def reduce_multigpu(tensor_list, dst_rank: int = 0, dst_tensor: int = 0, group_name: str = "default",
                    op=ReduceOp.SUM):
    for t in tensor_list:
        reduce(t, dst_rank, group_name, op)
    return tensor_list


def reducescatter_multigpu(output_tensor_list, input_tensor_lists, group_name: str = "default", op=ReduceOp.SUM):
    for out, ins in zip(output_tensor_list, input_tensor_lists):
        reducescatter(out, ins, group_name, op)
    return output_tensor_list


def send_multigpu(tensor, dst_rank: int, dst_gpu_index: int = 0, group_name: str = "default", n_elements: int = 0):
    send(tensor.reshape(-1)[:n_elements] if n_elements else tensor, dst_rank, group_name)


def recv_multigpu(tensor, src_rank: int, src_gpu_index: int = 0, group_name: str = "default", n_elements: int = 0):
    if n_elements:
        buf = tensor.reshape(-1)[:n_elements].contiguous()
        recv(buf, src_rank, group_name)
        tensor.reshape(-1)[:n_elements].copy_(buf)
    else:
        recv(tensor, src_rank, group_name)
    return tensor

