"""util.collective across actors. Mirrors reference python/ray/util/collective/tests (gloo on CPU here,
RCCL on the GPU box)."""
import pytest
import torch

import ray_memory_management_amd as ray
from ray_memory_management_amd.util import collective as col


class _WorkerBase:
    def __init__(self, device="cpu"):
        self.device = device

    def _collective_init(self, world_size, rank, backend, group_name):
        col.init_collective_group(world_size, rank, backend, group_name)
        return True

    def run(self, group):
        r = col.get_rank(group)
        n = col.get_collective_group_size(group)
        dev = self.device
        out = {}
        t = torch.full((4,), float(r + 1), device=dev)
        col.allreduce(t, group)
        out["allreduce"] = t.cpu().tolist()
        t = torch.full((2,), float(r), device=dev)
        col.allreduce(t, group, op=col.ReduceOp.MAX)
        out["max"] = t.cpu().tolist()
        t = torch.full((3,), float(r * 10), device=dev)
        col.broadcast(t, 1, group)
        out["bcast"] = t.cpu().tolist()
        lst = [torch.zeros(2, device=dev) for _ in range(n)]
        col.allgather(lst, torch.full((2,), float(r), device=dev), group)
        out["allgather"] = [x.cpu().tolist() for x in lst]
        parts = [torch.full((2,), float(r + i), device=dev) for i in range(n)]
        rs = torch.zeros(2, device=dev)
        col.reducescatter(rs, parts, group)
        out["reducescatter"] = rs.cpu().tolist()
        if r == 0:
            col.send(torch.arange(3, dtype=torch.float32, device=dev), 1, group)
        elif r == 1:
            buf = torch.zeros(3, device=dev)
            col.recv(buf, 0, group)
            out["recv"] = buf.cpu().tolist()
        col.barrier(group)
        col.destroy_collective_group(group)
        return out


Worker = ray.remote(num_cpus=0)(_WorkerBase)


def _check(outs, n):
    s = sum(range(1, n + 1))
    for r, o in enumerate(outs):
        assert o["allreduce"] == [float(s)] * 4
        assert o["max"] == [float(n - 1)] * 2
        assert o["bcast"] == [10.0] * 3
        assert o["allgather"] == [[float(i)] * 2 for i in range(n)]
        assert o["reducescatter"] == [float(sum(q + r for q in range(n)))] * 2
    assert outs[1]["recv"] == [0.0, 1.0, 2.0]


@pytest.mark.parametrize("n", [2, 3])
def test_gloo_collectives_between_actors(ray_start, n):
    ws = [Worker.remote() for _ in range(n)]
    col.create_collective_group(ws, n, list(range(n)), backend="gloo", group_name=f"g{n}")
    outs = ray.get([w.run.remote(f"g{n}") for w in ws])
    _check(outs, n)


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["nccl", "gloo"])
def test_gpu_tensor_collectives(backend, monkeypatch):
    """GPU tensors between actors over RCCL and gloo. With one GPU, the two RCCL ranks share it:
    RMM_RCCL_SAME_DEVICE=1 gives each rank its own RCCL host id (socket transport on loopback),
    so the full RCCL group path (init, all ops of `_WorkerBase.run`) still executes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ngpu = torch.cuda.device_count()
    same = backend == "nccl" and ngpu < 2
    if same:
        monkeypatch.setenv("RMM_RCCL_SAME_DEVICE", "1")  # inherited by the actors
    ray.init(num_cpus=2, num_gpus=ngpu, object_store_memory=256 << 20)
    try:
        G = ray.remote(num_gpus=1 if backend == "nccl" and not same else 0.5, num_cpus=0)(_WorkerBase)
        ws = [G.remote("cuda") for _ in range(2)]
        col.create_collective_group(ws, 2, [0, 1], backend=backend, group_name="gpu")
        outs = ray.get([w.run.remote("gpu") for w in ws], timeout=180)
        _check(outs, 2)
    finally:
        ray.shutdown()


@ray.remote(num_cpus=0)
class _Ops(_WorkerBase):
    def ops(self, group):
        r = col.get_rank(group)
        n = col.get_collective_group_size(group)
        out = {}
        t = torch.full((3,), float(r + 2))
        col.reduce(t, 1, group)  # only the destination holds the sum
        out["reduce"] = t.tolist()
        t = torch.full((2,), float(r + 2))
        col.allreduce(t, group, op=col.ReduceOp.PRODUCT)
        out["prod"] = t.tolist()
        t = torch.full((2,), float(r + 2))
        col.allreduce(t, group, op=col.ReduceOp.MIN)
        out["min"] = t.tolist()
        work = col.allreduce_async(torch.ones(5) * (r + 1), group)
        work.wait()
        inp = torch.arange(n * 2, dtype=torch.float32) + 100 * r
        o = torch.empty(n * 2)
        col.alltoall(o, inp, group_name=group)
        out["alltoall"] = o.tolist()
        # uneven splits: rank r sends (i + 1) rows to rank i
        ins = [i + 1 for i in range(n)]
        inp = torch.cat([torch.full((i + 1,), float(10 * r + i)) for i in range(n)])
        o = torch.empty((r + 1) * n)
        col.alltoall(o, inp, [r + 1] * n, ins, group_name=group)
        out["alltoall_v"] = o.tolist()
        try:
            col.send(torch.zeros(1), r, group)
        except RuntimeError as e:
            out["self_send"] = str(e)
        col.destroy_collective_group(group)
        out["after_destroy"] = (col.is_group_initialized(group), col.get_rank(group))
        return out

    def reinit(self, world, rank, group):
        col.init_collective_group(world, rank, "gloo", group)
        try:
            col.init_collective_group(world, rank, "gloo", group)
        except RuntimeError as e:
            dup = str(e)
        t = torch.tensor([float(rank)])
        col.allreduce(t, group)
        col.destroy_collective_group(group)
        return dup, float(t[0])


def test_gloo_reduce_product_min_alltoall_and_errors(ray_start):
    n = 3
    ws = [_Ops.remote() for _ in range(n)]
    col.create_collective_group(ws, n, list(range(n)), backend="gloo", group_name="ops")
    outs = ray.get([w.ops.remote("ops") for w in ws])
    assert outs[1]["reduce"] == [2.0 + 3.0 + 4.0] * 3
    for r, o in enumerate(outs):
        assert o["prod"] == [24.0, 24.0] and o["min"] == [2.0, 2.0]
        # alltoall: rank r receives slice r (2 rows) of every rank's input
        assert o["alltoall"] == [float(100 * s + 2 * r + j) for s in range(n) for j in range(2)]
        assert o["alltoall_v"] == [float(10 * s + r) for s in range(n) for _ in range(r + 1)]
        assert "current rank" in o["self_send"]
        assert o["after_destroy"] == (False, -1)


def test_group_join_inside_tasks_and_double_init_rejected(ray_start):
    ws = [_Ops.remote() for _ in range(2)]
    outs = ray.get([w.reinit.remote(2, i, "joined") for i, w in enumerate(ws)])
    for dup, s in outs:
        assert "twice" in dup and s == 1.0


def test_invalid_rank_and_uninitialized_group():
    with pytest.raises(ValueError):
        col.init_collective_group(2, 5, "gloo", "bad")
    with pytest.raises(RuntimeError, match="not initialized"):
        col.allreduce(torch.zeros(1), "missing")
    with pytest.raises(ValueError, match="_collective_init"):
        col.create_collective_group([object()], 1, [0], backend="gloo", group_name="x")
