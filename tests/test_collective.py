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
def test_gpu_tensor_collectives(backend):
    """GPU tensors between actors: RCCL needs one GPU per rank (skipped on a 1-GPU box);
    gloo over GPU tensors runs two ranks on one GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ngpu = torch.cuda.device_count()
    if backend == "nccl" and ngpu < 2:
        pytest.skip("RCCL rejects two ranks on one GPU; needs >= 2 GPUs")
    ray.init(num_cpus=2, num_gpus=ngpu, object_store_memory=256 << 20)
    try:
        G = ray.remote(num_gpus=1 if backend == "nccl" else 0.5, num_cpus=0)(_WorkerBase)
        ws = [G.remote("cuda") for _ in range(2)]
        col.create_collective_group(ws, 2, [0, 1], backend=backend, group_name="gpu")
        outs = ray.get([w.run.remote("gpu") for w in ws], timeout=180)
        _check(outs, 2)
    finally:
        ray.shutdown()
