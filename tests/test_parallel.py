"""parallel.BucketedAllReduce / all_reduce_coalesced on 2 gloo ranks (CPU): averaged gradients
must equal the mean of the per-rank gradients for every bucket size (incl. one param per bucket),
with unused parameters and repeated backward passes."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 8)
        self.unused = torch.nn.Linear(4, 4)

    def forward(self, x):
        return self.b(torch.relu(self.a(x)))


def _worker(rank, world, port, cap_mb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ray_memory_management_amd.parallel import BucketedAllReduce, all_reduce_coalesced

        torch.manual_seed(0)
        net = Net()
        ar = BucketedAllReduce(net.parameters(), bucket_cap_mb=cap_mb)
        assert len(ar.buckets) >= 1
        errs = []
        for it in range(2):
            net.zero_grad(set_to_none=True)
            torch.manual_seed(100 + rank + 10 * it)
            x = torch.randn(5, 16)
            net(x).square().sum().backward()
            got = {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None}
            # reference: local grads, all-reduced separately
            ref_net = Net()
            ref_net.load_state_dict(net.state_dict())
            ref_net(x).square().sum().backward()
            for n, p in ref_net.named_parameters():
                if p.grad is None:
                    continue
                g = p.grad.clone()
                dist.all_reduce(g)
                g /= world
                errs.append(float((got[n] - g).abs().max()))
        ts = [torch.full((7,), float(rank + 1)), torch.arange(5, dtype=torch.float32) * (rank + 1),
              torch.ones(3, 3, dtype=torch.float64)]
        all_reduce_coalesced(ts, average=True, bucket_cap_mb=1)
        errs.append(float((ts[0] - 1.5).abs().max()))
        errs.append(float((ts[1] - torch.arange(5) * 1.5).abs().max()))
        errs.append(float((ts[2] - 1.0).abs().max()))
        q.put((rank, max(errs)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cap_mb", [64, 1])
def test_bucketed_allreduce_matches_mean(cap_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cap_mb, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(30)
    assert all(p.exitcode == 0 for p in procs)
    assert max(res.values()) < 1e-5, res


def test_bucket_assignment_single_process():
    from ray_memory_management_amd.parallel import BucketedAllReduce

    net = Net()
    ar = BucketedAllReduce(net.parameters(), bucket_cap_mb=1)
    assert sum(len(b.params) for b in ar.buckets) == len(list(net.parameters()))
    # world == 1: hooks are no-ops, grads untouched
    net(torch.randn(2, 16)).sum().backward()
    assert net.a.weight.grad is not None
    ar.remove()
