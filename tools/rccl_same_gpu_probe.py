"""Probe: can RCCL run several ranks on ONE GPU when each rank claims a different host?

RCCL rejects two ranks of one communicator on the same device of the same host ("Duplicate GPU
detected"). Giving every rank its own NCCL_HOSTID makes them look like separate hosts, so the
ranks talk through the socket transport over loopback. That is slow, but it runs the real RCCL
code path (communicator init, all_reduce, all_reduce inside a captured HIP graph) on a 1-GPU box.

Usage: python tools/rccl_same_gpu_probe.py [world]   (spawns `world` child processes)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import time


def child(rank: int, world: int, store_path: str):
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    store = dist.FileStore(store_path, world)
    t0 = time.time()
    dist.init_process_group("nccl", store=store, rank=rank, world_size=world, device_id=dev)
    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    assert float(x.min()) == want and float(x.max()) == want, (float(x.min()), want)
    init_s = time.time() - t0
    # all_reduce captured in a HIP graph, replayed
    s = torch.cuda.Stream()
    y = torch.zeros(4096, device=dev)
    with torch.cuda.stream(s):
        dist.all_reduce(y)  # warm the communicator on this stream
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y.add_(1.0)
        dist.all_reduce(y)
    y.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert float(y[0]) == world, float(y[0])
    # bandwidth of a 16 MiB bucket (socket transport: a functional path, not the xGMI number)
    b = torch.ones(4 << 20, device=dev)
    dist.all_reduce(b)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        dist.all_reduce(b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t1) / 5
    if rank == 0:
        print(f"rank0 ok: init+first all_reduce {init_s:.2f}s, graph replay ok, 16 MiB all_reduce {dt*1e3:.1f} ms",
              flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        return
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    store_path = tempfile.mktemp(prefix="rccl_probe_")
    procs = []
    for r in range(world):
        env = dict(os.environ, NCCL_HOSTID=f"rmm-rehearsal-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, __file__, "--child", str(r), str(world), store_path], env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = 1
    print("probe rc", rc, flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
