"""Multi-rank PPO learner step over PeerComm, one process per rank, without the runtime: the layout the
learner actors take on an 8-GPU node, rehearsed on however many GPUs the box has (ranks share GPU 0 when it
has one). Each rank runs the fused fp32 learner (x3 kernels) with PeerComm's ZeRO-1 optimizer launch inside
the chained SGD graphs; RMM_PEER_MODE=fork puts the dense + heads bucket's ZeRO-1 launch on the comm stream
beside the trunk backward. The ranks exit normally, so `rocprofv3 --kernel-trace` sees every rank's kernels
(tools/trace_overlap.py then reports how much of each ZeRO-1 launch overlapped the trunk backward).

usage: python benchmarks/peer_fork_probe.py [--world 2] [--updates 5] [--mbs 500]
Prints one JSON line: per-rank update ms, communicator info, and whether the replicas are bit-identical.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rank(rank: int, world: int, store_path: str, updates: int, mbs: int, out: str):
    import hashlib

    import torch
    import torch.distributed as dist

    from ray_memory_management_amd.parallel.comm import PeerComm
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    ngpu = torch.cuda.device_count()
    dev_idx = rank % max(1, ngpu)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    store = dist.FileStore(store_path, world)
    comm = PeerComm(store, rank, world, key="fork-probe", device=dev_idx)
    torch.manual_seed(0)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": mbs, "num_sgd_iter": 10, "train_batch_size": 5000,
                                      "compute_dtype": "fp32"}, device=dev, comm=comm)
    g = torch.Generator(device="cpu").manual_seed(100 + rank)  # each rank its own shard
    N, A = 5000, 4
    obs = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    cols = torch.cat([torch.randn(N, A, generator=g), torch.randn(N, 1, generator=g) - 1.4,
                      torch.randn(N, 2, generator=g), torch.randint(0, A, (N, 1), generator=g).float()], 1).to(dev)
    for _ in range(2):
        L._update_tables(obs, cols, A)
    torch.cuda.synchronize()
    ts = []
    for _ in range(updates):
        t0 = time.perf_counter()
        st = L._update_tables(obs, cols, A)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    comm.check()
    h = hashlib.sha256(L.master.detach().cpu().numpy().tobytes()).hexdigest()
    info = {"rank": rank, "device": dev_idx, "update_ms": [round(t, 2) for t in ts], "digest": h,
            "zero1": bool(L._zero1()), "peer_mode": L._peer_mode(), "zero1_blocks": comm.zero1_blocks,
            "ranks_on_device": comm.ranks_on_device, "graph_has_comm": bool(L._graph_has_comm),
            "loss": float(st["total_loss"])}
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(info, f)
    comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--updates", type=int, default=5)
    ap.add_argument("--mbs", type=int, default=500)
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--store", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.rank >= 0:
        _rank(a.rank, a.world, a.store, a.updates, a.mbs, a.out)
        return
    out = tempfile.mkdtemp(prefix="peer_fork_")
    store = os.path.join(out, "store")
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), "--world", str(a.world),
                               "--store", store, "--out", out, "--updates", str(a.updates), "--mbs", str(a.mbs)],
                              env=env) for r in range(a.world)]
    rcs = [p.wait(timeout=600) for p in procs]
    ranks = []
    for r in range(a.world):
        try:
            with open(os.path.join(out, f"rank{r}.json")) as f:
                ranks.append(json.load(f))
        except OSError:
            ranks.append({"rank": r, "missing": True})
    digests = {x.get("digest") for x in ranks}
    print(json.dumps({"world": a.world, "rcs": rcs, "replicas_identical": len(digests) == 1 and None not in digests,
                      "peer_mode_env": os.environ.get("RMM_PEER_MODE"), "ranks": ranks}), flush=True)
    sys.exit(0 if all(rc == 0 for rc in rcs) else 1)


if __name__ == "__main__":
    main()
