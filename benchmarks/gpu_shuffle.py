"""GPU all-to-all shuffle throughput (BASELINE.json config 5: Exoshuffle of synthetic tensor blocks
across MI355X GPUs over RCCL/xGMI).

Run on N GPUs of one node:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 benchmarks/gpu_shuffle.py \
        --rows-per-gpu 8000000 --row-bytes 256 --rounds 5
Each rank holds rows_per_gpu rows (int64 key + row_bytes payload) in HBM; a round = K11 partition
+ counts all-to-all + keys/payload all-to-all (experimental/gpu_shuffle.py). Prints one JSON line:
whole-job GB/s of shuffled bytes (sum over ranks / max round time). Synthetic random keys.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-gpu", type=int, default=4_000_000)
    ap.add_argument("--row-bytes", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--backend", default="nccl")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from ray_memory_management_amd.experimental.gpu_shuffle import destinations, shuffle

    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if a.backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
    else:
        dev = torch.device("cpu")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group(a.backend, rank=rank, world_size=world,
                            **({"device_id": dev} if a.backend == "nccl" else {}))
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    keys = torch.randint(0, 2 ** 62, (a.rows_per_gpu,), device=dev, generator=g, dtype=torch.int64)
    vals = torch.randint(0, 256, (a.rows_per_gpu, a.row_bytes), device=dev, generator=g, dtype=torch.uint8)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier()

    for _ in range(a.warmup):
        shuffle(keys, vals)
    sync()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        k, v = shuffle(keys, vals)
    sync()
    el = (time.perf_counter() - t0) / a.rounds
    ok = bool((destinations(k, world) == rank).all().item())
    t = torch.tensor([el, 0.0 if ok else 1.0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        total = world * a.rows_per_gpu * (8 + a.row_bytes)
        print(json.dumps({"metric": "GPU all-to-all shuffle throughput", "value": round(total / t[0].item() / 1e9, 2),
                          "unit": "GB/s", "n_gpus": world, "rows_per_gpu": a.rows_per_gpu, "row_bytes": a.row_bytes,
                          "ms_per_round": round(t[0].item() * 1e3, 3), "correct": t[1].item() == 0.0,
                          "data": "synthetic random int64 keys + uint8 payload"}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
