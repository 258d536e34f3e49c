"""Headline benchmark: RLlib-style PPO training throughput (samples/s) on N MI355X + GPU object
store put/get throughput (GB/s), per BASELINE.json.

Run: ``python bench.py --gpus N --steps K --warmup W`` (N>1 under torch.distributed.run, one rank per
GPU, RCCL over xGMI). One "step" = one PPO training iteration on every rank: sample
train_batch_size=5000 env steps per GPU (50 vectorised envs x rollout_fragment_length 100, synthetic
84x84x4 uint8 frames generated on-device, policy inference on the GPU), GAE (HIP kernel), then
num_sgd_iter=10 epochs of 500-sample minibatch SGD with DDP all-reduce (reference Atari PPO config
rllib/tuned_examples/ppo/atari-ppo.yaml). Weak scaling: per-GPU batch is fixed.
`value` = whole-job env samples trained per second.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASE_PPO = 1250.0      # reference PPO Atari samples/s per GPU learner (anchor)
BASE_PUT_GBPS = 19.67  # reference single_client_put_gigabytes
METRIC = "GPU ray.put/get GB/s + RLlib PPO samples/sec at 1/2/4/8 MI355X"


def _put_get_bench(dev_index: int, gb: float = 4.0, iters: int = 5) -> float:
    """ray.put(cuda bf16 tensor) + ray.get through the real API; returns GB/s for this rank."""
    import torch

    import ray_memory_management_amd as ray

    ray.init(num_cpus=1, num_gpus=0, object_store_memory=512 << 20,
             _system_config={"prestart_workers": 0, "memory_monitor_refresh_ms": 0})
    try:
        nel = int(gb * (1 << 30)) // 2
        t = torch.randn(nel, device=f"cuda:{dev_index}", dtype=torch.bfloat16)
        r = ray.put(t)
        v = ray.get(r)
        assert v.shape == t.shape
        del v, r
        torch.cuda.synchronize()
        total = 0.0
        for _ in range(iters):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = ray.put(t)
            v = ray.get(r)
            torch.cuda.synchronize()
            total += time.perf_counter() - t0
            del v, r
        return nel * 2 * iters / total / 1e9
    finally:
        ray.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-envs", type=int, default=50)
    ap.add_argument("--fragment", type=int, default=100)
    ap.add_argument("--minibatch", type=int, default=500)
    ap.add_argument("--sgd-iters", type=int, default=10)
    ap.add_argument("--no-putget", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (=RCCL) or gloo (rehearsal)")
    ap.add_argument("--breakdown", action="store_true", help="time sampling and SGD phases separately")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (rehearsal only)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:  # rehearsal of the multi-rank path on a 1-GPU box (use --dist-backend gloo)
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner

    require_hip()
    torch.manual_seed(1234 + rank)
    env = GPUSyntheticAtariVectorEnv(args.num_envs, dev, num_actions=4, seed=rank)
    model = VisionNetwork(4)  # DDP broadcasts rank 0's weights at construction
    learner = PPOLearner(model, {"sgd_minibatch_size": args.minibatch, "num_sgd_iter": args.sgd_iters,
                                 "train_batch_size": args.num_envs * args.fragment},
                         device=dev, action_space=env.action_space)
    sampler = GPURolloutSampler(env, learner.model, fragment=args.fragment)

    phase = {"sample_s": 0.0, "update_s": 0.0}

    def step():
        if args.breakdown:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            batch = sampler.sample()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            st = learner.update(batch)
            torch.cuda.synchronize()
            phase["sample_s"] += t1 - t0
            phase["update_s"] += time.perf_counter() - t1
            return st
        batch = sampler.sample()
        return learner.update(batch)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stats = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    samples = args.num_envs * args.fragment * args.steps * world
    sps = samples / elapsed

    put_gbps = None
    if not args.no_putget:
        try:
            g = _put_get_bench(local_rank)
        except Exception as ex:  # report PPO even if the put/get phase fails
            print(f"[bench] put/get failed on rank {rank}: {ex!r}", file=sys.stderr)
            g = float("nan")
        if world > 1:
            gt = torch.tensor([g], device=dev)
            dist.all_reduce(gt, op=dist.ReduceOp.SUM)
            g = float(gt.item())
        put_gbps = g

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(sps, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(sps / BASE_PPO, 3), "dtype": "bf16",
            "data": "synthetic: on-device 84x84x4 uint8 frames (vectorised env), random-init weights",
            "config": {"model": "RLlib PPO VisionNetwork (Atari filters 16/32/256) + GPU object store put/get",
                       "global_batch": args.num_envs * args.fragment * world, "seq_len": args.fragment,
                       "parallelism": f"dp{world}", "sgd_minibatch_size": args.minibatch,
                       "num_sgd_iter": args.sgd_iters},
            "put_get_GBps": None if put_gbps is None else round(put_gbps, 2),
            "put_get_vs_baseline": None if put_gbps is None else round(put_gbps / BASE_PUT_GBPS, 2),
            "last_stats": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in stats.items()},
        }
        if args.breakdown:
            n = args.steps + args.warmup
            out["breakdown_ms"] = {k: round(v / n * 1e3, 3) for k, v in phase.items()}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
