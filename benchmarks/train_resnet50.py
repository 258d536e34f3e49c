"""Ray Train TorchTrainer ResNet-50 data-parallel benchmark (BASELINE.json config 3).

Parity: reference release/air_tests/air_benchmarks/workloads/torch_benchmark.py and
pytorch_training_e2e.py (TorchTrainer + prepare_model, SGD momentum, images/s). Here: one Train
worker actor per GPU, RCCL over xGMI for the gradient all-reduce, ResNet-50 in channels_last with
bf16 autocast (MIOpen NHWC implicit-GEMM on MFMA), synthetic 224x224 images generated on device
(no dataset access), random-init weights.

Usage: python benchmarks/train_resnet50.py --workers N --batch 256 --steps 30 --warmup 10
       [--strategy ddp|bucketed]   (prints one JSON line: images/s for the whole job)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def train_loop(config):
    import torch
    import torch.distributed as dist

    from ray_memory_management_amd.air import session
    from ray_memory_management_amd.models import resnet50
    from ray_memory_management_amd.train.torch import get_device, prepare_model

    dev = get_device()
    # MIOpen immediate mode (heuristic kernel choice): exhaustive find-mode tuning of every ResNet
    # conv costs minutes on a fresh box
    torch.backends.cudnn.benchmark = bool(config.get("tune", False))
    log = open(config["log"], "a") if config.get("log") else None

    def progress(msg):
        if log:
            log.write(f"[rank {session.get_world_rank()}] {time.strftime('%H:%M:%S')} {msg}\n")
            log.flush()
    torch.manual_seed(0)
    model = resnet50(num_classes=1000).to(dev, memory_format=torch.channels_last)
    model = prepare_model(model, parallel_strategy=config["strategy"] if session.get_world_size() > 1 else None)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    b = config["batch"]
    g = torch.Generator(device=dev).manual_seed(1234 + session.get_world_rank())
    x = torch.randn(b, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (b,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()
    progress("model and data ready")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(model(x), y)
        loss.backward()
        opt.step()
        return loss

    for i in range(config["warmup"]):
        step()
        torch.cuda.synchronize()
        progress(f"warmup step {i} done")
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(config["steps"]):
        loss = step()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = time.perf_counter() - t0
    progress(f"timed {config['steps']} steps in {el:.3f}s")
    if dist.is_initialized():
        e = torch.tensor([el], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    session.report({"elapsed_s": el, "loss": float(loss), "images": b * config["steps"] * session.get_world_size()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--strategy", default="ddp", choices=["ddp", "bucketed"])
    ap.add_argument("--tune", action="store_true", help="MIOpen find mode (cudnn.benchmark)")
    ap.add_argument("--log", default=os.path.join(ROOT, "gpurun_out", "resnet50_progress.log"))
    a = ap.parse_args()

    os.makedirs(os.path.dirname(a.log), exist_ok=True)
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.air import RunConfig, ScalingConfig
    from ray_memory_management_amd.train.torch import TorchTrainer

    ray.init(num_cpus=max(2, a.workers + 1), num_gpus=a.workers,
             _system_config={"memory_monitor_refresh_ms": 0})
    import threading

    stop = threading.Event()

    def heartbeat():  # keep the run visibly alive while the workers warm up
        t0 = time.time()
        while not stop.wait(20):
            print(f"[train_resnet50] running {time.time() - t0:.0f}s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    try:
        tr = TorchTrainer(train_loop, train_loop_config={"batch": a.batch, "steps": a.steps, "warmup": a.warmup,
                                                         "strategy": a.strategy, "tune": a.tune,
                                                         "log": a.log},
                          scaling_config=ScalingConfig(num_workers=a.workers, use_gpu=True),
                          run_config=RunConfig(name="resnet50_bench"))
        res = tr.fit()
        if res.error:
            raise res.error
        m = res.metrics
        ips = m["images"] / m["elapsed_s"]
        print(json.dumps({"metric": "TorchTrainer ResNet-50 DDP training throughput", "value": round(ips, 1),
                          "unit": "images/s", "n_gpus": a.workers, "per_gpu_batch": a.batch, "steps": a.steps,
                          "warmup": a.warmup, "ms_per_step": round(m["elapsed_s"] / a.steps * 1e3, 2),
                          "dtype": "bf16 autocast", "strategy": a.strategy, "loss": round(m["loss"], 4),
                          "data": "synthetic 224x224 on-device, random init"}), flush=True)
    finally:
        stop.set()
        ray.shutdown()


if __name__ == "__main__":
    main()
