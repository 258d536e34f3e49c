"""Headline benchmark: RLlib PPO training throughput (samples/s) on N MI355X through the runtime,
plus GPU object store put/get throughput (GB/s), per BASELINE.json.

Run: ``python bench.py --gpus N --steps K --warmup W``. For N>1 the driver launches N copies under
torch.distributed.run; rank 0 becomes the runtime's driver (``ray.init``) and the other ranks only
join the timing barriers (gloo, CPU) — they never touch a GPU, so each GPU holds exactly one
learner process.

Default mode ``runtime`` (BASELINE config "RLlib PPO, N GPU learner actors + CPU rollout workers,
synthetic 84x84 frames, sample-batch GPU ingest + GAE HIP scan"):

* ``PPO`` with ``num_learner_workers=N``: N learner ACTORS, one per GPU, each running the fused
  precision-matched fp32 learner (HIP graphs, hand-written split-bf16 MFMA kernels, fp32 master /
  gradients / Adam) and all-reducing gradients across GPUs (peer-memory kernel over xGMI, RCCL fallback);
* CPU rollout-worker ACTORS stepping the synthetic Atari vector env (native env core) on their CPU,
  with the policy on the worker's slice of the learner GPU (RLlib ``num_gpus_per_worker > 0``;
  default ``--rollout hybrid``): the whole fragment loop runs in C++ (csrc/hip/rollout_loop.cc) and
  every env step is one HIP-graph launch (K10 trunk reading the newest frames from mapped pinned
  memory → K13s dense → K16 heads + Gumbel sampling → actions into mapped pinned memory); ONE worker
  x 50 envs x 100 steps = 5000 samples per learner per iteration (atari-ppo.yaml: train_batch_size
  5000, rollout_fragment_length 100, sgd_minibatch_size 500, num_sgd_iter 10; its 10 workers x 5
  envs layout is what ``--rollout cpu`` runs, with the policy on the worker CPUs as
  num_gpus_per_worker: 0 does);
* fragments stay in HBM: rollout worker → HBM object store (hipIPC, same GPU) → learner, where
  GAE + advantage standardisation run as one kernel (K17); with N learners the gradient bucket is
  all-reduced by the peer-memory kernel (csrc/hip/peer_allreduce.hip) inside the chained SGD graph.

``--dtype fp32`` (default, the reference's precision: its torch PPO trains fp32,
rllib/algorithms/ppo/ppo_torch_policy.py:70): the learner and the rollout policy run the x3 kernels
(csrc/hip/x3_kernels.hip: every fp32 operand as a hi + lo bf16 pair, three bf16 MFMAs per product,
fp32 accumulation; fp32 master weights, gradients, loss and Adam) — gfx950 has no TF32 and its fp32 MFMA
runs at 1/16 of the bf16 rate. ``--dtype bf16``: bf16 operands (8 significant bits) with fp32 master
weights / Adam moments; at N=1 the fp32 run also reports it as ``runtime_bf16_samples_per_s``.

One timed step = one ``algo.train()`` iteration: sample 5000·N env steps, ingest, 10 epochs of
500-sample minibatch SGD on every learner, publish weights. Weak scaling (per-GPU batch fixed).
``value`` = whole-job env samples trained per second.

At N=1 the bench also reports (separately labelled, same K/W): ``runtime_cpu_rollout_*`` — the
same path with the policy on the rollout workers' CPUs (10 x 5 envs, the yaml's layout);
``runtime_gpu_rollout_*`` — one GPU rollout actor per learner (device env + on-GPU inference,
fragments through the HBM object store via hipIPC); ``fused_loop_samples_per_s`` — the
single-process fused loop (no runtime). ``--rollout {cpu,gpu}`` times those modes instead;
``--mode fused`` times the fused loop (torchrun for N>1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASE_PPO = 1250.0      # reference PPO Atari samples/s per GPU learner (weak anchor)
BASE_PUT_GBPS = 19.67  # reference single_client_put_gigabytes (host plasma)
METRIC = "GPU ray.put/get GB/s + RLlib PPO samples/sec at 1/2/4/8 MI355X"
TRAIN_BATCH = 5000     # atari-ppo.yaml, per learner


def _cpu_budget(n_gpus: int = 1) -> int:
    """CPUs this job may use: cgroup quota if any, else the affinity mask (and, where the GPU pool
    exports OMP_NUM_THREADS as the CPU share of ONE GPU, that share times the GPUs in use)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0 and n > 4 * int(omp) * max(1, n_gpus):
        n = min(n, int(omp) * max(1, n_gpus))
    return max(1, n)


def _rollout_layout(n_gpus: int, budget: int, fragment: int):
    """(workers per learner, envs per worker) with workers*envs*fragment == TRAIN_BATCH, as many
    workers (up to the reference's 10) as the CPU budget allows after 1 CPU per learner + 1."""
    per = max(1, (budget - 1) // n_gpus - 1)
    total_envs = TRAIN_BATCH // fragment
    for w in (10, 5, 2, 1):
        if w <= per and total_envs % w == 0:
            return w, total_envs // w
    return 1, total_envs


def _put_get_bench(dev_index: int, gb: float = 4.0, iters: int = 5):
    """GPU object store numbers (BASELINE config #2). Returns (put_get_GBps, details):
    put_get_GBps = same-process ray.put (HBM copy) + owner zero-copy get of one 4 GiB bf16 tensor;
    details = benchmarks/gpu_object_store_bench.py: put GB/s at 1 and 16 GiB, cross-process get
    (hipIPC, zero-copy) + full read, native spill / restore GB/s and bf16 compression ratio."""
    import torch

    import ray_memory_management_amd as ray
    from benchmarks import gpu_object_store_bench as gb_bench

    ray.init(num_cpus=2, num_gpus=1, object_store_memory=4 << 30,
             _system_config={"prestart_workers": 0, "memory_monitor_refresh_ms": 0,
                             "gpu_object_store_memory": 40 << 30})
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
        del t
        details = {}
        try:
            details.update(gb_bench.bench_put_get([1.0, 16.0], 3))
            details.update(gb_bench.bench_xproc(1.0, 3))
            from ray_memory_management_amd._private.worker import global_worker

            details.update(gb_bench.bench_spill(1.0, global_worker.store_name))
        except Exception as ex:  # noqa: BLE001
            details["error"] = repr(ex)
        return nel * 2 * iters / total / 1e9, details
    finally:
        ray.shutdown()


def _fused_loop(args, world, rank, local_rank, dist_backend):
    """Round-1 single-process fused PPO loop (no runtime): returns elapsed seconds for K steps."""
    import torch
    import torch.distributed as dist

    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner

    require_hip()
    if args.same_device:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(dist_backend, device_id=dev) if dist_backend == "nccl" else \
            dist.init_process_group(dist_backend)
    torch.manual_seed(1234 + rank)
    n_envs = TRAIN_BATCH // args.fragment
    env = GPUSyntheticAtariVectorEnv(n_envs, dev, num_actions=4, seed=rank)
    learner = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": args.minibatch, "num_sgd_iter": args.sgd_iters,
                                            "train_batch_size": TRAIN_BATCH,
                                            "compute_dtype": getattr(args, "dtype", "fp32")}, device=dev,
                         action_space=env.action_space)
    sampler = GPURolloutSampler(env, learner.model, fragment=args.fragment)
    for _ in range(args.warmup):
        learner.update(sampler.sample())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stats = learner.update(sampler.sample())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0, stats


def _worker_timing(algo):
    """Seconds the first rollout worker has spent in sample() so far (None if it does not report it)."""
    try:
        import ray_memory_management_amd as ray

        ws = algo.workers.remote_workers()
        return float(ray.get(ws[0].timing.remote())["sample_s"]) if ws else None
    except Exception:  # noqa: BLE001 - a worker class without timing()
        return None


def _runtime(args, n_gpus):
    """PPO through the runtime (rank 0 only). Returns (elapsed_s for K iterations, info)."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    budget = _cpu_budget(n_gpus)
    K = max(1, int(getattr(args, "learners_per_gpu", 1)))
    n_l = n_gpus * K          # learner actors (K share each GPU, each with its own rollout worker(s))
    per_l = TRAIN_BATCH // K  # samples per learner per iteration
    if args.rollout in ("cpu", "hybrid"):
        w_per, envs = _rollout_layout(n_l, budget, args.fragment)
        envs = max(1, per_l // (args.fragment * w_per))
        if args.rollout == "hybrid" and not args.workers_per_learner:
            # GPU policy: ONE worker x 50 envs per learner GPU measured best on MI355X with the native
            # rollout loop (profiles/native_rollout_r3.txt: 15.4-15.9 ms/iter vs 16.9-17.0 for 2 x 25
            # and 34-35 for 5 x 10): one policy step of all 50 envs per env step, one GPU context
            w_per, envs = 1, per_l // args.fragment
        if args.workers_per_learner:
            w_per = args.workers_per_learner
            envs = max(1, per_l // (args.fragment * w_per))
        # hybrid: --env-threads N gives each rollout worker N CPUs and splits its env steps over them
        # (native rollout loop); 1 by default (measured neutral, profiles/native_rollout_r3.txt)
        cpw = max(1, args.env_threads) if args.rollout != "cpu" else 1
        n_cpus = max(budget, n_l * (w_per * cpw + 1) + 1)
    else:
        w_per, envs, cpw = 1, per_l // args.fragment, 1
        n_cpus = max(budget, 2 * n_l + 1)
    phys = 1 if args.same_device else n_gpus
    # the runtime's processes (head, learner / rollout actors) do not inherit the launcher's torchrun
    # rendezvous variables: they form their own groups (util.collective), and a stray RANK /
    # WORLD_SIZE / MASTER_* must never be mistaken for theirs
    saved = {k: os.environ.pop(k) for k in list(os.environ)
             if k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                      "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")
             or k.startswith("TORCHELASTIC_")}
    if saved:
        print(f"[bench] runtime processes start without the launcher's {sorted(saved)}", file=sys.stderr)
    if (args.same_device or K > 1) and args.dist_backend == "nccl":
        # 1-GPU rehearsal of the RCCL learner group: every learner claims its own host id so RCCL
        # accepts several ranks on one device (socket transport over loopback; functional only)
        os.environ["RMM_RCCL_SAME_DEVICE"] = "1"
    ray.init(num_cpus=n_cpus, num_gpus=phys, object_store_memory=args.store_gb << 30,
             _system_config={"prestart_workers": 0})
    try:
        cfg = (PPOConfig()
               .environment("GPUSyntheticAtari-v0" if args.rollout == "gpu" else "SyntheticAtariVec-v0",
                            env_config={"num_actions": 4, "episode_len": 1000})
               .rollouts(num_rollout_workers=w_per * n_l, num_envs_per_worker=envs,
                         rollout_fragment_length=args.fragment, postprocess_on_learner=True, rollout_env_threads=cpw,
                         gpu_rollouts=args.rollout == "gpu")
               .training(train_batch_size=TRAIN_BATCH * n_gpus, sgd_minibatch_size=args.minibatch * n_gpus,
                         num_sgd_iter=args.sgd_iters, lr=5e-5, lambda_=0.95, kl_coeff=0.5, clip_param=0.1,
                         vf_clip_param=10.0, entropy_coeff=0.01, vf_loss_coeff=1.0, gamma=0.99,
                         compute_dtype=getattr(args, "dtype", "bf16"))
               .resources(num_learner_workers=n_l, num_cpus_per_worker=cpw,
                          num_gpus_per_learner_worker=(0.5 if args.rollout != "cpu" else 1.0) * phys / n_l,
                          # hybrid: CPU env, policy on the worker's slice of the learner's GPU
                          num_gpus_per_worker={"gpu": 0.5, "hybrid": 0.5 / w_per}.get(args.rollout, 0) * phys / n_l,
                          learner_collective_backend=args.dist_backend)
               .debugging(seed=0))
        algo = cfg.build()
        info = {"rollout_workers": w_per * n_l, "envs_per_worker": envs, "cpus_per_rollout_worker": cpw,
                "learner_actors": n_l, "learners_per_gpu": K,
                "cpu_budget": budget, "learners": algo.learner_group.device_info()}
        for _ in range(args.warmup):
            algo.train()
        if n_l > 1:  # communicator, peer mode and whether the optimizer step is the ZeRO-1 launch
            info["learner_comm"] = ray.get([a.comm_info.remote() for a in algo.learner_group.learners])
        dev = bool(getattr(algo, "_device_weights_ok", lambda: False)())
        info["weights_sync"] = ("shared-hbm" if dev and algo._shared_weights_ok() else "hbm-object" if dev
                                else "host")
        return algo, info
    except BaseException:
        ray.shutdown()
        raise


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=("runtime", "fused"), default="runtime")
    ap.add_argument("--rollout", choices=("cpu", "gpu", "hybrid"), default="hybrid",
                    help="cpu: CPU env + CPU policy (atari-ppo.yaml); hybrid: CPU env + policy on the rollout "
                         "worker's GPU slice (num_gpus_per_worker > 0); gpu: device env + GPU policy")
    ap.add_argument("--workers-per-learner", type=int, default=0)
    ap.add_argument("--env-threads", type=int, default=1, help="CPUs (env-step threads) per hybrid rollout worker")
    ap.add_argument("--fragment", type=int, default=100)
    ap.add_argument("--minibatch", type=int, default=500)
    ap.add_argument("--sgd-iters", type=int, default=10)
    ap.add_argument("--store-gb", type=int, default=8)
    ap.add_argument("--no-putget", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="skip the fused-loop reference number (N=1)")
    ap.add_argument("--no-gpu-rollout", action="store_true",
                    help="skip the extra runtime measurement with GPU rollout actors")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (=RCCL) or gloo (rehearsal)")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="fp32",
                    help="learner / GPU policy compute precision (fp32 = precision-matched with the reference)")
    ap.add_argument("--no-fp32", action="store_true", help="bf16 headline: skip the extra fp32 runtime measurement")
    ap.add_argument("--no-bf16", action="store_true", help="fp32 headline: skip the extra bf16 runtime measurement")
    ap.add_argument("--learners-per-gpu", type=int, default=1,
                    help="learner actors (data-parallel ranks, gradients averaged every SGD step) per GPU; the "
                         "per-GPU batch (5000) and minibatch (500) are split between them")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every learner on GPU 0 (RCCL ranks get distinct host ids "
                         "and use the socket transport; or --dist-backend gloo)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(args.gpus, world)
    out = None

    if args.mode == "fused":
        elapsed, stats = _fused_loop(args, world, rank, local_rank, args.dist_backend)
        import torch
        import torch.distributed as dist

        if world > 1:
            e = torch.tensor([elapsed], device=f"cuda:{0 if args.same_device else local_rank}")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        sps = TRAIN_BATCH * args.steps * world / elapsed
        mode_info = {"mode": "fused-loop", "note": "single process per GPU: on-device env + sampler + learner, "
                     "no runtime (actors / object store) in the timed region"}
    else:
        import torch.distributed as dist

        if world > 1:  # timing barriers only: CPU/gloo, the launcher ranks never touch a GPU
            dist.init_process_group("gloo")
        algo = info = None
        err = None
        if rank == 0:
            try:
                algo, info = _runtime(args, n_gpus)
            except BaseException as e:  # noqa: BLE001 - report after releasing the other ranks
                err = e
        tw0 = _worker_timing(algo) if rank == 0 and err is None else None
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        stats = {}
        iter_ms = []
        if rank == 0 and err is None:
            try:
                for _ in range(args.steps):
                    ti = time.perf_counter()
                    r = algo.train()  # learners end every update with a device sync
                    iter_ms.append(round((time.perf_counter() - ti) * 1e3, 3))
                stats = r["info"]["learner"]["default_policy"]["learner_stats"]
                # per-iteration wall times (inside the timed region, one perf_counter each): the spread
                # between iterations, reported next to the aggregate
                info["iter_ms"] = iter_ms
                # next iteration's samples queued behind the last update (RMM_PREFETCH_SAMPLE, shared weights)
                info["sample_prefetch"] = getattr(algo, "_prefetched", None) is not None
            except BaseException as e:  # noqa: BLE001
                err = e
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if tw0 is not None and err is None:  # after the timed region: mean sample() time per iteration
            tw1 = _worker_timing(algo)
            if tw1 is not None:
                info["worker_sample_ms"] = round((tw1 - tw0) / max(1, args.steps) * 1e3, 3)
        if world > 1:
            import torch

            e = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        if rank == 0:
            import ray_memory_management_amd as ray

            if algo is not None and err is None and len(algo.learner_group.learners) > 1:
                # after the timed region: data-parallel replicas must hold the same weights bit for bit
                try:
                    digests = ray.get([a.weights_digest.remote() for a in algo.learner_group.learners])
                    info["replicas_identical"] = len(set(digests)) == 1
                    info["learner_comm"] = ray.get([a.comm_info.remote() for a in algo.learner_group.learners])
                except Exception as ex:  # noqa: BLE001
                    info["replicas_check_error"] = repr(ex)[:300]
            if algo is not None:
                try:
                    algo.stop()
                except Exception:
                    pass
            ray.shutdown()
        if err is not None:
            if world > 1:
                dist.destroy_process_group()
            raise err
        sps = TRAIN_BATCH * n_gpus * args.steps / elapsed
        mode_info = {"mode": "runtime", "rollout": args.rollout,
                     "rollout_env": "gpu" if args.rollout == "gpu" else "cpu",
                     "rollout_policy_device": "cpu" if args.rollout == "cpu" else "gpu", **(info or {})}
        if world > 1:
            dist.destroy_process_group()

    if rank == 0:
        extra = {}
        if args.mode == "runtime" and n_gpus == 1 and not args.no_gpu_rollout and not args.same_device:
            # extra, clearly separate runtime measurements on the same config: (1) cpu — the CPU envs
            # with the policy on the rollout workers' CPUs (atari-ppo.yaml num_gpus_per_worker: 0);
            # (2) gpu — GPU rollout actors (device env + on-GPU inference), fragments through the
            # HBM object store (hipIPC)
            import copy

            import ray_memory_management_amd as ray

            modes = [m for m in ("cpu", "hybrid", "gpu") if m != args.rollout]
            if args.dtype == "bf16" and not args.no_fp32:
                modes.append("fp32")  # precision-matched learner + policy, same runtime path as `value`
            if args.dtype == "fp32" and not args.no_bf16:
                modes.append("bf16")  # bf16 operands, same runtime path as `value`
            for mode in modes:
                a2 = copy.copy(args)
                if mode in ("fp32", "bf16"):
                    a2.dtype = mode
                else:
                    a2.rollout = mode
                algo2 = None
                try:
                    algo2, info2 = _runtime(a2, n_gpus)
                    t0 = time.perf_counter()
                    for _ in range(args.steps):
                        algo2.train()
                    e2 = time.perf_counter() - t0
                    key = f"runtime_{mode}" if mode in ("fp32", "bf16") else f"runtime_{mode}_rollout"
                    extra[f"{key}_samples_per_s"] = round(TRAIN_BATCH * n_gpus * args.steps / e2, 1)
                    extra[f"{key}_ms_per_step"] = round(e2 / args.steps * 1e3, 3)
                except Exception as ex:  # noqa: BLE001
                    print(f"[bench] {mode}-rollout runtime mode failed: {ex!r}", file=sys.stderr)
                    extra[f"runtime_{mode}_rollout_error"] = repr(ex)[:300]
                finally:
                    if algo2 is not None:
                        try:
                            algo2.stop()
                        except Exception:
                            pass
                    ray.shutdown()
        if args.mode == "runtime" and n_gpus == 1 and world == 1 and not args.no_fused:
            try:
                import copy

                a2 = copy.copy(args)
                a2.warmup, a2.steps = 2, 10
                fe, _ = _fused_loop(a2, 1, 0, 0, "nccl")
                extra["fused_loop_samples_per_s"] = round(TRAIN_BATCH * a2.steps / fe, 1)
            except Exception as ex:  # noqa: BLE001
                print(f"[bench] fused loop failed: {ex!r}", file=sys.stderr)
        put_gbps, store_details = None, None
        if not args.no_putget and world == 1:
            try:
                put_gbps, store_details = _put_get_bench(0)
            except Exception as ex:  # noqa: BLE001
                print(f"[bench] put/get failed: {ex!r}", file=sys.stderr)
        out = {
            "metric": METRIC, "value": round(sps, 1), "unit": "samples/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(sps / BASE_PPO, 3), "dtype": args.dtype,
            "data": "synthetic 84x84x4 uint8 frames (vectorised synthetic Atari env), random-init weights",
            "config": {"model": "RLlib PPO VisionNetwork (Atari filters 16/32/256), atari-ppo.yaml hyper-parameters",
                       "global_batch": TRAIN_BATCH * n_gpus, "seq_len": args.fragment,
                       "parallelism": f"dp{n_gpus}" if args.learners_per_gpu <= 1 else
                       f"dp{n_gpus * args.learners_per_gpu} ({args.learners_per_gpu} learner ranks per GPU)",
                       "sgd_minibatch_size": args.minibatch,
                       "num_sgd_iter": args.sgd_iters, **mode_info},
            **extra,
            "put_get_GBps": None if put_gbps is None else round(put_gbps, 2),
            "put_get_note": "same-process put (HBM copy) + owner zero-copy get of one 4 GiB bf16 tensor",
            "gpu_object_store": store_details,
            "baseline_note": "vs_baseline divides by 1250 samples/s: RLlib 0.8.7 PPO Breakout, real emulator, "
                             "one V100 learner on a shared node (weak anchor, not like-for-like)",
            "last_stats": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in stats.items()
                           if isinstance(v, (int, float))},
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
