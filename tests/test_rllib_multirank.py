"""Multi-rank PPO learner: replicas stay bit-identical. CPU: eager path over gloo (world 2).
GPU box: the fused/graph path with 2 ranks on one GPU over gloo (RCCL needs distinct GPUs)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, device, out_q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner

    torch.manual_seed(100 + rank)  # different init per rank: the learner must broadcast rank 0's
    env = GPUSyntheticAtariVectorEnv(4, device, num_actions=4, seed=rank)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 8, "num_sgd_iter": 2}, device=device,
                   action_space=env.action_space)
    S = GPURolloutSampler(env, L.model, fragment=4)
    for _ in range(2):
        st = L.update(S.sample())
    w = torch.cat([p.detach().float().reshape(-1).cpu() for p in L.model.parameters()])
    ws = [torch.zeros_like(w) for _ in range(world)]
    dist.all_gather(ws, w)
    out_q.put((rank, all(torch.equal(ws[0], x) for x in ws), st["kl"]))
    dist.destroy_process_group()


def _run(device, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, device, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(60)
    return res


def test_learner_replicas_identical_cpu_gloo():
    res = _run("cpu")
    assert all(r[1] for r in res)
    assert len({round(r[2], 8) for r in res}) == 1  # identical global stats on every rank


@pytest.mark.gpu
def test_learner_replicas_identical_gpu_fused_gloo():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run("cuda:0")
    assert all(r[1] for r in res)


@pytest.mark.gpu
def test_bench_two_ranks_same_gpu():
    """bench.py's distributed path (2 ranks, rehearsal on one GPU with gloo)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--no-putget", "--dist-backend", "gloo", "--same-device",
           "--mode", "fused", "--fragment", "100", "--minibatch", "500", "--sgd-iters", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert all(v == v for v in out["last_stats"].values() if isinstance(v, float))


@pytest.mark.gpu
def test_bench_runtime_two_learner_actors_same_gpu():
    """bench.py's runtime mode under torchrun: rank 0 drives 2 learner ACTORS (rehearsal: both on
    GPU 0 over gloo, the 8-GPU node uses RCCL), rank 1 only joins the timing barriers."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--no-putget", "--same-device", "--workers-per-learner", "2",
           "--sgd-iters", "2", "--store-gb", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["mode"] == "runtime"
    assert out["config"]["learner_actors"] == 2 and len(out["config"]["learners"]) == 2
