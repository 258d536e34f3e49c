"""The framework-owned RCCL communicator (csrc/hip/rccl_comm.cc, parallel/comm.py:RcclComm).

GPU tests run 2 ranks on ONE MI355X: with RMM_RCCL_SAME_DEVICE=1 each rank claims its own RCCL host
id, so RCCL accepts both ranks on one device and connects them over its socket transport (the
8-GPU node uses xGMI; the code path above the transport is the same). Checked: all-reduce / broadcast
values, all-reduces forked onto the comm stream between graph replays (the PPO learner's multi-rank
SGD step), and 2 PPO learner actors whose gradient all-reduces keep the replicas bit-identical. Reference parity: util/collective/tests/single_node_gpu_tests/test_allreduce.py and
rllib/execution/tests/test_multi_gpu_learner_thread.py."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, sys
sys.path.insert(0, {root!r})
import torch
import torch.distributed as dist
from ray_memory_management_amd.parallel.comm import RcclComm
rank, world, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
torch.cuda.set_device(0)
c = RcclComm(dist.FileStore(path, world), rank, world, key="t")
dev = torch.device("cuda:0")
x = torch.full((1000,), float(rank + 1), device=dev, dtype=torch.bfloat16)
c.allreduce(x)
y = torch.full((3,), float(rank), device=dev)
c.allreduce(y, "max")
b = torch.arange(5, device=dev, dtype=torch.float32) * (rank + 1)
c.broadcast(b, 1)
torch.cuda.synchronize()
ok = float(x.float().min()) == world * (world + 1) / 2 and float(y[0]) == world - 1
ok = ok and torch.equal(b.cpu(), torch.arange(5, dtype=torch.float32) * 2)
# eager fork / join around graph replays (the learner's split-graph step): compute graph, the
# all-reduce forked onto the comm stream, more compute overlapping it, join, finishing graph
a = torch.zeros(4096, device=dev)
z = torch.zeros(16, device=dev)
g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    a.add_(0.0); z.add_(0.0); a.mul_(1.0)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(g1):
    a.add_(float(rank + 1))
with torch.cuda.graph(g2):
    z.add_(1.0)
with torch.cuda.graph(g3):
    a.mul_(0.5)
a.zero_()
for _ in range(3):
    g1.replay()
    h = c.allreduce_async(a)
    g2.replay()  # overlaps the collective
    h.wait()
    g3.replay()
torch.cuda.synchronize()
want = 0.0
for _ in range(3):
    want = (want * world + world * (world + 1) / 2) * 0.5
ok = ok and abs(float(a[0]) - want) < 1e-3 and float(z[0]) == 3.0
if os.environ.get("RMM_RCCL_IN_GRAPH") == "1":  # the collective captured inside one graph
    gg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gg, capture_error_mode=os.environ.get("RMM_CAPTURE_MODE", "thread_local")):
        cap = torch.cuda.current_stream()
        a.add_(1.0)
        if os.environ.get("RMM_RCCL_FORK", "1") == "1":
            c.stream.wait_stream(cap)
            c.allreduce_on(a, c.stream)
            cap.wait_stream(c.stream)
        else:
            c.allreduce_on(a, cap)
    a.zero_()
    gg.replay()
    torch.cuda.synchronize()
    ok = ok and float(a[0]) == world
c.check()
c.close()
print("RESULT", rank, ok, float(a[0]), want, flush=True)
"""


def _spawn(world=2, timeout=240, env=None):
    d = tempfile.mkdtemp(prefix="rccl_t_")
    script = os.path.join(d, "child.py")
    with open(script, "w") as f:
        f.write(_CHILD.format(root=ROOT))
    env = dict(os.environ, RMM_RCCL_SAME_DEVICE="1", **(env or {}))
    ps = [subprocess.Popen([sys.executable, script, str(r), str(world), os.path.join(d, "store")], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in ps:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in ps:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    return outs


def test_rehearsal_host_id_only_when_enabled(monkeypatch):
    from ray_memory_management_amd.parallel.comm import rehearsal_host_id

    monkeypatch.delenv("RMM_RCCL_SAME_DEVICE", raising=False)
    monkeypatch.delenv("NCCL_HOSTID", raising=False)
    rehearsal_host_id("g", 1)
    assert "NCCL_HOSTID" not in os.environ
    monkeypatch.setenv("RMM_RCCL_SAME_DEVICE", "1")
    rehearsal_host_id("g", 1)
    assert os.environ["NCCL_HOSTID"] == "rmm-g-1"


def test_rccl_binding_loads_and_makes_unique_ids():
    """The binding resolves RCCL from torch's librccl at run time (no GPU needed for this)."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    v = h.rccl_load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
    assert v >= 22000
    a, b = h.rccl_unique_id(), h.rccl_unique_id()
    assert len(a) == 128 and a != b
    assert h.NCCL_BFLOAT16 == 9 and h.NCCL_SUM == 0


@pytest.mark.gpu
def test_rccl_comm_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    outs = _spawn(2)
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
        line = [x for x in o.splitlines() if x.startswith("RESULT")][-1]
        assert line.split()[2] == "True", line


@pytest.mark.gpu
def test_ppo_learner_actors_rccl_identical(ray_start):
    """2 fused PPO learner actors on one GPU over the native RCCL communicator (bucket all-reduces
    forked onto the comm stream between the SGD step's graphs): the replicas stay bit-identical."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    ray.shutdown()
    os.environ["RMM_RCCL_SAME_DEVICE"] = "1"
    os.environ["RMM_PEER_COMM"] = "0"  # this test is about RCCL: the peer-memory comm would win on one GPU
    try:
        ray.init(num_cpus=6, num_gpus=1, object_store_memory=1 << 30, _system_config={"prestart_workers": 0})
        algo = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"num_actions": 4, "episode_len": 50})
                .rollouts(num_rollout_workers=2, num_envs_per_worker=4, rollout_fragment_length=25,
                          postprocess_on_learner=True)
                .training(train_batch_size=200, sgd_minibatch_size=100, num_sgd_iter=2, lr=1e-4)
                .resources(num_learner_workers=2, num_gpus_per_learner_worker=0.5,
                           learner_collective_backend="nccl")
                .debugging(seed=1)).build()
        try:
            for _ in range(2):
                r = algo.train()
            st = r["info"]["learner"]["default_policy"]["learner_stats"]
            assert np.isfinite(st["total_loss"]) and st["num_learners"] == 2
            info = ray.get([a.comm_info.remote() for a in algo.learner_group.learners])
            assert all(i["comm"] == "RcclComm" and (i["graph_has_comm"] or i["split_graphs"]) for i in info), info
            d = algo.learner_group.weights_digests()
            assert d[0] == d[1]
        finally:
            algo.stop()
    finally:
        os.environ.pop("RMM_RCCL_SAME_DEVICE", None)
        os.environ.pop("RMM_PEER_COMM", None)
