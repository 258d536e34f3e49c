"""Peer-memory all-reduce (csrc/hip/peer_allreduce.hip, parallel/comm.py:PeerComm).

GPU tests run several rank PROCESSES on one MI355X (the 1-GPU rehearsal of the 8-GPU node: the
same hipIPC export / map and flag protocol, the peer reads stay on one device instead of crossing
xGMI). Every rank checks its result bit-for-bit against the fp32 sum of the per-rank buffers in
rank order, rounded once (ray_memory_management_amd/parallel/peer_selftest.py). Reference parity:
util/collective/tests/single_node_gpu_tests/test_allreduce.py, rllib/execution/tests/
test_multi_gpu_learner_thread.py."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_peer_binding_and_decode_cpu():
    """The binding exists without a GPU; argument validation happens before any device call."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    assert hasattr(h, "PeerAllReduce")
    with pytest.raises(Exception):
        h.PeerAllReduce(3, 2, 0)  # rank >= world
    with pytest.raises(Exception):
        h.PeerAllReduce(0, 17, 0)  # > 16 ranks


def _selftest(world, timeout=300):
    d = tempfile.mkdtemp(prefix="peer_t_")
    r = subprocess.run([sys.executable, "-m", "ray_memory_management_amd.parallel.peer_selftest", "--world",
                        str(world), "--out", d, "--iters", "100"], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=dict(os.environ, PYTHONPATH=ROOT))
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert line, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(line[-1])
    bad = {rk["rank"]: {k: v for k, v in rk.get("cases", {}).items() if not v["ok"]} for rk in out["ranks"]}
    assert out["ok"], (bad, out["rcs"], r.stderr[-3000:])
    return out


@pytest.mark.gpu
def test_peer_allreduce_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _selftest(2)
    r0 = out["ranks"][0]
    print("peer all-reduce, 2 ranks / 1 GPU: bucket us eager %.1f graph %.1f, uncached signals %s"
          % (r0["bucket_us_eager"], r0["bucket_us_graph"], r0["uncached_signals"]))


@pytest.mark.gpu
def test_peer_allreduce_three_ranks_two_shot():
    """World 3 picks the two-shot (reduce-scatter + all-gather) kernel for the large cases."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _selftest(3)


@pytest.mark.gpu
@pytest.mark.parametrize("learners,mode", [(2, None), (3, None), (2, "fork"), (4, "fork")])
def test_ppo_learner_actors_peer_comm_in_graph(ray_start, learners, mode, monkeypatch):
    """2 / 3 fused PPO learner actors on one GPU over PeerComm: the optimizer step is the ZeRO-1 launch
    (reduce-scatter + Adam + all-gather; its bits equal all-reduce -> K6 in the peer self-test) INSIDE
    the chained SGD graph (chain > 1), and the replicas stay bit-identical. mode "fork": the layout ranks
    on separate GPUs take (dense bucket's launch on the comm stream beside the trunk backward, then the
    trunk bucket's), forced here on one GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if mode:
        monkeypatch.setenv("RMM_PEER_MODE", mode)
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    ray.shutdown()
    ray.init(num_cpus=8, num_gpus=1, object_store_memory=1 << 30, _system_config={"prestart_workers": 0})
    algo = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"num_actions": 4, "episode_len": 50})
            .rollouts(num_rollout_workers=learners, num_envs_per_worker=4, rollout_fragment_length=240 // (4 * learners),
                      postprocess_on_learner=True)
            .training(train_batch_size=240, sgd_minibatch_size=60, num_sgd_iter=2, lr=1e-4)
            .resources(num_learner_workers=learners, num_gpus_per_learner_worker=round(1.0 / learners, 3),
                       learner_collective_backend="nccl")
            .debugging(seed=1)).build()
    try:
        for _ in range(3):
            r = algo.train()
        st = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert np.isfinite(st["total_loss"]) and st["num_learners"] == learners
        info = ray.get([a.comm_info.remote() for a in algo.learner_group.learners])
        assert all(i["comm"] == "PeerComm" and i["graph_has_comm"] and i["chain"] > 1 and i["zero1"]
                   and i["peer_mode"] == (mode or "one") for i in info), info
        assert len({i["launches"] for i in info}) == 1 and info[0]["launches"] > 0, info
        # ZeRO-1 workgroups derived from the kernel's occupancy: every rank's workgroups resident together
        # beside one concurrent workgroup per CU (the trunk backward in fork mode)
        from ray_memory_management_amd._native import require_hip
        from ray_memory_management_amd.parallel.comm import zero1_blocks_for

        want = zero1_blocks_for(require_hip(), 0, learners)
        occ = require_hip().peer_occupancy(0)
        assert all(i["ranks_on_device"] == learners and i["zero1_blocks"] == want for i in info), (info, want)
        assert learners * want <= (occ["zero1_per_cu"] - 1) * occ["cus"], (occ, want)
        d = algo.learner_group.weights_digests()
        assert len(set(d)) == 1, d
    finally:
        algo.stop()
