"""GPU tests of the runtime PPO path: K17 ingest vs the fp32 reference, the manual (overlap-ready)
SGD step vs the autograd step, K6b gradient clipping vs torch, a fused update vs an fp32 eager
reference on the same index table, a learnable task, and PPO with a GPU learner ACTOR fed by CPU
rollout workers through the object store."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fragments(T=20, n=5, A=4, k=3, seed=0):
    from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment

    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        out.append(pack_fragment(rng.integers(0, 256, size=(T, n, 4, 84, 84), dtype=np.uint8),
                                 rng.standard_normal((T, n, A)).astype(np.float32),
                                 rng.standard_normal((T, n)).astype(np.float32),
                                 rng.standard_normal((T, n)).astype(np.float32),
                                 (rng.random((T, n)) < 0.3).astype(np.float32),
                                 (rng.random((T, n)) < 0.1).astype(np.float32),
                                 rng.integers(0, A, size=(T, n)), rng.standard_normal(n).astype(np.float32)))
    return out


@pytest.mark.parametrize("T,n", [(20, 5), (100, 50), (3000, 2)])
def test_k17_ingest_matches_fp32_reference(cuda, T, n):
    from ray_memory_management_amd.rllib.execution.sample_ingest import SampleIngest, fragments_to_batch_cpu

    frags = _fragments(T, n, k=2)
    obs_ref, cols_ref = fragments_to_batch_cpu(frags, 0.99, 0.95, standardize=True)
    ing = SampleIngest(cuda, 0.99, 0.95)
    obs, cols = ing.ingest(frags, standardize=True)
    assert torch.equal(obs.cpu(), obs_ref)
    torch.testing.assert_close(cols.cpu(), cols_ref, rtol=2e-4, atol=2e-4)
    # buffers are reused by the next ingest of the same shape
    p = obs.data_ptr()
    obs2, _ = ing.ingest(frags)
    assert obs2.data_ptr() == p


def _learner(cuda, **cfg):
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    torch.manual_seed(0)
    base = {"sgd_minibatch_size": 100, "num_sgd_iter": 2}
    base.update(cfg)
    return PPOLearner(VisionNetwork(4), base, device=cuda)


def _tables(cuda, N=400, A=4, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    obs = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    cols = torch.cat([torch.randn(N, A, generator=g), torch.randn(N, 1, generator=g) - 1.4,
                      torch.randn(N, 2, generator=g), torch.randint(0, A, (N, 1), generator=g).float()], 1).to(cuda)
    return obs, cols


@pytest.mark.parametrize("graphs", [False, True])
def test_manual_step_matches_autograd_step(cuda, graphs, monkeypatch):
    # the autograd path runs K12 unsplit: pin the manual step's K12 to the same row order
    monkeypatch.setenv("RMM_K12_SPLIT", "1")
    outs = []
    for manual in (True, False):
        L = _learner(cuda, manual_step=manual, use_graphs=graphs)
        assert (L._manual is not None) == manual
        obs, cols = _tables(cuda)
        torch.manual_seed(5)
        st = L._update_tables(obs, cols, 4)
        outs.append((L.master.clone(), st))
    (m1, s1), (m2, s2) = outs
    assert torch.equal(m1, m2)  # same kernels, same order: bit-identical weights
    # loss statistics are accumulated with device atomics (order-dependent in the last ulp)
    assert abs(s1["total_loss"] - s2["total_loss"]) < 1e-5 * max(1.0, abs(s1["total_loss"]))


@pytest.mark.parametrize("graphs", [False, True])
def test_tail_adam_matches_k6(cuda, graphs, monkeypatch):
    """Adam folded into the K10 trunk-reduce launch (tail Adam, the world-of-one default) vs the separate
    K6 launch: same weights, moments and step counters after two updates (4 minibatches x 2 epochs)."""
    monkeypatch.setenv("RMM_K12_SPLIT", "1")  # same K12 row order both sides
    outs = []
    for tail in (True, False):
        monkeypatch.setenv("RMM_TAIL_ADAM", "1" if tail else "0")
        L = _learner(cuda, use_graphs=graphs, lr=1e-3, weight_decay=0.01)
        assert L._tail_adam() == tail
        obs, cols = _tables(cuda)
        torch.manual_seed(5)
        st = L._update_tables(obs, cols, 4)
        torch.manual_seed(6)
        L._update_tables(obs, cols, 4)
        outs.append((L.master.clone(), L.m1.clone(), L.m2.clone(), L.w_bf16.clone(), L.ctr.clone(), st))
    a, b = outs
    assert torch.equal(a[4], b[4])                               # step counters advanced identically
    for x, y in zip(a[:4], b[:4]):  # bf16-rounded gradients, uncontracted Adam math: bit-identical
        assert torch.equal(x, y), float((x.float() - y.float()).abs().max())
    assert abs(a[5]["total_loss"] - b[5]["total_loss"]) < 1e-5 * max(1.0, abs(a[5]["total_loss"]))


@pytest.mark.parametrize("graphs", [False, True])
def test_x3_tail_adam_matches_k6(cuda, graphs, monkeypatch):
    """fp32 learner (x3 kernels): Adam folded into the x3 trunk-reduce launch vs the separate K6 launch —
    identical fp32 master, moments, split-pair planes and step counters after two updates."""
    outs = []
    for tail in (True, False):
        monkeypatch.setenv("RMM_TAIL_ADAM", "1" if tail else "0")
        L = _learner(cuda, use_graphs=graphs, lr=1e-3, weight_decay=0.01, compute_dtype="fp32")
        assert L.x3 and L._tail_adam() == tail
        obs, cols = _tables(cuda)
        torch.manual_seed(5)
        st = L._update_tables(obs, cols, 4)
        torch.manual_seed(6)
        L._update_tables(obs, cols, 4)
        outs.append((L.master.clone(), L.m1.clone(), L.m2.clone(), L.w_x3.hi.clone(), L.w_x3.lo.clone(),
                     L.ctr.clone(), st))
    a, b = outs
    assert torch.equal(a[5], b[5])
    for x, y in zip(a[:5], b[:5]):
        assert torch.equal(x, y), float((x.float() - y.float()).abs().max())
    # the split pair is the master's split
    assert torch.equal(a[3], a[0].to(torch.bfloat16))
    assert abs(a[6]["total_loss"] - b[6]["total_loss"]) < 1e-5 * max(1.0, abs(a[6]["total_loss"]))


def test_x3_dense_adam_fork_matches_folded(cuda, monkeypatch):
    """fp32 learner with graphs (parity counters): the dense + heads Adam forked onto a side stream beside
    the trunk backward (RMM_X3_DENSE_ADAM_FORK=1) gives bit-identical masters, moments, weight planes and
    counters to the Adam folded into the trunk-reduce launch."""
    outs = []
    monkeypatch.setenv("RMM_TAIL_ADAM", "1")
    for fork in ("0", "1"):
        monkeypatch.setenv("RMM_X3_DENSE_ADAM_FORK", fork)
        L = _learner(cuda, use_graphs=True, lr=1e-3, weight_decay=0.01, compute_dtype="fp32")
        assert L.x3 and L._tail_adam()
        obs, cols = _tables(cuda)
        torch.manual_seed(5)
        st = L._update_tables(obs, cols, 4)
        torch.manual_seed(6)
        L._update_tables(obs, cols, 4)
        if fork == "1":
            assert getattr(L, "_adam_stream", None) is not None  # the fork was taken
        outs.append((L.master.clone(), L.m1.clone(), L.m2.clone(), L.w_x3.hi.clone(), L.w_x3.lo.clone(),
                     L.ctr.clone(), st))
    a, b = outs
    assert torch.equal(a[5], b[5])
    for x, y in zip(a[:5], b[:5]):
        assert torch.equal(x, y), float((x.float() - y.float()).abs().max())


def test_grad_clip_coef_matches_torch(cuda):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    g = (torch.randn(1_000_003, device=cuda) * 3).to(torch.bfloat16)
    ws = torch.zeros(h.grad_clip_workspace_floats(), device=cuda)
    out = torch.zeros(2, device=cuda)
    for scale, max_norm in ((1.0, 10.0), (0.5, 1e9), (0.125, 1.0)):
        h.grad_clip_coef(g.data_ptr(), True, g.numel(), scale, max_norm, ws.data_ptr(), out.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
        norm = float((g.double() * scale).norm())
        assert abs(float(out[1]) - norm) / norm < 1e-4
        assert abs(float(out[0]) - min(1.0, max_norm / (norm + 1e-6))) < 1e-5


def test_fused_update_with_clip_matches_fp32_reference(cuda):
    """One fused bf16 SGD step (K10/K13/K15/K12 → flat bf16 gradient bucket, K6b clip coefficient)
    vs fp32 autograd on the same minibatch rows: gradients, clip coefficient and loss agree."""
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import ppo_categorical_loss_reference

    L = _learner(cuda, sgd_minibatch_size=200, num_sgd_iter=1, grad_clip=0.5, lr=1e-3, kl_coeff=0.2,
                 entropy_coeff=0.01)
    ref = VisionNetwork(4).to(cuda)
    ref.load_state_dict({k: torch.as_tensor(v).to(cuda) for k, v in L.get_weights().items()})
    obs, cols = _tables(cuda, N=200)
    torch.manual_seed(9)
    st = L._update_tables(obs, cols, 4)  # one minibatch holding all 200 rows (the mean is order-free)
    fused_by_name = {n: p._rmm_grad_out.float().reshape(-1) for n, p in L.model.named_parameters()}
    g_fused = torch.cat([fused_by_name[n] for n, _ in ref.named_parameters()])
    logits, v = ref(obs)
    coef = torch.tensor([0.1, 10.0, 1.0, 0.01, 0.2])
    total, _ = ppo_categorical_loss_reference(logits, v, cols[:, :4], cols[:, 7].long(), cols[:, 4], cols[:, 5],
                                              cols[:, 6], coef)
    total.backward()
    g_ref = torch.cat([p.grad.float().reshape(-1) for p in ref.parameters()])
    cos = float(torch.nn.functional.cosine_similarity(g_ref, g_fused, dim=0))
    assert cos > 0.99, cos
    assert abs(float(g_fused.norm() / g_ref.norm()) - 1) < 0.05
    ref_norm = float(g_ref.norm())
    assert abs(float(L.clip_out[1]) / ref_norm - 1) < 0.05
    assert abs(float(L.clip_out[0]) - min(1.0, 0.5 / ref_norm)) < 0.05 * min(1.0, 0.5 / ref_norm)
    assert abs(st["total_loss"] - float(total)) < 0.02 * max(1.0, abs(float(total)))


class _ActionZeroEnv:
    """Device env whose reward is 1 for action 0: a policy-gradient sign check."""

    def __init__(self, n, device):
        from ray_memory_management_amd.rllib.env import Discrete

        self.num_envs = n
        self.device = torch.device(device)
        self.frames = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=self.device)
        self.action_space = Discrete(4)

    def reset(self):
        return self.frames

    def step(self, actions):
        r = (actions == 0).float()
        return self.frames, r, torch.zeros(self.num_envs, device=self.device)


def test_fused_ppo_learns_action0_task(cuda):
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler

    L = _learner(cuda, sgd_minibatch_size=200, num_sgd_iter=4, lr=1e-3, entropy_coeff=0.0)
    env = _ActionZeroEnv(20, cuda)
    S = GPURolloutSampler(env, L.model, fragment=40)
    first = None
    for _ in range(25):
        b = S.sample()
        m = float(b["rewards"].float().mean())
        first = m if first is None else first
        L.update(b)
    assert first < 0.45 and m > 0.8, (first, m)


def test_ppo_gpu_learner_actor_cpu_rollouts(cuda):
    """The bench's runtime path at small scale: 1 GPU learner actor, 2 CPU rollout workers."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    ray.init(num_cpus=4, num_gpus=1, object_store_memory=1 << 30)
    try:
        cfg = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"episode_len": 50})
               .rollouts(num_rollout_workers=2, num_envs_per_worker=5, rollout_fragment_length=20,
                         postprocess_on_learner=True)
               .training(train_batch_size=200, sgd_minibatch_size=50, num_sgd_iter=2, grad_clip=40.0)
               .resources(num_learner_workers=1, num_gpus_per_learner_worker=1)
               .debugging(seed=0))
        algo = cfg.build()
        info = algo.learner_group.device_info()
        assert info[0]["device"] == "cuda:0"
        for _ in range(3):
            r = algo.train()
        st = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert np.isfinite(st["total_loss"]) and st["num_sgd_steps"] == 8 and st["grad_gnorm"] > 0
        assert st["ingest_bytes"] > 0
        algo.stop()
    finally:
        ray.shutdown()


def test_hybrid_worker_fragment_consistent(cuda):
    """CPU env + GPU policy worker: one graph replay per step; the fragment's logp must equal
    log_softmax(logits)[action] and rows must be time-major like a CPU worker's."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker
    from ray_memory_management_amd.rllib.execution.sample_ingest import fragment_dims

    w = HybridRolloutWorker(config={"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 30},
                                    "num_envs_per_worker": 4, "rollout_fragment_length": 16, "seed": 3})
    for _ in range(2):
        f = w.sample()
        T, n, A = fragment_dims(f)
        assert (T, n) == (16, 4) and tuple(f["obs"].shape) == (64, 4, 84, 84) and f["obs"].dtype == torch.uint8
        assert f["obs"].is_cuda and f["_raw"].is_cuda  # frames stay in HBM
        raw = f["_raw"].cpu().numpy()
        lsm = torch.log_softmax(torch.as_tensor(raw[:, :A]), -1).numpy()
        act = raw[:, A + 4].astype(np.int64)
        assert act.min() >= 0 and act.max() < A
        np.testing.assert_allclose(lsm[np.arange(len(act)), act], raw[:, A], atol=2e-3)
        boot = f["_boot"].cpu().numpy()
        assert np.isfinite(boot).all() and boot.shape == (4,)
        # row t*n+e of obs is the frame env e saw at step t: first rows match the reset frames
        assert int(f["obs"][:4].float().sum()) > 0
    # weights from a learner land in the graph-captured bf16 parameters in place
    wts = {k: np.zeros(v.shape, np.float32) for k, v in w.get_weights().items()}
    w.set_weights(wts)
    f = w.sample()
    np.testing.assert_allclose(f["_raw"][:, :A].cpu().numpy(), 0.0, atol=1e-6)  # zero weights -> zero logits
    assert len(w.get_metrics()) > 0  # episode_len 30 < 3 x 16 steps


def test_k19_frame_push_matches_torch(cuda):
    import torch

    from ray_memory_management_amd._native import require_hip

    B, T, hw = 5, 3, 84 * 84
    g = torch.Generator(device="cuda").manual_seed(0)
    stack = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
    new = torch.randint(0, 256, (B, 84, 84), dtype=torch.uint8, device="cuda", generator=g)
    buf = torch.zeros((T, B, 4, 84, 84), dtype=torch.uint8, device="cuda")
    t = torch.tensor([2], dtype=torch.int64, device="cuda")
    want = torch.cat([stack[:, 1:], new.unsqueeze(1)], dim=1)
    require_hip().frame_push(stack.data_ptr(), new.data_ptr(), buf.data_ptr(), t.data_ptr(), B, hw,
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(stack, want) and torch.equal(buf[2], want) and int(buf[:2].sum()) == 0


def test_hybrid_device_frame_stacks_match_host_stacks(cuda):
    """K19 path (newest frame uploaded, stacks kept in HBM) yields the same fragments, bit for bit,
    as uploading the CPU env's full frame stacks every step."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 20}, "num_envs_per_worker": 6,
           "rollout_fragment_length": 12, "seed": 5}
    a = HybridRolloutWorker(config=cfg)
    b = HybridRolloutWorker(config=cfg)
    assert all(g.device_stack for g in a.groups)
    assert all(g.h_new_dev and g.h_act_dev for g in a.groups)  # zero-copy frames in, actions out
    for g in b.groups:
        g.device_stack = False  # h_obs still holds the reset stacks: full-stack upload path
        g.h_act_dev = 0  # staged D2H action copies (env transitions depend on the actions)
    for _ in range(3):
        fa, fb = a.sample(), b.sample()
        assert torch.equal(fa["obs"], fb["obs"])
        assert torch.equal(fa["_raw"], fb["_raw"]) and torch.equal(fa["_boot"], fb["_boot"])


def test_ppo_hybrid_rollouts(cuda):
    """PPO with CPU-env / GPU-policy rollout workers co-located with the learner actor."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    ray.init(num_cpus=4, num_gpus=1, object_store_memory=1 << 30)
    try:
        cfg = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"episode_len": 50})
               .rollouts(num_rollout_workers=2, num_envs_per_worker=5, rollout_fragment_length=20,
                         postprocess_on_learner=True)
               .training(train_batch_size=200, sgd_minibatch_size=50, num_sgd_iter=2)
               .resources(num_learner_workers=1, num_gpus_per_learner_worker=0.5, num_gpus_per_worker=0.25)
               .debugging(seed=0))
        algo = cfg.build()
        names = ray.get([w.apply.remote(lambda x: type(x).__name__) for w in algo.workers.remote_workers()])
        assert names == ["HybridRolloutWorker"] * 2
        for _ in range(2):
            r = algo.train()
        st = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert np.isfinite(st["total_loss"]) and st["num_sgd_steps"] == 8
        # weights travel learner -> workers as ONE flat bf16 HBM object (hipIPC), not host numpy
        assert algo._device_weights_ok() and algo._dev_refs is not None
        w0 = algo.workers.remote_workers()[0]
        ray.get(w0.set_weights.remote(algo.learner_group.device_weights_refs()[0]))
        got = ray.get(w0.get_weights.remote())
        master = algo.learner_group.get_weights()
        for k, v in master.items():
            want = torch.from_numpy(np.ascontiguousarray(v)).to(torch.bfloat16).float().numpy()
            np.testing.assert_array_equal(got[k], want)
        algo.stop()
    finally:
        ray.shutdown()


@pytest.mark.parametrize("double_buffer", [False, True])
def test_hybrid_step_gate_matches_ungated(cuda, double_buffer, monkeypatch):
    """Step gate (opt-in; step t+1 enqueued before step t's env step, held on the device until the
    host releases it) yields the same fragments, bit for bit, as launching after the env step; the gate
    never times out, and the device / host sequence counters agree."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 20}, "num_envs_per_worker": 6,
           "rollout_fragment_length": 12, "seed": 7, "rollout_double_buffer": double_buffer}
    monkeypatch.setenv("RMM_ROLLOUT_GATE", "1")
    a = HybridRolloutWorker(config=cfg)
    fa = [a.sample() for _ in range(3)]
    assert all(g.gate for g in a.groups)
    monkeypatch.setenv("RMM_ROLLOUT_GATE", "0")
    b = HybridRolloutWorker(config=cfg)
    fb = [b.sample() for _ in range(3)]
    assert not any(g.gate for g in b.groups)
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k
    torch.cuda.synchronize()
    for g in a.groups:
        assert int(g.gate_err.item()) == 0
        assert int(g.dev_seq.item()) == int(g._rel[0]) == 2 + 3 * 12  # 2 warm-up steps + 3 fragments


@pytest.mark.parametrize("double_buffer", [False, True])
def test_native_rollout_loop_matches_python_loop(cuda, double_buffer, monkeypatch):
    """The native hybrid rollout loop (csrc/hip/rollout_loop.cc: event wait → native env step →
    graph launch per group step) yields the same fragments, bit for bit, and the same finished
    episodes as the Python loop over the same envs and graphs."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 9}, "num_envs_per_worker": 6,
           "rollout_fragment_length": 12, "seed": 3, "rollout_double_buffer": double_buffer}
    monkeypatch.delenv("RMM_NO_NATIVE_ROLLOUT", raising=False)
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "0")  # the graph-launch loop (direct launches: their own test)
    a = HybridRolloutWorker(config=cfg)
    fa = [a.sample() for _ in range(3)]
    assert a._native_desc is not None and len(a._native_desc) == (2 if double_buffer else 1)
    monkeypatch.setenv("RMM_NO_NATIVE_ROLLOUT", "1")
    b = HybridRolloutWorker(config=cfg)
    fb = [b.sample() for _ in range(3)]
    assert getattr(b, "_native_desc", None) is None
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k
    assert len(a._completed) > 0 and a._completed == b._completed


@pytest.mark.parametrize("n_envs,T", [(6, 12), (50, 20)])
def test_rollout_server_matches_graph_loop(cuda, monkeypatch, n_envs, T):
    """K21 persistent rollout server (one launch per fragment, host ↔ GPU through mapped words,
    grid barriers between the trunk / dense / heads phases) yields the same fragments, bit for bit,
    and the same finished episodes as the per-step graph loop; its workgroups drain cleanly."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 9}, "num_envs_per_worker": n_envs,
           "rollout_fragment_length": T, "seed": 3}
    monkeypatch.delenv("RMM_NO_NATIVE_ROLLOUT", raising=False)
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "0")  # reference side: the per-step graph-launch loop
    monkeypatch.setenv("RMM_ROLLOUT_SERVER", "1")
    a = HybridRolloutWorker(config=cfg)
    fa = [a.sample() for _ in range(3)]
    assert getattr(a, "_server_cache", None) is not None and not getattr(a, "_server_off", False)
    monkeypatch.setenv("RMM_ROLLOUT_SERVER", "0")
    b = HybridRolloutWorker(config=cfg)
    fb = [b.sample() for _ in range(3)]
    assert getattr(b, "_server_cache", None) is None and b._native_desc is not None
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k
    assert len(a._completed) > 0 and a._completed == b._completed


def test_k10_band_push_matches_stack_push(cuda, monkeypatch):
    """K10 rollout band mode (4 workgroups per frame, frame stack = rollout row t-1) yields the same
    fragments, bit for bit, as the one-workgroup-per-frame push over a separate device frame stack."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 7}, "num_envs_per_worker": 9,
           "rollout_fragment_length": 6, "seed": 5}
    monkeypatch.setenv("RMM_BAND_PUSH", "1")
    a = HybridRolloutWorker(config=cfg)
    fa = [a.sample() for _ in range(3)]
    assert all(g.band for g in a.groups)
    monkeypatch.setenv("RMM_BAND_PUSH", "0")
    b = HybridRolloutWorker(config=cfg)
    fb = [b.sample() for _ in range(3)]
    assert not any(g.band for g in b.groups)
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k


def test_hybrid_recapture_mid_life_keeps_fragments(cuda):
    """A hybrid worker that recaptures its policy-step graphs after a fragment (parameters rebound:
    zero-copy shared weights) must produce the same fragments as one that never recaptured. The
    recapture's warm-up steps used to run at rollout row T (the previous fragment's end) and store
    rows T, T+1 past the rollout buffers — a GPU memory fault (profiles/shared_weights_r4.txt)."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 20}, "num_envs_per_worker": 6,
           "rollout_fragment_length": 12, "seed": 5}
    a = HybridRolloutWorker(config=cfg)
    b = HybridRolloutWorker(config=cfg)
    for i in range(3):
        if i:
            a._on_params_rebound()  # recapture before this fragment
        fa, fb = a.sample(), b.sample()
        assert torch.equal(fa["obs"], fb["obs"])
        assert torch.equal(fa["_raw"], fb["_raw"]) and torch.equal(fa["_boot"], fb["_boot"])


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_ppo_hybrid_shared_weights(cuda, monkeypatch, dtype):
    """Zero-copy weights (RMM_SHARED_WEIGHTS=1): the learner's live weights move once into HBM objects
    that the co-located hybrid rollout workers alias over hipIPC; after the learner's next in-place
    Adam steps the workers' parameters ARE the new weights (no per-iteration publish). bf16: the bf16
    compute weights. fp32 (precision-matched): the fp32 master (the workers' parameters) and its split
    pair (what their x3 kernels read) — and the weights the workers sample with change every iteration
    (a one-time snapshot must never be mistaken for a live alias)."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    monkeypatch.setenv("RMM_SHARED_WEIGHTS", "1")
    ray.init(num_cpus=4, num_gpus=1, object_store_memory=1 << 30)
    try:
        cfg = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"episode_len": 50})
               .rollouts(num_rollout_workers=2, num_envs_per_worker=5, rollout_fragment_length=20,
                         postprocess_on_learner=True)
               .training(train_batch_size=200, sgd_minibatch_size=50, num_sgd_iter=2, compute_dtype=dtype, lr=1e-3)
               .resources(num_learner_workers=1, num_gpus_per_learner_worker=0.5, num_gpus_per_worker=0.25)
               .debugging(seed=0))
        algo = cfg.build()
        ws = algo.workers.remote_workers()
        seen = []
        for _ in range(3):
            r = algo.train()
            if dtype == "fp32":  # what the workers' kernels read: the pair they alias
                seen.append(ray.get(ws[0].apply.remote(
                    lambda x: {n: p.float().cpu().numpy() for n, p in x.model.x3_pairs().items()})))
        st = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert np.isfinite(st["total_loss"]) and st["num_sgd_steps"] == 8
        assert algo._shared_weights_ok() and algo._dev_refs is not None
        assert algo.learner_group.shared_kind() == ("x3" if dtype == "fp32" else "bf16")
        # the next iteration's samples were queued behind the last update (RMM_PREFETCH_SAMPLE default)
        assert algo._prefetched is not None and len(algo._prefetched) == 2
        assert all(ray.get([w.apply.remote(lambda x: getattr(x, "_shared_key", None) is not None) for w in ws]))
        master = algo.learner_group.get_weights()
        for w in ws:  # no set_weights here: the aliased parameters already hold the last update
            got = ray.get(w.get_weights.remote())
            for k, v in master.items():
                want = np.ascontiguousarray(v)
                if dtype == "bf16":
                    want = torch.from_numpy(want).to(torch.bfloat16).float().numpy()
                np.testing.assert_array_equal(got[k], want)
        if dtype == "fp32":
            pair = ray.get(ws[1].apply.remote(lambda x: {n: p.float().cpu().numpy() for n, p in x.model.x3_pairs().items()}))
            for k, v in master.items():  # hi + lo == the fp32 master to the split's 2^-17
                np.testing.assert_allclose(pair[k], v, rtol=2.0 ** -16, atol=1e-12)
            for a, b in zip(seen, seen[1:]):  # weights move every iteration (not a stale snapshot)
                assert any(not np.array_equal(a[k], b[k]) for k in a)
        algo.stop()
    finally:
        ray.shutdown()


@pytest.mark.parametrize("seq", ["0", "1"])
@pytest.mark.parametrize("n_envs,T,dtype", [(6, 12, "bf16"), (50, 20, "bf16"), (6, 12, "fp32"), (50, 20, "fp32")])
def test_rollout_direct_launch_matches_graph_loop(cuda, monkeypatch, n_envs, T, seq, dtype):
    """The native loop with direct kernel launches per policy step (RMM_ROLLOUT_DIRECT=1: K10 push →
    K13s → K16 launched from the loop's thread, no graph; fp32 policy: K10x push → K13x → K16x) yields
    the same fragments, bit for bit, and the same finished episodes as the per-step graph launches."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 9}, "num_envs_per_worker": n_envs,
           "rollout_fragment_length": T, "seed": 3, "compute_dtype": dtype}
    monkeypatch.delenv("RMM_NO_NATIVE_ROLLOUT", raising=False)
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "1")
    monkeypatch.setenv("RMM_ROLLOUT_SEQ", seq)  # "1": completion through K16's host word, no events
    a = HybridRolloutWorker(config=cfg)
    fa = [a.sample() for _ in range(3)]
    assert getattr(a, "_server_cache", None) is not None  # the direct path's argument cache
    assert bool(a._server_cache.get("x3")) == (dtype == "fp32")  # fp32: the split-bf16 kernels
    if seq == "1":
        assert int(a._h_seq[0]) == T  # the last step (row T-1) stored T
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "0")
    b = HybridRolloutWorker(config=cfg)
    fb = [b.sample() for _ in range(3)]
    assert getattr(b, "_server_cache", None) is None and b._native_desc is not None
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k
    assert len(a._completed) > 0 and a._completed == b._completed


@pytest.mark.parametrize("n_envs", [6, 50])
def test_rollout_fused_heads_matches_two_launches(cuda, monkeypatch, n_envs):
    """fp32 direct rollout launches with K13x + K16x fused into one launch (RMM_ROLLOUT_FUSED_HEADS=1):
    fragments and finished episodes bit-identical to the two-launch step."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 9}, "num_envs_per_worker": n_envs,
           "rollout_fragment_length": 20, "seed": 3, "compute_dtype": "fp32"}
    monkeypatch.delenv("RMM_NO_NATIVE_ROLLOUT", raising=False)
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "1")
    frags = []
    for fused in ("0", "1"):
        monkeypatch.setenv("RMM_ROLLOUT_FUSED_HEADS", fused)
        w = HybridRolloutWorker(config=cfg)
        frags.append(([w.sample() for _ in range(3)], list(w._completed)))
        assert bool(w._direct_args(w.groups, w.group_streams).get("fused_heads")) == (fused == "1")
    (fa, ca), (fb, cb) = frags
    for x, y in zip(fa, fb):
        for k in ("obs", "_raw", "_boot"):
            assert torch.equal(x[k], y[k]), k
    assert len(ca) > 0 and ca == cb


def test_gate_timeout_resamples_the_fragment_ungated(cuda, monkeypatch):
    """A host that stalls longer than the step gate's bound between a launch and its release
    (RMM_TEST_GATE_DELAY_US in the native loop, gate bound 1 ms) makes the gated policy steps give up
    and read stale frames: sample() discards that fragment and re-samples it on the ungated path instead
    of failing the iteration; once the host keeps up again the gated path is used with no timeout."""
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    cfg = {"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 9}, "num_envs_per_worker": 6,
           "rollout_fragment_length": 8, "seed": 3, "compute_dtype": "fp32", "rollout_gate_timeout_ms": 1}
    monkeypatch.delenv("RMM_NO_NATIVE_ROLLOUT", raising=False)
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT", "1")
    monkeypatch.setenv("RMM_ROLLOUT_DIRECT_GATE", "1")
    monkeypatch.setenv("RMM_TEST_GATE_DELAY_US", "20000")
    a = HybridRolloutWorker(config=cfg)
    fa = a.sample()
    assert getattr(a, "gate_timeouts", 0) == 1
    monkeypatch.delenv("RMM_TEST_GATE_DELAY_US")
    a.config["rollout_gate_timeout_ms"] = 2000
    fb = a.sample()
    assert getattr(a, "gate_timeouts", 0) == 1
    for f in (fa, fb):
        assert f["obs"].shape[0] == 8 * 6 and torch.isfinite(f["_raw"].float()).all()
