"""Precision: the fp32 (precision-matched) learner on the hand-written split-bf16 kernels vs plain
torch fp32, and bf16-vs-fp32 learning parity.

The reference trains PPO in fp32 torch (rllib/algorithms/ppo/ppo_torch_policy.py:70). Here
``compute_dtype="fp32"`` runs the SGD step on the x3 kernels (csrc/hip/x3_kernels.hip: K10x / K13x /
K15x / K12x, fp32 operands as hi + lo bf16 pairs, fp32 accumulation, fp32 gradients, K6 Adam on the fp32
master) and the bf16 learner on K10 / K13s / K15 / K12. Checked on an MI355X:

* one fp32 update equals the plain-torch fp32 update (same minibatch, same Adam step), on the
  hand-written kernel step (``_manual is not None``);
* a multi-step task with GAE (gamma 0.99, lambda 0.95), rewards of scale 3 and value targets up to
  ~40: 60 iterations in LOCKSTEP (every learner trains on the same batches, collected by the torch
  learner's policy, one full-batch SGD step per iteration) — the fp32 kernel learner's weights must
  track the torch fp32 learner's far closer than the bf16 learner's do (measured drift after 60
  iterations: 3.4 % vs 10.8 % of the weights' total movement);
* on the same task each learner collecting its own data learns, and the fp32 kernel learner ends
  within a stated return tolerance of the torch fp32 learner.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# ---------------------------------------------------------------- one-step bandit (single update check)
def _frames(B, g, dev):
    """uint8 [B, 4, 84, 84] noise frames with one bright 42x42 quadrant: the class (0..3)."""
    c = torch.randint(0, 4, (B,), generator=g, device=dev)
    return _render(c, None, 1, g, dev), c


def _render(c, t_left, T_ep, g, dev):
    """Noise frames, the bright quadrant c, and (multi-step task) a bar on rows 0-3 whose length is the
    fraction of the episode left."""
    B = c.shape[0]
    x = torch.randint(0, 90, (B, 4, 84, 84), generator=g, device=dev, dtype=torch.uint8)
    r0, c0 = (c // 2) * 42, (c % 2) * 42
    rows = torch.arange(84, device=dev)
    m = ((rows[None, :, None] >= r0[:, None, None]) & (rows[None, :, None] < r0[:, None, None] + 42) &
         (rows[None, None, :] >= c0[:, None, None]) & (rows[None, None, :] < c0[:, None, None] + 42))
    x = torch.where(m[:, None], x + 150, x)
    if t_left is not None:
        bar = (rows[None, None, :] < (84 * t_left // T_ep)[:, None, None]) & (rows[None, :, None] < 4)
        x = torch.where(bar[:, None], torch.full_like(x, 255), x)
    return x.contiguous()


def _policy_sample(learner, obs, g):
    with torch.no_grad():
        logits, v = learner.model(obs)
        logits, v = logits.float(), v.float()
        u = torch.rand(logits.shape, generator=g, device=obs.device).clamp_(1e-10, 1.0)
        a = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1)
        logp = torch.log_softmax(logits, -1).gather(1, a[:, None]).squeeze(1)
    return a, logp, logits, v


def _batch(learner, B, g, dev):
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    obs, c = _frames(B, g, dev)
    a, logp, logits, v = _policy_sample(learner, obs, g)
    r = (a == c).float()  # one-step episodes: value target = reward, advantage = r - V
    return SampleBatch({SampleBatch.OBS: obs, SampleBatch.ACTIONS: a, SampleBatch.ACTION_LOGP: logp,
                        SampleBatch.ACTION_DIST_INPUTS: logits, SampleBatch.ADVANTAGES: r - v,
                        SampleBatch.VALUE_TARGETS: r}), float(r.mean())


def _learner(cuda, cfg, dtype):
    from ray_memory_management_amd.rllib.env import Discrete
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    if dtype == "torch":
        return PPOLearner(VisionNetwork(4), {**cfg, "fused": False}, device=cuda, action_space=Discrete(4))
    return PPOLearner(VisionNetwork(4), {**cfg, "compute_dtype": dtype}, device=cuda, action_space=Discrete(4))


def test_fp32_fast_learner_matches_torch_fp32_update(cuda):
    """One Adam step on one minibatch: the fp32 kernel learner's update vs the torch fp32 learner's,
    relative to the update's size. Dense / heads agree to ~1e-5 (the split-pair precision); the convs
    to <= 1 %: at ~1e-5 relative activation precision a few of the ~1.8M conv pre-activations lie close
    enough to zero for their ReLU masks to differ (measured 0.5 % on conv1, 0.1 % on conv2). The bf16
    learner deviates by 1-30 % on the same update (reported, and required to be >= 10x worse on average)."""
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(0)
    base = VisionNetwork(4)
    # adam_eps 1e-3: Adam's first step is lr * g / (|g| + eps); with the default 1e-8 an element whose
    # gradient is ~0 moves by +-lr on its rounding noise's sign, which no two fp32 implementations share
    cfg = {"sgd_minibatch_size": 256, "num_sgd_iter": 1, "lr": 1e-3, "standardize_advantages": False,
           "kl_coeff": 0.0, "entropy_coeff": 0.01, "adam_eps": 1e-3}
    lns = {dt: _learner(cuda, cfg, dt) for dt in ("torch", "fp32", "bf16")}
    for ln in lns.values():
        ln.set_weights({k: v.clone() for k, v in base.state_dict().items()})
    fast, ref = lns["fp32"], lns["torch"]
    assert fast.fast and fast.fp32 and fast.w_bf16 is None and not ref.fast
    assert fast.x3 and fast._manual is not None  # the hand-written split-bf16 SGD step, not autograd
    # world of one, no clip: the tail Adam adds K12x's two row parts (256 rows = 4 chunks)
    assert fast._x3_rows(256) == (2 if fast._tail_adam() else 1)
    g = torch.Generator(device=cuda).manual_seed(1)
    batch, _ = _batch(ref, 256, g, cuda)
    w0 = {k: v.float().cpu() for k, v in ref.get_weights().items()}
    for ln in lns.values():
        ln.update(batch.copy())
    W = {dt: ln.get_weights() for dt, ln in lns.items()}
    err = {dt: {k: float((W[dt][k] - W["torch"][k]).abs().max() / (W["torch"][k] - w0[k]).abs().max().clamp_min(1e-12))
                for k in w0} for dt in ("fp32", "bf16")}
    print("update error relative to the update", err)
    for k, e in err["fp32"].items():
        assert e < (1e-2 if k.startswith("convs") else 1e-4), (k, e)
    assert np.mean(list(err["fp32"].values())) * 10 < np.mean(list(err["bf16"].values())), err


# ---------------------------------------------------------------- multi-step task with GAE
class _ChaseEnv:
    """B parallel episodes of T_ep steps (staggered starts). Each step shows a bright quadrant c (fresh
    every step) and a bar with the steps left; reward +3 for the action naming c, -1 otherwise; the
    value of a state is the discounted reward still to come, so the critic must read the bar (multi-step
    returns through GAE, targets up to ~40 for a good policy)."""

    def __init__(self, B, T_ep, g, dev):
        self.B, self.T_ep, self.g, self.dev = B, T_ep, g, dev
        self.t = torch.randint(0, T_ep, (B,), generator=g, device=dev)
        self.c = torch.randint(0, 4, (B,), generator=g, device=dev)

    def obs(self):
        return _render(self.c, self.T_ep - self.t, self.T_ep, self.g, self.dev)

    def step(self, a):
        r = torch.where(a == self.c, 3.0, -1.0)
        self.t = self.t + 1
        done = self.t >= self.T_ep
        self.t = torch.where(done, torch.zeros_like(self.t), self.t)
        self.c = torch.randint(0, 4, (self.B,), generator=self.g, device=self.dev)
        return r, done.float()


def _rollout(learner, env, T, g, gamma=0.99, lam=0.95):
    """T steps of the env under learner's policy -> (SampleBatch with GAE advantages / targets, mean reward)."""
    from ray_memory_management_amd import ops
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    obs_l, a_l, lp_l, lg_l, v_l, r_l, d_l = [], [], [], [], [], [], []
    for _ in range(T):
        o = env.obs()
        a, logp, logits, v = _policy_sample(learner, o, g)
        r, d = env.step(a)
        for lst, x in zip((obs_l, a_l, lp_l, lg_l, v_l, r_l, d_l), (o, a, logp, logits, v, r, d)):
            lst.append(x)
    with torch.no_grad():
        _, last_v = learner.model(env.obs())
    rew, val, done = torch.stack(r_l), torch.stack(v_l), torch.stack(d_l)
    adv, ret = ops.gae(rew, val, done, last_v.float(), gamma, lam)
    n = T * env.B
    b = SampleBatch({SampleBatch.OBS: torch.stack(obs_l).view(n, 4, 84, 84), SampleBatch.ACTIONS: torch.stack(a_l).view(n),
                     SampleBatch.ACTION_LOGP: torch.stack(lp_l).view(n),
                     SampleBatch.ACTION_DIST_INPUTS: torch.stack(lg_l).view(n, -1),
                     SampleBatch.ADVANTAGES: adv.reshape(n), SampleBatch.VALUE_TARGETS: ret.reshape(n)})
    return b, float(rew.mean())


_MS_CFG = {"num_sgd_iter": 1, "lr": 3e-4, "kl_coeff": 0.2, "entropy_coeff": 0.01, "clip_param": 0.2,
           "vf_loss_coeff": 0.5, "vf_clip_param": 1e4, "gamma": 0.99, "lambda_": 0.95, "adam_eps": 1e-5}


def _flat(ln):
    return torch.cat([v.float().reshape(-1) for _, v in sorted(ln.get_weights().items())])


def test_fp32_kernel_learner_tracks_torch_fp32_over_60_iterations(cuda):
    """LOCKSTEP: the torch fp32 learner collects every batch (multi-step task, GAE); the torch, fp32-kernel
    and bf16 learners all train on it (one full-batch SGD step per iteration, so all three follow the
    same gradient path). Drift = |w_learner - w_torch| / |w_torch - w_0|. Measured on MI355X (adam_eps
    1e-3, lr 1e-3): fp32 kernels 0.05 % after 1 iteration, 3.4 % after 60; bf16 2.8 % and 10.8 %."""
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(0)
    base = VisionNetwork(4)
    B, T = 32, 16
    cfg = {**_MS_CFG, "sgd_minibatch_size": B * T, "adam_eps": 1e-3, "lr": 1e-3}
    lns = {dt: _learner(cuda, cfg, dt) for dt in ("torch", "fp32", "bf16")}
    for ln in lns.values():
        ln.set_weights({k: v.clone() for k, v in base.state_dict().items()})
    assert lns["fp32"]._manual is not None and lns["bf16"]._manual is not None
    w0 = _flat(lns["torch"])
    g = torch.Generator(device=cuda).manual_seed(3)
    env = _ChaseEnv(B, 16, g, cuda)
    drift = {}
    for it in range(60):
        batch, _ = _rollout(lns["torch"], env, T, g)
        for ln in lns.values():
            ln.update(batch.copy())
        if it in (0, 9, 59):
            wt = _flat(lns["torch"])
            moved = float((wt - w0).norm())
            drift[it + 1] = {dt: float((_flat(lns[dt]) - wt).norm()) / moved for dt in ("fp32", "bf16")}
    print("drift from the torch fp32 learner", drift)
    assert drift[1]["fp32"] < 5e-3 and drift[1]["bf16"] > 10 * drift[1]["fp32"], drift
    assert drift[10]["fp32"] < 0.06 and drift[10]["bf16"] > 2 * drift[10]["fp32"], drift
    assert drift[60]["fp32"] < 0.08 and drift[60]["bf16"] > 2 * drift[60]["fp32"], drift
    obs = _ChaseEnv(256, 16, g, cuda).obs()
    with torch.no_grad():
        lt, vt = (x.float() for x in lns["torch"].model(obs))
        lf, vf = (x.float() for x in lns["fp32"].model(obs))
    print("max |value diff|", float((vf - vt).abs().max()), "of", float(vt.abs().max()),
          "max |logit diff|", float((lf - lt).abs().max()), "of", float(lt.abs().max()))
    assert float((vf - vt).abs().max()) < 0.1 * float(vt.abs().max()) + 1e-3
    assert float((lf - lt).abs().max()) < 0.1 * float(lt.abs().max()) + 1e-3


def test_fp32_kernel_learner_learns_like_torch_fp32_and_bf16(cuda):
    """Each learner collects its own data on the multi-step task for 50 iterations (4 minibatch SGD
    steps each): all three learn, and the fp32-kernel and bf16 learners end within 0.6 reward per step
    (scale: -1 .. +3) of the torch fp32 learner."""
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(0)
    base = VisionNetwork(4)
    B, T = 32, 16
    cfg = {**_MS_CFG, "sgd_minibatch_size": 128, "num_sgd_iter": 2, "lr": 5e-4}
    curves = {}
    for dt in ("torch", "fp32", "bf16"):
        ln = _learner(cuda, cfg, dt)
        ln.set_weights({k: v.clone() for k, v in base.state_dict().items()})
        g = torch.Generator(device=cuda).manual_seed(11)
        env = _ChaseEnv(B, 16, g, cuda)
        rets = []
        for _ in range(50):
            b, r = _rollout(ln, env, T, g)
            rets.append(r)
            ln.update(b)
        curves[dt] = rets
    last = {dt: float(np.mean(c[-5:])) for dt, c in curves.items()}
    for dt, c in curves.items():
        print(dt, np.round(c[::5], 3).tolist())
    for dt in curves:
        assert curves[dt][0] < 0.6 and last[dt] > 1.8, (dt, curves[dt][0], last[dt])  # chance: 0.0 per step
    assert abs(last["fp32"] - last["torch"]) < 0.6 and abs(last["bf16"] - last["torch"]) < 0.6, last
