"""Precision: the fp32 (precision-matched) fused learner, and bf16-vs-fp32 learning parity.

The reference trains PPO in fp32 torch. Here the headline learner computes in bf16 on MFMA with
fp32 master weights / Adam moments (K10 / K12 / K13 / K15 / K6), and ``compute_dtype="fp32"``
runs the same fast path (device index tables, chained HIP-graph SGD steps, K5b loss, K6 Adam)
with fp32 weights, gradients and convolutions. Checked on an MI355X:

* one fp32 fast-path update equals the plain-torch fp32 update (same minibatch, same Adam step);
* on a learnable frame task (a bright quadrant names the rewarded action) the bf16 fused learner
  and the fp32 learner, from identical initial weights, both learn it and end within a stated
  return tolerance of each other — the evidence that bf16 training does not change learning.
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


def _frames(B, g, dev):
    """uint8 [B, 4, 84, 84] noise frames with one bright 42x42 quadrant: the class (0..3)."""
    c = torch.randint(0, 4, (B,), generator=g, device=dev)
    x = torch.randint(0, 90, (B, 4, 84, 84), generator=g, device=dev, dtype=torch.uint8)
    r0 = (c // 2) * 42
    c0 = (c % 2) * 42
    rows = torch.arange(84, device=dev)
    m = ((rows[None, :, None] >= r0[:, None, None]) & (rows[None, :, None] < r0[:, None, None] + 42) &
         (rows[None, None, :] >= c0[:, None, None]) & (rows[None, None, :] < c0[:, None, None] + 42))
    x = torch.where(m[:, None], x + 150, x)
    return x.contiguous(), c


def _batch(learner, B, g, dev):
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    obs, c = _frames(B, g, dev)
    with torch.no_grad():
        logits, v = learner.model(obs)
        logits, v = logits.float(), v.float()
        u = torch.rand(logits.shape, generator=g, device=dev).clamp_(1e-10, 1.0)
        a = torch.argmax(logits - torch.log(-torch.log(u)), dim=-1)
        logp = torch.log_softmax(logits, -1).gather(1, a[:, None]).squeeze(1)
    r = (a == c).float()  # one-step episodes: value target = reward, advantage = r - V
    return SampleBatch({SampleBatch.OBS: obs, SampleBatch.ACTIONS: a, SampleBatch.ACTION_LOGP: logp,
                        SampleBatch.ACTION_DIST_INPUTS: logits, SampleBatch.ADVANTAGES: r - v,
                        SampleBatch.VALUE_TARGETS: r}), float(r.mean())


def test_fp32_fast_learner_matches_torch_fp32_update(cuda):
    from ray_memory_management_amd.rllib.env import Discrete
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    torch.manual_seed(0)
    base = VisionNetwork(4)
    # adam_eps 1e-3: Adam's first step is lr * g / (|g| + eps); with the default 1e-8 an element whose
    # gradient is ~0 moves by +-lr on its rounding noise's sign, which no two fp32 implementations share
    cfg = {"sgd_minibatch_size": 256, "num_sgd_iter": 1, "lr": 1e-3, "standardize_advantages": False,
           "kl_coeff": 0.0, "entropy_coeff": 0.01, "adam_eps": 1e-3}
    fast = PPOLearner(VisionNetwork(4), {**cfg, "compute_dtype": "fp32"}, device=cuda, action_space=Discrete(4))
    ref = PPOLearner(VisionNetwork(4), {**cfg, "fused": False}, device=cuda, action_space=Discrete(4))
    for ln in (fast, ref):
        ln.set_weights({k: v.clone() for k, v in base.state_dict().items()})
    assert fast.fast and fast.fp32 and fast.w_bf16 is None and not ref.fast
    g = torch.Generator(device=cuda).manual_seed(1)
    batch, _ = _batch(ref, 256, g, cuda)
    w0 = {k: v.float().cpu() for k, v in fast.get_weights().items()}
    fast.update(batch.copy())
    ref.update(batch.copy())
    wf, wr = fast.get_weights(), ref.get_weights()
    for k in wr:
        d_ref = (wr[k] - w0[k]).abs().max()
        err = (wf[k] - wr[k]).abs().max()
        assert err <= 2e-3 * max(float(d_ref), 1e-6) + 1e-6, (k, float(err), float(d_ref))


@pytest.mark.parametrize("iters", [30])
def test_bf16_learner_learns_like_fp32_learner(cuda, iters):
    from ray_memory_management_amd.rllib.env import Discrete
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    torch.manual_seed(0)
    base = VisionNetwork(4)
    cfg = {"sgd_minibatch_size": 250, "num_sgd_iter": 4, "lr": 3e-4, "kl_coeff": 0.0, "entropy_coeff": 0.0,
           "clip_param": 0.2, "vf_loss_coeff": 0.5}
    curves = {}
    for dt in ("bf16", "fp32"):
        ln = PPOLearner(VisionNetwork(4), {**cfg, "compute_dtype": dt}, device=cuda, action_space=Discrete(4))
        ln.set_weights({k: v.clone() for k, v in base.state_dict().items()})
        assert ln.fast and (ln._manual is not None) == (dt == "bf16")  # bf16: the hand-written K10..K15 step
        g = torch.Generator(device=cuda).manual_seed(7)
        rets = []
        for _ in range(iters):
            b, r = _batch(ln, 1000, g, cuda)
            rets.append(r)
            ln.update(b)
        curves[dt] = rets
    last_bf, last_fp = np.mean(curves["bf16"][-5:]), np.mean(curves["fp32"][-5:])
    print("bf16", np.round(curves["bf16"], 3).tolist())
    print("fp32", np.round(curves["fp32"], 3).tolist())
    assert curves["bf16"][0] < 0.45 and curves["fp32"][0] < 0.45  # starts near chance (0.25)
    assert last_bf > 0.85 and last_fp > 0.85, (last_bf, last_fp)
    assert abs(last_bf - last_fp) < 0.1, (last_bf, last_fp)
