"""Trajectory postprocessing. Parity: reference rllib/evaluation/postprocessing.py
(Postprocessing, discount_cumsum, compute_advantages, compute_gae_for_sample_batch).
Batched fragments of the built-in algorithms go through the GAE HIP kernel (policy.
compute_gae_for_trajectories); these helpers handle one trajectory at a time, as in the reference."""
from __future__ import annotations

import numpy as np

from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class Postprocessing:
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"


def discount_cumsum(x: np.ndarray, gamma: float) -> np.ndarray:
    """y[t] = Σ_k γ^k x[t+k]."""
    x = np.asarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    acc = 0.0
    for t in range(len(x) - 1, -1, -1):
        acc = x[t] + gamma * acc
        out[t] = acc
    return out


def compute_advantages(rollout: SampleBatch, last_r: float, gamma: float = 0.9, lambda_: float = 1.0,
                       use_gae: bool = True, use_critic: bool = True) -> SampleBatch:
    """GAE (use_gae) or discounted returns (minus the value baseline when use_critic)."""
    rew = np.asarray(rollout[SampleBatch.REWARDS], dtype=np.float64)
    if use_gae:
        if SampleBatch.VF_PREDS not in rollout:
            raise ValueError("use_gae=True needs vf_preds in the rollout")
        vpred = np.concatenate([np.asarray(rollout[SampleBatch.VF_PREDS], dtype=np.float64), [float(last_r)]])
        delta = rew + gamma * vpred[1:] - vpred[:-1]
        adv = discount_cumsum(delta, gamma * lambda_)
        rollout[Postprocessing.ADVANTAGES] = adv.astype(np.float32)
        rollout[Postprocessing.VALUE_TARGETS] = (adv + vpred[:-1]).astype(np.float32)
    else:
        ret = discount_cumsum(np.concatenate([rew, [float(last_r)]]), gamma)[:-1]
        if use_critic:
            rollout[Postprocessing.ADVANTAGES] = (ret - np.asarray(rollout[SampleBatch.VF_PREDS])).astype(np.float32)
            rollout[Postprocessing.VALUE_TARGETS] = ret.astype(np.float32)
        else:
            rollout[Postprocessing.ADVANTAGES] = ret.astype(np.float32)
            rollout[Postprocessing.VALUE_TARGETS] = np.zeros_like(ret, dtype=np.float32)
    return rollout


def compute_gae_for_sample_batch(policy, sample_batch: SampleBatch, other_agent_batches=None, episode=None):
    """Bootstrap with the value of the last next-observation unless the trajectory ended."""
    dones = np.asarray(sample_batch[SampleBatch.DONES])
    if len(dones) and dones[-1]:
        last_r = 0.0
    else:
        last_obs = np.asarray(sample_batch[SampleBatch.NEXT_OBS])[-1:]
        last_r = float(np.asarray(policy.value(last_obs))[0]) if hasattr(policy, "value") else 0.0
    cfg = getattr(policy, "config", {}) or {}
    return compute_advantages(sample_batch, last_r, cfg.get("gamma", 0.99), cfg.get("lambda", cfg.get("lambda_", 1.0)),
                              cfg.get("use_gae", True), cfg.get("use_critic", True))
