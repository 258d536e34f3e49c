"""MARWIL (monotonic advantage re-weighted imitation learning) from offline data; BC is MARWIL
with beta = 0.

Parity: reference rllib/algorithms/marwil/marwil.py (MARWILConfig: beta 1.0, vf_coeff 1.0,
moving_average_sqd_adv_norm_start 100, moving_average_sqd_adv_norm_update_rate 1e-8, lr 1e-4,
train_batch_size 2000; training_step = sample (from the offline input reader) → train_one_step →
sync weights) and marwil_torch_policy.py (advantages = discounted episode returns − V(s);
policy loss −mean(exp(beta·adv/√ma_adv²)·logπ(a|s)), value loss 0.5·mean(adv²)).
"""
from __future__ import annotations

import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch, concat_samples


class MARWILConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or MARWIL)
        self.beta = 1.0
        self.vf_coeff = 1.0
        self.moving_average_sqd_adv_norm_start = 100.0
        self.moving_average_sqd_adv_norm_update_rate = 1e-8
        self.lr = 1e-4
        self.grad_clip = None
        self.train_batch_size = 2000
        self.num_workers = 0
        self.postprocess_inputs = False
        self.input_ = "sampler"


def discounted_returns(rew: np.ndarray, dones: np.ndarray, eps: np.ndarray, gamma: float) -> np.ndarray:
    """Discounted reward-to-go within each episode segment (a segment ends at a done, at an
    episode-id change or at the end of the batch)."""
    out = np.zeros(len(rew), dtype=np.float32)
    acc = 0.0
    for i in range(len(rew) - 1, -1, -1):
        last = i == len(rew) - 1 or bool(dones[i]) or (eps is not None and eps[i + 1] != eps[i])
        acc = float(rew[i]) + (0.0 if last else gamma * acc)
        out[i] = acc
    return out


class MARWILLearner:
    def __init__(self, model: nn.Module, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.cfg = cfg
        self.opt = torch.optim.Adam(self.model.parameters(), lr=cfg["lr"])
        self.ma_adv_norm = float(cfg["moving_average_sqd_adv_norm_start"])

    def update(self, b: SampleBatch) -> Dict:
        c = self.cfg
        dev = self.device
        obs = torch.as_tensor(np.asarray(b[SampleBatch.OBS]), device=dev)
        act = torch.as_tensor(np.asarray(b[SampleBatch.ACTIONS]), device=dev).long()
        ret = torch.as_tensor(np.asarray(b["returns"]), device=dev).float()
        logits, v = self.model(obs)
        logp = torch.log_softmax(logits.float(), -1).gather(1, act.view(-1, 1)).squeeze(1)
        beta = float(c["beta"])
        if beta != 0.0:
            adv = ret - v.float()
            with torch.no_grad():
                self.ma_adv_norm += c["moving_average_sqd_adv_norm_update_rate"] * (
                    float((adv.detach() ** 2).mean()) - self.ma_adv_norm)
                w = torch.exp(beta * adv.detach() / (1e-8 + self.ma_adv_norm ** 0.5))
            vf_loss = 0.5 * (adv ** 2).mean()
        else:  # behaviour cloning
            w = torch.ones_like(logp)
            vf_loss = torch.zeros((), device=dev)
        p_loss = -(w * logp).mean()
        total = p_loss + c["vf_coeff"] * vf_loss
        self.opt.zero_grad(set_to_none=True)
        total.backward()
        if c.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.model.parameters(), c["grad_clip"])
        self.opt.step()
        return {"policy_loss": float(p_loss.detach()), "vf_loss": float(vf_loss.detach()),
                "total_loss": float(total.detach()), "moving_average_sqd_adv_norm": self.ma_adv_norm}

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        self.model.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})


class MARWIL(Algorithm):
    _config_class = MARWILConfig

    def validate_config(self, c):
        super().validate_config(c)
        if c.beta < 0:
            raise ValueError("beta must be >= 0")

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        cfg = {k: getattr(c, k) for k in ("lr", "beta", "vf_coeff", "grad_clip", "moving_average_sqd_adv_norm_start",
                                           "moving_average_sqd_adv_norm_update_rate")}
        self.learner = MARWILLearner(copy.deepcopy(self.workers.local_worker().policy.model), cfg, device=dev)
        self._sync()

    def _sync(self):
        w = self.learner.get_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def training_step(self) -> Dict:
        c = self.algo_config
        parts, n = [], 0
        while n < c.train_batch_size:
            b = self.workers.local_worker().sample() if not self.workers.remote_workers() else \
                concat_samples(self.workers.synchronous_parallel_sample(1, concat=False))
            parts.append(b)
            n += b.count
        for b in parts:  # returns per episode segment, inside each stored batch
            eps = b[SampleBatch.EPS_ID] if SampleBatch.EPS_ID in b else None
            dict.__setitem__(b, "returns", discounted_returns(np.asarray(b[SampleBatch.REWARDS]),
                                                             np.asarray(b[SampleBatch.DONES]),
                                                             None if eps is None else np.asarray(eps), c.gamma))
        keep = [SampleBatch.OBS, SampleBatch.ACTIONS, "returns"]
        batch = concat_samples([SampleBatch({k: p[k] for k in keep}) for p in parts])
        self._counters["num_env_steps_sampled"] += batch.count
        self._counters["num_agent_steps_trained"] += batch.count
        self._counters["num_env_steps_trained"] += batch.count
        self._timesteps_total += batch.count
        stats = self.learner.update(batch)
        self._sync()
        return stats

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, weights):
        self.learner.set_weights(weights)
        self._sync()


DEFAULT_CONFIG = MARWILConfig().to_dict()
