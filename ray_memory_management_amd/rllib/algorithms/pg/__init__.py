"""Vanilla policy gradient (REINFORCE with discounted returns).

Parity: reference rllib/algorithms/pg/pg.py (PGConfig: lr 0.0004, train_batch_size 200,
rollout_fragment_length 200, num_workers 0; training_step = synchronous_parallel_sample →
train_one_step → sync weights) and pg_torch_policy.py (loss = -mean(logp(a) * discounted
return), advantages from postprocessing.compute_advantages(use_gae=False, use_critic=False)).

The on-policy torch learner here (``OnPolicyLearner``) is shared with A2C: one optimizer step per
train batch (or per microbatch with gradient accumulation), optional global-norm clipping,
lr / entropy schedules.
"""
from __future__ import annotations

import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch
from ray_memory_management_amd.rllib.utils.schedules import make_schedule


class PGConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or PG)
        self.lr = 0.0004
        self.train_batch_size = 200
        self.rollout_fragment_length = 200
        self.num_workers = 0
        self.use_critic = False
        self.lambda_ = 1.0
        self.lr_schedule = None
        self.grad_clip = None


class OnPolicyLearner:
    """Policy-gradient family learner on one device. Subclasses define ``loss``."""

    def __init__(self, model: nn.Module, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.cfg = cfg
        self.opt = torch.optim.Adam(self.model.parameters(), lr=cfg["lr"])
        self.lr_sched = make_schedule(cfg.get("lr_schedule"), cfg["lr"])
        self.ent_sched = make_schedule(cfg.get("entropy_coeff_schedule"), cfg.get("entropy_coeff", 0.0))
        self.num_steps_trained = 0

    def _tensors(self, b: SampleBatch):
        t = lambda k, dt=None: torch.as_tensor(np.asarray(b[k]), device=self.device) if dt is None else \
            torch.as_tensor(np.asarray(b[k]), device=self.device).to(dt)  # noqa: E731
        return (t(SampleBatch.OBS), t(SampleBatch.ACTIONS, torch.int64), t(SampleBatch.ADVANTAGES, torch.float32),
                t(SampleBatch.VALUE_TARGETS, torch.float32))

    def loss(self, logits, values, act, adv, vt):
        raise NotImplementedError

    def update(self, batch: SampleBatch) -> Dict:
        c = self.cfg
        obs, act, adv, vt = self._tensors(batch)
        for g in self.opt.param_groups:
            g["lr"] = self.lr_sched(self.num_steps_trained)
        mb = int(c.get("microbatch_size") or 0) or len(act)
        self.opt.zero_grad(set_to_none=True)
        stats: Dict = {}
        nmb = (len(act) + mb - 1) // mb
        for i in range(0, len(act), mb):
            sl = slice(i, i + mb)
            logits, values = self.model(obs[sl])
            total, stats = self.loss(logits.float(), values.float(), act[sl], adv[sl], vt[sl])
            (total / nmb).backward()  # microbatches accumulate one step's gradient
        if c.get("grad_clip"):
            stats["grad_gnorm"] = float(nn.utils.clip_grad_norm_(self.model.parameters(), c["grad_clip"]))
        self.opt.step()
        self.num_steps_trained += len(act)
        stats["cur_lr"] = self.opt.param_groups[0]["lr"]
        return stats

    def compute_gradients(self, batch: SampleBatch):
        """Loss gradients for `batch` without stepping (A3C workers): ([np.ndarray per parameter], stats)."""
        obs, act, adv, vt = self._tensors(batch)
        self.model.zero_grad(set_to_none=True)
        logits, values = self.model(obs)
        total, stats = self.loss(logits.float(), values.float(), act, adv, vt)
        total.backward()
        grads = [(p.grad.detach().cpu().numpy().copy() if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
                 for p in self.model.parameters()]
        self.num_steps_trained += len(act)
        return grads, stats

    def apply_gradients(self, grads) -> Dict:
        """One optimizer step on externally computed gradients (A3C driver)."""
        c = self.cfg
        for g in self.opt.param_groups:
            g["lr"] = self.lr_sched(self.num_steps_trained)
        for p, g in zip(self.model.parameters(), grads):
            p.grad = torch.as_tensor(np.asarray(g), device=self.device, dtype=p.dtype)
        stats = {}
        if c.get("grad_clip"):
            stats["grad_gnorm"] = float(nn.utils.clip_grad_norm_(self.model.parameters(), c["grad_clip"]))
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        stats["cur_lr"] = self.opt.param_groups[0]["lr"]
        return stats

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        self.model.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})


class PGLearner(OnPolicyLearner):
    def loss(self, logits, values, act, adv, vt):
        logp = torch.log_softmax(logits, -1).gather(1, act.view(-1, 1)).squeeze(1)
        pi = -(logp * adv).mean()
        return pi, {"policy_loss": float(pi.detach())}


class PG(Algorithm):
    _config_class = PGConfig
    _learner_class = PGLearner

    def _learner_cfg(self) -> Dict:
        c = self.algo_config
        return {k: getattr(c, k, None) for k in ("lr", "lr_schedule", "grad_clip", "entropy_coeff",
                                                  "entropy_coeff_schedule", "vf_loss_coeff", "microbatch_size")}

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        cfg = {k: v for k, v in self._learner_cfg().items() if v is not None}
        self.learner = self._learner_class(copy.deepcopy(self.workers.local_worker().policy.model), cfg, device=dev)
        self._sync()

    def _sync(self):
        w = self.learner.get_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def _ma_learner(self, pid, policy):
        dev = "cuda" if self.algo_config.num_gpus and torch.cuda.is_available() else "cpu"
        cfg = {k: v for k, v in self._learner_cfg().items() if v is not None}
        return self._learner_class(copy.deepcopy(policy.model), cfg, device=dev)

    def training_step(self) -> Dict:
        if self._multi_agent:
            return self._ma_training_step()
        c = self.algo_config
        batch = self.workers.synchronous_parallel_sample(c.train_batch_size)
        self._counters["num_env_steps_sampled"] += batch.count
        self._timesteps_total += batch.count
        stats = self.learner.update(batch)
        self._counters["num_env_steps_trained"] += batch.count
        self._sync()
        return stats

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, weights):
        self.learner.set_weights(weights)
        self._sync()


DEFAULT_CONFIG = PGConfig().to_dict()
