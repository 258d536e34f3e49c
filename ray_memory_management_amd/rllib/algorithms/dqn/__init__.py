"""DQN (double / dueling Q-learning with a replay buffer and a target network).

Parity: reference rllib/algorithms/dqn/dqn.py (DQNConfig defaults, training_step: sample →
store in the replay buffer → sample train batches → learn → update priorities → target-network
sync every `target_network_update_freq` sampled steps → broadcast weights),
rllib/algorithms/dqn/dqn_torch_policy.py (Huber TD loss, double-Q action selection, dueling
aggregation, importance weights, grad clipping) and rllib/utils/exploration/epsilon_greedy.py.

MI355X design: the learner's Q and target networks and the replay buffer live on the learner
device; with ``num_gpus > 0`` the buffer is HBM-resident and training batches are gathered with the
K2 row-gather kernel, so the per-update host traffic is only the new rollouts.
"""
from __future__ import annotations

import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.policy import TorchPolicy
from ray_memory_management_amd.rllib.sample_batch import SampleBatch, concat_samples
from ray_memory_management_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer
from ray_memory_management_amd.rllib.utils.schedules import PiecewiseSchedule


def q_values(model, obs, dueling: bool):
    """Q(s, .) from the policy network: logits are the advantage stream, the value head the
    state-value stream when dueling (Q = V + A - mean A)."""
    a, v = model(obs)
    a = a.float()
    if dueling:
        return v.float().unsqueeze(-1) + a - a.mean(dim=-1, keepdim=True)
    return a


class DQNPolicy(TorchPolicy):
    """Epsilon-greedy Q policy for rollout workers."""

    def __init__(self, observation_space, action_space, config: Dict, device="cpu"):
        super().__init__(observation_space, action_space, config, device)
        ec = dict(config.get("exploration_config") or {})
        if ec.get("type") == "PerWorkerEpsilonGreedy":
            # Ape-X: worker i of N explores with the constant eps 0.4^(1 + 7 (i-1)/(N-1)); the local
            # (driver) worker acts greedily (reference exploration/per_worker_epsilon_greedy.py)
            i, n = int(config.get("worker_index", 0)), int(config.get("num_workers", 0))
            e = 0.0 if i == 0 else 0.4 ** (1 + 7.0 * (i - 1) / max(1, n - 1))
            self.eps = PiecewiseSchedule([[0, e], [1, e]])
        else:
            self.eps = PiecewiseSchedule([[0, ec.get("initial_epsilon", 1.0)],
                                          [ec.get("epsilon_timesteps", 10000), ec.get("final_epsilon", 0.02)]])
        self.dueling = bool(config.get("dueling", True))
        self._rng = np.random.default_rng(config.get("seed"))

    @torch.no_grad()
    def compute_actions(self, obs_batch, explore: bool = True):
        obs = torch.as_tensor(np.asarray(obs_batch), device=self.device)
        q = q_values(self.model, obs, self.dueling)
        a = q.argmax(dim=-1).cpu().numpy()
        if explore:
            eps = self.eps(self.global_timestep)
            rnd = self._rng.random(len(a)) < eps
            a = np.where(rnd, self._rng.integers(0, q.shape[-1], size=len(a)), a)
        self.global_timestep += len(a)
        qn = q.cpu().numpy()
        return a, [], {SampleBatch.ACTION_LOGP: np.zeros(len(a), np.float32),
                       SampleBatch.VF_PREDS: qn.max(-1).astype(np.float32),
                       SampleBatch.ACTION_DIST_INPUTS: qn.astype(np.float32)}

    @torch.no_grad()
    def value(self, obs_batch):
        obs = torch.as_tensor(np.asarray(obs_batch), device=self.device)
        return q_values(self.model, obs, self.dueling).max(-1).values.cpu().numpy()


class DQNConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or DQN)
        self.lr = 5e-4
        self.gamma = 0.99
        self.train_batch_size = 32
        self.rollout_fragment_length = 4
        self.num_workers = 0
        self.target_network_update_freq = 500
        self.num_steps_sampled_before_learning_starts = 1000
        self.replay_buffer_config = {"type": "MultiAgentPrioritizedReplayBuffer", "capacity": 50000,
                                     "prioritized_replay_alpha": 0.6, "prioritized_replay_beta": 0.4,
                                     "prioritized_replay_eps": 1e-6}
        self.double_q = True
        self.dueling = True
        self.n_step = 1
        self.grad_clip = 40.0
        self.training_intensity = None
        self.min_sample_timesteps_per_iteration = 1000
        self.exploration_config = {"type": "EpsilonGreedy", "initial_epsilon": 1.0, "final_epsilon": 0.02,
                                   "epsilon_timesteps": 10000}
        self.model = {**self.model, "vf_share_layers": True}
        self.policy_class = "ray_memory_management_amd.rllib.algorithms.dqn.DQNPolicy"

    def training(self, *, target_network_update_freq=None, replay_buffer_config=None, double_q=None, dueling=None,
                 n_step=None, grad_clip=None, training_intensity=None,
                 num_steps_sampled_before_learning_starts=None, **kwargs) -> "DQNConfig":
        super().training(**kwargs)
        for k, v in dict(target_network_update_freq=target_network_update_freq, double_q=double_q, dueling=dueling,
                         n_step=n_step, grad_clip=grad_clip, training_intensity=training_intensity,
                         num_steps_sampled_before_learning_starts=num_steps_sampled_before_learning_starts).items():
            if v is not None:
                setattr(self, k, v)
        if replay_buffer_config is not None:
            self.replay_buffer_config = {**self.replay_buffer_config, **replay_buffer_config}
        return self


class DQNLearner:
    """Q / target networks + Adam on one device; one `update` = one SGD step on a train batch."""

    def __init__(self, model: nn.Module, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.q = model.to(self.device)
        self.target = copy.deepcopy(self.q)
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.cfg = cfg
        self.opt = torch.optim.Adam(self.q.parameters(), lr=cfg["lr"], eps=1e-8)
        self.steps = 0

    def update(self, b: SampleBatch) -> Dict:
        c = self.cfg
        dev = self.device
        t = lambda k, dt=None: torch.as_tensor(b[k], device=dev) if dt is None else \
            torch.as_tensor(b[k], device=dev).to(dt)  # noqa: E731
        obs, nobs = t(SampleBatch.OBS), t(SampleBatch.NEXT_OBS)
        act = t(SampleBatch.ACTIONS, torch.int64)
        rew, done = t(SampleBatch.REWARDS, torch.float32), t(SampleBatch.DONES, torch.float32)
        w = t("weights", torch.float32) if "weights" in b else torch.ones_like(rew)
        q_t = q_values(self.q, obs, c["dueling"])
        q_sel = q_t.gather(1, act.view(-1, 1)).squeeze(1)
        with torch.no_grad():
            q_tp1_target = q_values(self.target, nobs, c["dueling"])
            if c["double_q"]:
                a_star = q_values(self.q, nobs, c["dueling"]).argmax(-1, keepdim=True)
            else:
                a_star = q_tp1_target.argmax(-1, keepdim=True)
            q_tp1 = q_tp1_target.gather(1, a_star).squeeze(1)
            target = rew + (c["gamma"] ** c["n_step"]) * (1.0 - done) * q_tp1
        td = q_sel - target
        loss = (w * torch.nn.functional.huber_loss(q_sel, target, reduction="none", delta=1.0)).mean()
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if c.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.q.parameters(), c["grad_clip"])
        self.opt.step()
        self.steps += 1
        return {"loss": float(loss.detach()), "mean_q": float(q_sel.detach().mean()),
                "td_error": td.detach().abs().cpu().numpy()}

    def sync_target(self):
        self.target.load_state_dict(self.q.state_dict())

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.q.state_dict().items()}

    def set_weights(self, w):
        self.q.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})
        self.sync_target()


class DQN(Algorithm):
    _config_class = DQNConfig

    def validate_config(self, c):
        super().validate_config(c)
        if c.n_step < 1:
            raise ValueError("n_step must be >= 1")

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        local = self.workers.local_worker()
        self.learner = DQNLearner(copy.deepcopy(local.policy.model),
                                  dict(lr=c.lr, gamma=c.gamma, n_step=c.n_step, double_q=c.double_q, dueling=c.dueling,
                                       grad_clip=c.grad_clip), device=dev)
        rb = dict(c.replay_buffer_config)
        prioritized = "Prioritized" in str(rb.get("type", ""))
        buf_dev = dev if dev != "cpu" else None
        if prioritized:
            self.buffer = PrioritizedReplayBuffer(rb.get("capacity", 50000), alpha=rb.get("prioritized_replay_alpha", 0.6),
                                                  device=buf_dev, seed=c.seed)
        else:
            self.buffer = ReplayBuffer(rb.get("capacity", 50000), device=buf_dev, seed=c.seed)
        self._prioritized = prioritized
        self._last_target_update = 0
        self._sync()

    def _sync(self):
        w = self.learner.get_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def _sample(self) -> SampleBatch:
        if self.workers.remote_workers():
            return concat_samples(ray.get([w.sample.remote() for w in self.workers.remote_workers()]))
        return self.workers.local_worker().sample()

    def training_step(self) -> Dict:
        c = self.algo_config
        batch = self._sample()
        keep = [SampleBatch.OBS, SampleBatch.NEXT_OBS, SampleBatch.ACTIONS, SampleBatch.REWARDS, SampleBatch.DONES]
        batch = SampleBatch({k: batch[k] for k in keep})
        self.buffer.add(batch)
        n = batch.count
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        ts = self._counters["num_env_steps_sampled"]
        stats = {}
        if ts > c.num_steps_sampled_before_learning_starts:
            intensity = c.training_intensity
            n_updates = max(1, int(round(intensity * n / c.train_batch_size))) if intensity else 1
            rb = c.replay_buffer_config
            for _ in range(n_updates):
                tb = self.buffer.sample(c.train_batch_size, beta=rb.get("prioritized_replay_beta", 0.4))
                out = self.learner.update(tb)
                if self._prioritized:
                    self.buffer.update_priorities(tb["batch_indexes"],
                                                  out["td_error"] + rb.get("prioritized_replay_eps", 1e-6))
                stats = {k: v for k, v in out.items() if k != "td_error"}
                self._counters["num_env_steps_trained"] += c.train_batch_size
            if ts - self._last_target_update >= c.target_network_update_freq:
                self.learner.sync_target()
                self._last_target_update = ts
                self._counters["num_target_updates"] += 1
            self._sync()
        stats["epsilon"] = float(self.workers.local_worker().policy.eps(
            self.workers.local_worker().policy.global_timestep)) if not self.workers.remote_workers() else None
        stats["replay_buffer"] = self.buffer.stats()
        return stats

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, weights):
        self.learner.set_weights(weights)
        self._sync()


DEFAULT_CONFIG = DQNConfig().to_dict()
