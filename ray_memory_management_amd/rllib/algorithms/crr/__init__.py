"""CRR: critic-regularized regression (offline actor-critic).

Parity: reference rllib/algorithms/crr/crr.py (CRRConfig: weight_type "bin" | "exp", temperature
1.0, max_weight 20.0, advantage_type "mean" | "max" | "expectation", n_action_sample 4, twin_q,
target_update_grad_intervals 100, tau 5e-4, actor_hidden_activation / critic_hidden_activation relu,
train_batch_size 128) and torch/crr_torch_policy.py (actor loss −mean(f(Â(s, a_data)) ·
log π(a_data|s)) with Â = Q(s, a_data) − V̂(s), V̂ from `n_action_sample` policy actions;
critic TD loss against the target networks with a′ ~ π′(s′)).
"""
from __future__ import annotations

from typing import Dict

import torch

from ray_memory_management_amd.rllib.algorithms.ddpg import DDPGLearner, polyak_update
from ray_memory_management_amd.rllib.algorithms.sac import SAC, SACConfig, SACPolicy


class CRRPolicy(SACPolicy):
    pass


class CRRConfig(SACConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or CRR)
        self.weight_type = "bin"
        self.temperature = 1.0
        self.max_weight = 20.0
        self.advantage_type = "mean"
        self.n_action_sample = 4
        self.twin_q = True
        self.target_update_grad_intervals = 100
        self.tau = 5e-4
        self.train_batch_size = 128
        self.num_steps_sampled_before_learning_starts = 0
        self.actor_lr = 3e-4
        self.critic_lr = 3e-4
        self.use_huber = False
        self.policy_class = "ray_memory_management_amd.rllib.algorithms.crr.CRRPolicy"


class CRRLearner(DDPGLearner):
    def critic_target(self, nobs, rew, done):
        c = self.cfg
        with torch.no_grad():
            a2, _ = self.target.sample_squashed(nobs)
            q1t, q2t = self.target.q(nobs, a2)
            qt = torch.min(q1t, q2t) if q2t is not None else q1t
            return rew + (c["gamma"] ** c["n_step"]) * (1.0 - done) * qt

    def _advantage(self, obs, act):
        c = self.cfg
        with torch.no_grad():
            q1, q2 = self.m.q(obs, act)
            q = torch.min(q1, q2) if q2 is not None else q1
            B, N = obs.shape[0], int(c.get("n_action_sample", 4))
            o = obs.flatten(1).float().unsqueeze(1).expand(B, N, -1).reshape(B * N, -1)
            a, _ = self.m.sample_squashed(o)
            qa1, qa2 = self.m.q(o, a)
            qs = (torch.min(qa1, qa2) if qa2 is not None else qa1).view(B, N)
            v = qs.max(1).values if c.get("advantage_type") == "max" else qs.mean(1)
            return q - v

    def update(self, b) -> Dict:
        c = self.cfg
        obs, act, rew, done, nobs, w = self._tensors(b)
        target = self.critic_target(nobs, rew, done)
        q1, q2 = self.m.q(obs, act)
        td = q1 - target
        critic_loss = (self._critic_err(td) + (self._critic_err(q2 - target) if q2 is not None else 0.0)).mean()
        self.critic_opt.zero_grad(set_to_none=True)
        critic_loss.backward()
        self.critic_opt.step()
        adv = self._advantage(obs, act)
        if c.get("weight_type") == "exp":
            wts = torch.exp(adv / float(c.get("temperature", 1.0))).clamp(max=float(c.get("max_weight", 20.0)))
        else:
            wts = (adv > 0).float()
        actor_loss = -(wts * self.m.logp_of(obs, act)).mean()
        self.actor_opt.zero_grad(set_to_none=True)
        actor_loss.backward()
        self.actor_opt.step()
        self.steps += 1
        if self.steps % max(1, int(c.get("target_update_grad_intervals", 100))) == 0:
            polyak_update(self.target, self.m, c["tau"])
        return {"critic_loss": float(critic_loss.detach()), "actor_loss": float(actor_loss.detach()),
                "mean_q": float(q1.detach().mean()), "mean_weight": float(wts.mean()),
                "td_error": td.detach().abs().cpu().numpy()}


class CRR(SAC):
    _config_class = CRRConfig
    _learner_class = CRRLearner

    def validate_config(self, c):
        super().validate_config(c)
        if not c.input_ or c.input_ == "sampler":
            raise ValueError("CRR is an offline algorithm: set config.offline_data(input_=<recorded data>)")

    def _learner_cfg(self, c) -> Dict:
        d = super()._learner_cfg(c)
        d.update(actor_lr=c.actor_lr, critic_lr=c.critic_lr, weight_type=c.weight_type, temperature=c.temperature,
                 max_weight=c.max_weight, advantage_type=c.advantage_type, n_action_sample=c.n_action_sample,
                 target_update_grad_intervals=c.target_update_grad_intervals, target_network_update_freq=1)
        return d


DEFAULT_CONFIG = CRRConfig().to_dict()
