"""SAC (soft actor-critic): tanh-squashed Gaussian actor, twin soft-Q critics with Polyak targets,
automatic entropy-temperature tuning.

Parity: reference rllib/algorithms/sac/sac.py (SACConfig defaults: twin_q, tau 5e-3, initial_alpha
1.0, target_entropy "auto" = -|A|, n_step 1, train_batch_size 256, separate actor / critic /
entropy learning rates 3e-4, Polyak update every step), sac_torch_model.py (policy + Q nets,
log-std clamp) and sac_torch_policy.py (critic target r + γⁿ(1-d)(min Q'(s',a') - α log π(a'|s')),
Huber critic loss with importance weights, actor loss E[α log π - min Q], alpha loss
-log α · (log π + H̄)). Continuous (Box) action spaces.
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.ddpg import (ContinuousPolicy, DDPGConfig, DDPGLearner,
                                                             OffPolicyContinuousAlgorithm, polyak_update)


class SACPolicy(ContinuousPolicy):
    stochastic = True


class SACConfig(DDPGConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or SAC)
        self.twin_q = True
        self.actor_hiddens = [256, 256]
        self.critic_hiddens = [256, 256]
        self.tau = 5e-3
        self.initial_alpha = 1.0
        self.target_entropy = "auto"
        self.n_step = 1
        self.train_batch_size = 256
        self.target_network_update_freq = 0
        self.num_steps_sampled_before_learning_starts = 1500
        self.replay_buffer_config = {**self.replay_buffer_config, "capacity": 1000000}
        self.optimization = {"actor_learning_rate": 3e-4, "critic_learning_rate": 3e-4,
                             "entropy_learning_rate": 3e-4}
        self.use_huber = True
        self.l2_reg = 0.0
        self.grad_clip = None
        self.exploration_config = {"type": "StochasticSampling"}
        self.policy_class = "ray_memory_management_amd.rllib.algorithms.sac.SACPolicy"

    def training(self, *, optimization_config=None, **kwargs) -> "SACConfig":
        if optimization_config is not None:
            self.optimization = {**self.optimization, **optimization_config}
        return super().training(**kwargs)


class SACLearner(DDPGLearner):
    def __init__(self, model, cfg: Dict, device="cpu"):
        super().__init__(model, {**cfg, "actor_lr": cfg["actor_learning_rate"],
                                 "critic_lr": cfg["critic_learning_rate"]}, device)
        te = cfg.get("target_entropy", "auto")
        self.target_entropy = -float(self.m.act_dim) if te in (None, "auto") else float(te)
        self.log_alpha = torch.tensor(math.log(cfg.get("initial_alpha", 1.0)), device=self.device, requires_grad=True)
        self.alpha_opt = torch.optim.Adam([self.log_alpha], lr=cfg["entropy_learning_rate"])

    def critic_target(self, nobs, rew, done):
        c = self.cfg
        with torch.no_grad():
            a2, logp2 = self.m.sample_squashed(nobs)  # next actions from the CURRENT policy
            q1t, q2t = self.target.q(nobs, a2)
            qt = torch.min(q1t, q2t) if q2t is not None else q1t
            return rew + (c["gamma"] ** c["n_step"]) * (1.0 - done) * (qt - self.log_alpha.exp() * logp2)

    def update(self, b) -> Dict:
        obs, act, rew, done, nobs, w = self._tensors(b)
        target = self.critic_target(nobs, rew, done)
        q1, q2 = self.m.q(obs, act)
        td = q1 - target
        err = self._critic_err(td) + (self._critic_err(q2 - target) if q2 is not None else 0.0)
        critic_loss = (err * w).mean() if w is not None else err.mean()
        self.critic_opt.zero_grad(set_to_none=True)
        critic_loss.backward()
        if self.cfg.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.critic_params, self.cfg["grad_clip"])
        self.critic_opt.step()
        # actor: reparameterised sample through the (just-updated) critics
        a_pi, logp = self.m.sample_squashed(obs)
        qa1, qa2 = self.m.q(obs, a_pi)
        q_pi = torch.min(qa1, qa2) if qa2 is not None else qa1
        alpha = self.log_alpha.exp().detach()
        actor_loss = (alpha * logp - q_pi).mean()
        self.actor_opt.zero_grad(set_to_none=True)
        actor_loss.backward()
        if self.cfg.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.m.actor.parameters(), self.cfg["grad_clip"])
        self.actor_opt.step()
        self.critic_opt.zero_grad(set_to_none=True)
        alpha_loss = -(self.log_alpha * (logp.detach() + self.target_entropy)).mean()
        self.alpha_opt.zero_grad(set_to_none=True)
        alpha_loss.backward()
        self.alpha_opt.step()
        self.steps += 1
        if not self.cfg.get("target_network_update_freq"):
            polyak_update(self.target, self.m, self.cfg["tau"])
        return {"critic_loss": float(critic_loss.detach()), "actor_loss": float(actor_loss.detach()),
                "alpha_loss": float(alpha_loss.detach()), "alpha_value": float(alpha),
                "log_alpha_value": float(self.log_alpha.detach()), "target_entropy": self.target_entropy,
                "mean_q": float(q1.detach().mean()), "policy_entropy": float(-logp.detach().mean()),
                "td_error": td.detach().abs().cpu().numpy()}

    def get_state(self):
        s = super().get_state()
        s["log_alpha"] = float(self.log_alpha.detach())
        return s

    def set_state(self, s):
        super().set_state(s)
        with torch.no_grad():
            self.log_alpha.fill_(s.get("log_alpha", 0.0))


class SAC(OffPolicyContinuousAlgorithm):
    _config_class = SACConfig
    _learner_class = SACLearner

    def _learner_cfg(self, c) -> Dict:
        d = super()._learner_cfg(c)
        d.update(c.optimization)
        d.update(initial_alpha=c.initial_alpha, target_entropy=c.target_entropy)
        return d


DEFAULT_CONFIG = SACConfig().to_dict()
