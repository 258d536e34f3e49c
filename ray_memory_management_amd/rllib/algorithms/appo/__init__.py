"""APPO: IMPALA's asynchronous architecture with a PPO-style clipped surrogate.

Parity: reference rllib/algorithms/appo/appo.py (APPOConfig defaults: clip_param 0.4, use_kl_loss,
kl_coeff / kl_target adaptation, target_update_frequency, tau) and appo_torch_policy.py (V-trace
targets from the TARGET network's action log-probs; is_ratio = clamp(exp(behaviour - target), 0, 2);
surrogate min(adv * r, adv * clamp(r, 1 - clip, 1 + clip)) with r = is_ratio * exp(logp - behaviour);
mean losses; KL(behaviour || current) term when use_kl_loss).

The target network is a second copy of the model on the learner device; it is refreshed (soft
update with `tau`) once the learner has trained on `target_update_frequency * train_batch_size *
num_sgd_iter` samples since the last refresh, which is also when the KL coefficient is adapted.
"""
from __future__ import annotations

import copy
from typing import Dict

import torch

from ray_memory_management_amd import ops
from ray_memory_management_amd.rllib.algorithms.impala import Impala, ImpalaConfig, VTraceLearner


class APPOConfig(ImpalaConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or APPO)
        self.vtrace = True
        self.use_critic = True
        self.use_gae = True
        self.lambda_ = 1.0
        self.clip_param = 0.4
        self.use_kl_loss = False
        self.kl_coeff = 1.0
        self.kl_target = 0.01
        self.target_update_frequency = 1
        self.tau = 1.0
        self.replay_buffer_num_slots = 100
        self.num_gpus = 0


class APPOLearner(VTraceLearner):
    def __init__(self, model, cfg: Dict, device="cpu"):
        super().__init__(model, cfg, device)
        self.target = copy.deepcopy(self.model)
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.kl_coeff = float(cfg.get("kl_coeff", 1.0))
        self._trained_since_target = 0
        self._kl_hist = []
        self.num_target_updates = 0

    def loss(self, T, b, last_obs):
        c = self.cfg
        logits, values, boot = self._forward(self.model, b, last_obs)
        lsm = torch.log_softmax(logits, -1)
        act = b["actions"].unsqueeze(-1)
        logp = lsm.gather(2, act).squeeze(-1)
        blogp = b["action_logp"]
        with torch.no_grad():
            tlogits, _, _ = self._forward(self.target, b, last_obs)
            old_logp = torch.log_softmax(tlogits, -1).gather(2, act).squeeze(-1)
            vs, adv = ops.vtrace(blogp, old_logp, b["rewards"], values, b["dones"], boot, c["gamma"],
                                 c["vtrace_clip_rho_threshold"], c["vtrace_clip_pg_rho_threshold"],
                                 lam=c.get("lambda", 1.0))
            is_ratio = torch.clamp(torch.exp(blogp - old_logp), 0.0, 2.0)
        ratio = is_ratio * torch.exp(logp - blogp)
        clip = c["clip_param"]
        surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
        pi_loss = -surr.mean()
        vf_loss = 0.5 * ((values - vs) ** 2).mean()
        ent = -(lsm.exp() * lsm).sum(-1).mean()
        blsm = torch.log_softmax(b["action_dist_inputs"].float(), -1)
        kl = (blsm.exp() * (blsm - lsm)).sum(-1).mean()  # KL(behaviour || current)
        ent_coeff = self.ent_sched(self.num_steps_trained)
        total = pi_loss + c["vf_loss_coeff"] * vf_loss - ent_coeff * ent
        if c.get("use_kl_loss"):
            total = total + self.kl_coeff * kl
        self._kl_hist.append(kl.detach())
        return total, {"policy_loss": float(pi_loss.detach()), "vf_loss": float(vf_loss.detach()),
                       "entropy": float(ent.detach()), "entropy_coeff": float(ent_coeff), "kl": float(kl.detach()),
                       "kl_coeff": self.kl_coeff, "mean_is_ratio": float(is_ratio.mean()),
                       "vs_mean": float(vs.mean())}

    def after_update(self, stats: Dict, rows: int):
        c = self.cfg
        self._trained_since_target += rows
        need = c["target_update_frequency"] * c["train_batch_size"] * c.get("num_sgd_iter", 1)
        if self._trained_since_target < need:
            return
        self._trained_since_target = 0
        tau = float(c.get("tau", 1.0))
        with torch.no_grad():
            for pt, p in zip(self.target.parameters(), self.model.parameters()):
                pt.mul_(1.0 - tau).add_(p, alpha=tau)
            for bt, b in zip(self.target.buffers(), self.model.buffers()):
                bt.copy_(b)
        self.num_target_updates += 1
        stats["num_target_updates"] = self.num_target_updates
        if c.get("use_kl_loss") and self._kl_hist:  # reference appo: adapt on the mean sampled KL
            kl = float(torch.stack(self._kl_hist).mean())
            if kl > 2.0 * c["kl_target"]:
                self.kl_coeff *= 1.5
            elif kl < 0.5 * c["kl_target"]:
                self.kl_coeff *= 0.5
        self._kl_hist = []


class APPO(Impala):
    _config_class = APPOConfig
    _learner_class = APPOLearner

    def _learner_cfg(self) -> Dict:
        c = self.algo_config
        d = super()._learner_cfg()
        d.update({k: getattr(c, k) for k in ("clip_param", "use_kl_loss", "kl_coeff", "kl_target",
                                             "target_update_frequency", "tau", "train_batch_size")})
        d["lambda"] = c.lambda_
        return d


DEFAULT_CONFIG = APPOConfig().to_dict()
