"""GPU PPO learner + on-device rollout sampler (the MI355X fast path of RLlib PPO).

Parity: reference rllib/algorithms/ppo/ppo_torch_policy.py (loss: clipped surrogate, clipped
value loss, entropy bonus, KL penalty with adaptive coefficient), rllib/algorithms/ppo/ppo.py
(training_step: sample → standardize advantages → num_sgd_iter × minibatch SGD → update KL),
rllib/execution/multi_gpu_learner_thread.py + train_ops.multi_gpu_train_one_step (multi-GPU
learner). Design here: one learner process per GPU (torch.distributed over RCCL/xGMI, DDP with a
single flat gradient bucket since the Atari net is ~1M params), the whole batch resident in HBM,
minibatches gathered on-device by the K2 kernel, GAE by the K3 kernel, the PPO loss + its gradient
by the fused K5 kernel, bf16 autocast for the convolutions.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import torch
import torch.nn as nn

from ray_memory_management_amd import ops
from ray_memory_management_amd.rllib.distributions import Categorical, dist_class_for
from ray_memory_management_amd.rllib.sample_batch import SampleBatch

DEFAULT_PPO = dict(
    gamma=0.99, lambda_=0.95, kl_coeff=0.5, kl_target=0.01, clip_param=0.1, vf_clip_param=10.0,
    vf_loss_coeff=1.0, entropy_coeff=0.01, lr=5e-5, train_batch_size=5000, sgd_minibatch_size=500,
    num_sgd_iter=10, grad_clip=None, use_fused_loss=True, bf16=True, standardize_advantages=True,
)


class PPOLearner:
    def __init__(self, model: nn.Module, config: Optional[dict] = None, device="cuda", process_group=None,
                 action_space=None):
        self.cfg = {**DEFAULT_PPO, **(config or {})}
        self.device = torch.device(device)
        self.model = model.to(self.device)
        if self.device.type == "cuda":
            self.model = self.model.to(memory_format=torch.channels_last)
        self.dist_cls = dist_class_for(action_space) if action_space is not None else Categorical
        self.ddp = None
        self.pg = process_group
        if torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size(process_group) > 1:
            # one flat bucket: the whole gradient in a single RCCL all-reduce per minibatch step
            nparams = sum(p.numel() for p in self.model.parameters())
            self.ddp = nn.parallel.DistributedDataParallel(
                self.model, device_ids=[self.device.index] if self.device.type == "cuda" else None,
                process_group=process_group, bucket_cap_mb=max(1, nparams * 4 // (1 << 20) + 1),
                gradient_as_bucket_view=True, broadcast_buffers=False)
        self.net = self.ddp if self.ddp is not None else self.model
        fused = self.device.type == "cuda"
        try:
            self.opt = torch.optim.Adam(self.model.parameters(), lr=self.cfg["lr"], fused=fused)
        except (TypeError, RuntimeError):
            self.opt = torch.optim.Adam(self.model.parameters(), lr=self.cfg["lr"])
        self.kl_coeff = float(self.cfg["kl_coeff"])
        self.stats: Dict[str, float] = {}

    # ------------------------------------------------------------------ loss
    def _forward(self, obs):
        if self.cfg["bf16"] and self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, v = self.net(obs)
            return logits.float(), v.float()
        return self.net(obs)

    def loss(self, mb: SampleBatch):
        c = self.cfg
        logits, v = self._forward(mb[SampleBatch.OBS])
        dist = self.dist_cls(logits)
        old = self.dist_cls(mb[SampleBatch.ACTION_DIST_INPUTS])
        logp = dist.logp(mb[SampleBatch.ACTIONS])
        ent = dist.entropy()
        kl = old.kl(dist).mean()
        if c["use_fused_loss"] and self.device.type == "cuda":
            total, means = ops.ppo_loss(logp, mb[SampleBatch.ACTION_LOGP], mb[SampleBatch.ADVANTAGES], v,
                                        mb[SampleBatch.VALUE_TARGETS], ent, c["clip_param"], c["vf_clip_param"],
                                        c["vf_loss_coeff"], c["entropy_coeff"])
        else:
            total, means = ops.ppo_loss_reference(logp, mb[SampleBatch.ACTION_LOGP], mb[SampleBatch.ADVANTAGES], v,
                                                  mb[SampleBatch.VALUE_TARGETS], ent, c["clip_param"],
                                                  c["vf_clip_param"], c["vf_loss_coeff"], c["entropy_coeff"])
        if self.kl_coeff > 0:
            total = total + self.kl_coeff * kl
        return total, means, kl

    # ------------------------------------------------------------------ update
    def update(self, batch: SampleBatch) -> Dict[str, float]:
        """num_sgd_iter epochs of shuffled minibatch SGD over a device-resident batch."""
        c = self.cfg
        if c["standardize_advantages"]:
            a = batch[SampleBatch.ADVANTAGES].float()
            batch[SampleBatch.ADVANTAGES] = (a - a.mean()) / a.std().clamp_min(1e-4)
        n = batch.count
        mbs = min(c["sgd_minibatch_size"], n)
        acc = torch.zeros(5, device=self.device)
        steps = 0
        for _ in range(c["num_sgd_iter"]):
            for mb in batch.minibatches(mbs, shuffle=True):
                total, means, kl = self.loss(mb)
                self.opt.zero_grad(set_to_none=True)
                total.backward()
                if c["grad_clip"]:
                    nn.utils.clip_grad_norm_(self.model.parameters(), c["grad_clip"])
                self.opt.step()
                acc += torch.cat([total.detach().reshape(1), means[:3].detach(), kl.detach().reshape(1)])
                steps += 1
        acc = (acc / max(steps, 1)).tolist()  # one host sync per update
        kl_mean = acc[4]
        # adaptive KL coefficient (reference ppo.py UpdateKL)
        if kl_mean > 2.0 * c["kl_target"]:
            self.kl_coeff *= 1.5
        elif kl_mean < 0.5 * c["kl_target"]:
            self.kl_coeff *= 0.5
        self.stats = {"total_loss": acc[0], "policy_loss": acc[1], "vf_loss": acc[2], "entropy": acc[3],
                      "kl": kl_mean, "cur_kl_coeff": self.kl_coeff, "num_sgd_steps": steps}
        return self.stats

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        self.model.load_state_dict(w)


class GPURolloutSampler:
    """Samples `fragment` steps from a device-resident vectorised env with on-GPU inference and
    postprocesses with the GAE kernel. Output: a flat SampleBatch of fragment*num_envs rows in HBM."""

    def __init__(self, env, model: nn.Module, fragment: int, gamma=0.99, lam=0.95, bf16=True):
        self.env = env
        self.model = model
        self.T = fragment
        self.B = env.num_envs
        self.gamma, self.lam, self.bf16 = gamma, lam, bf16
        dev = env.device
        self.obs = env.reset()
        T, B = self.T, self.B
        self.buf_obs = torch.empty((T, B, *self.obs.shape[1:]), dtype=self.obs.dtype, device=dev)
        self.buf_act = torch.empty((T, B), dtype=torch.int64, device=dev)
        self.buf_logp = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_vf = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_rew = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_done = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_logits = None

    @torch.no_grad()
    def _policy(self, obs):
        if self.bf16:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, v = self.model(obs)
            return logits.float(), v.float()
        return self.model(obs)

    @torch.no_grad()
    def sample(self) -> SampleBatch:
        for t in range(self.T):
            logits, v = self._policy(self.obs)
            if self.buf_logits is None:
                self.buf_logits = torch.empty((self.T, self.B, logits.shape[-1]), dtype=torch.float32,
                                              device=logits.device)
            d = Categorical(logits)
            a = d.sample()
            self.buf_obs[t].copy_(self.obs)
            self.buf_act[t] = a
            self.buf_logp[t] = d.logp(a)
            self.buf_vf[t] = v
            self.buf_logits[t] = logits
            self.obs, r, done = self.env.step(a)
            self.buf_rew[t] = r
            self.buf_done[t] = done
        _, last_v = self._policy(self.obs)
        adv, ret = ops.gae(self.buf_rew, self.buf_vf, self.buf_done, last_v, self.gamma, self.lam)
        n = self.T * self.B
        return SampleBatch({
            SampleBatch.OBS: self.buf_obs.view(n, *self.buf_obs.shape[2:]),
            SampleBatch.ACTIONS: self.buf_act.view(n),
            SampleBatch.ACTION_LOGP: self.buf_logp.view(n),
            SampleBatch.VF_PREDS: self.buf_vf.view(n),
            SampleBatch.ACTION_DIST_INPUTS: self.buf_logits.view(n, -1),
            SampleBatch.REWARDS: self.buf_rew.view(n),
            SampleBatch.DONES: self.buf_done.view(n),
            SampleBatch.ADVANTAGES: adv.view(n),
            SampleBatch.VALUE_TARGETS: ret.view(n),
        })


def smoke_step(device="cuda:0"):
    """One tiny PPO iteration (sample → GAE kernel → fused-loss SGD step) on `device`."""
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(0)
    env = GPUSyntheticAtariVectorEnv(8, device, num_actions=4)
    model = VisionNetwork(4).to(device)
    learner = PPOLearner(model, {"sgd_minibatch_size": 32, "num_sgd_iter": 1}, device=device,
                         action_space=env.action_space)
    sampler = GPURolloutSampler(env, learner.model, fragment=8)
    batch = sampler.sample()
    stats = learner.update(batch)
    torch.cuda.synchronize()
    return stats
