"""GPU PPO learner + on-device rollout sampler (the MI355X fast path of RLlib PPO).

Parity: reference rllib/algorithms/ppo/ppo_torch_policy.py (loss: clipped surrogate, clipped
value loss, entropy bonus, KL penalty with adaptive coefficient), rllib/algorithms/ppo/ppo.py
(training_step: sample → standardize advantages → num_sgd_iter × minibatch SGD → update KL),
rllib/execution/multi_gpu_learner_thread.py + train_ops.multi_gpu_train_one_step (multi-GPU
learner).

MI355X design:
  * one learner process per GPU; gradients live in ONE flat fp32 bucket (every ``p.grad`` is a view
    into it) so the data-parallel sync is a single RCCL all-reduce per minibatch step over xGMI —
    the Atari net is ~1M params (4 MB), far below where splitting buckets pays on a 7-link ring;
  * the batch stays in HBM: minibatches are gathered on-device (K2), frames converted to bf16 NHWC by
    K2b, GAE by K3, the PPO loss + its gradient by the fused K5 kernel, bf16 autocast convolutions;
  * launch overhead is removed with HIP graphs: one graph per rollout step (policy forward, action
    sampling, env step, writes into the [T, B] buffers at a device-side step counter) and one per SGD
    step (zero grads, gather, forward, fused loss, backward, [all-reduce], capturable fused Adam).
"""
from __future__ import annotations

import os
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
    use_graphs=True, allreduce_in_graph=True,
)

_LOSS_KEYS = (SampleBatch.OBS, SampleBatch.ACTIONS, SampleBatch.ACTION_LOGP, SampleBatch.ACTION_DIST_INPUTS,
              SampleBatch.ADVANTAGES, SampleBatch.VALUE_TARGETS)


def _graphs_enabled(cfg, device) -> bool:
    return bool(cfg.get("use_graphs")) and device.type == "cuda" and not os.environ.get("RMM_NO_GRAPHS")


class PPOLearner:
    def __init__(self, model: nn.Module, config: Optional[dict] = None, device="cuda", process_group=None,
                 action_space=None):
        self.cfg = {**DEFAULT_PPO, **(config or {})}
        self.device = torch.device(device)
        self.model = model.to(self.device)
        if self.device.type == "cuda":
            self.model = self.model.to(memory_format=torch.channels_last)
        self.dist_cls = dist_class_for(action_space) if action_space is not None else Categorical
        self.pg = process_group
        self.world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world = torch.distributed.get_world_size(process_group)
        params = [p for p in self.model.parameters() if p.requires_grad]
        self.params = params
        if self.world > 1:  # identical initial weights: broadcast rank 0's
            with torch.no_grad():
                flat = torch.cat([p.detach().reshape(-1) for p in params])
                torch.distributed.broadcast(flat, src=torch.distributed.get_global_rank(process_group, 0)
                                            if process_group is not None else 0, group=process_group)
                off = 0
                for p in params:
                    p.copy_(flat[off:off + p.numel()].view_as(p))
                    off += p.numel()
        # one flat gradient bucket
        n = sum(p.numel() for p in params)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=self.device)
        off = 0
        for p in params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.graphs = _graphs_enabled(self.cfg, self.device)
        kw = {"lr": self.cfg["lr"]}
        if self.device.type == "cuda":
            kw["fused"] = True
            if self.graphs:
                kw["capturable"] = True
        try:
            self.opt = torch.optim.Adam(params, **kw)
        except (TypeError, RuntimeError, ValueError):
            kw.pop("fused", None)
            self.opt = torch.optim.Adam(params, **kw)
        self.kl_coeff = float(self.cfg["kl_coeff"])
        self.kl_coeff_t = torch.tensor(self.kl_coeff, device=self.device)
        self.acc = torch.zeros(5, device=self.device)
        self.stats: Dict[str, float] = {}
        self._graph = None
        self._static = None
        self._sidx = None
        self._mbs = None

    # ------------------------------------------------------------------ loss
    def _forward(self, obs):
        if self.cfg["bf16"] and self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, v = self.model(obs)
            return logits.float(), v.float()
        return self.model(obs)

    def loss(self, mb):
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
        total = total + self.kl_coeff_t * kl
        return total, means, kl

    # ------------------------------------------------------------------ one SGD step
    def _allreduce(self):
        torch.distributed.all_reduce(self.flat_grad, group=self.pg)
        self.flat_grad.mul_(1.0 / self.world)

    def _step_body(self, full, idx, with_sync: bool):
        self.flat_grad.zero_()
        mb = {k: ops.gather_rows(full[k], idx) for k in _LOSS_KEYS}
        total, means, kl = self.loss(mb)
        total.backward()
        if with_sync:
            if self.world > 1:
                self._allreduce()
            if self.cfg["grad_clip"]:
                nn.utils.clip_grad_norm_(self.params, self.cfg["grad_clip"])
            self.opt.step()
        self.acc += torch.cat([total.detach().reshape(1), means[:3].detach(), kl.detach().reshape(1)])

    def _eager_step(self, full, idx):
        self._step_body(full, idx, True)

    def _capture(self, full, mbs):
        in_graph_sync = self.world == 1 or self.cfg["allreduce_in_graph"]
        self._sidx = torch.arange(mbs, device=self.device, dtype=torch.int64)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        saved = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        saved_opt = None
        with torch.cuda.stream(s):
            for _ in range(3):  # warm up kernels / MIOpen find / allocator before capture
                self._step_body(full, self._sidx, in_graph_sync)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_body(full, self._sidx, in_graph_sync)
        # undo the warm-up/capture updates (capture does not execute, warm-up did)
        with torch.no_grad():
            self.model.load_state_dict(saved)
        for st in self.opt.state.values():
            for k, v in st.items():
                if torch.is_tensor(v):
                    v.zero_()
        self._graph = g
        self._graph_sync = in_graph_sync
        self._mbs = mbs

    # ------------------------------------------------------------------ update
    def update(self, batch: SampleBatch) -> Dict[str, float]:
        """num_sgd_iter epochs of shuffled minibatch SGD over a device-resident batch."""
        c = self.cfg
        if c["standardize_advantages"]:
            a = batch[SampleBatch.ADVANTAGES].float()
            batch[SampleBatch.ADVANTAGES] = (a - a.mean()) / a.std().clamp_min(1e-4)
        n = batch.count
        mbs = min(c["sgd_minibatch_size"], n)
        nmb = max(n // mbs, 1)
        use_graph = self.graphs
        if use_graph:
            if self._static is None or self._static[SampleBatch.OBS].shape != batch[SampleBatch.OBS].shape:
                self._static = {k: batch[k].detach().clone() for k in _LOSS_KEYS}
                self._graph = None
            else:
                for k in _LOSS_KEYS:
                    self._static[k].copy_(batch[k])
            if self._graph is None or self._mbs != mbs:
                try:
                    self._capture(self._static, mbs)
                except Exception as e:  # pragma: no cover - capture unsupported: stay eager
                    print(f"[PPOLearner] HIP graph capture failed ({e!r}); running eagerly")
                    self.graphs = use_graph = False
                    torch.cuda.synchronize(self.device)
        full = self._static if use_graph else {k: batch[k] for k in _LOSS_KEYS}
        self.acc.zero_()
        self.kl_coeff_t.fill_(self.kl_coeff)
        steps = 0
        for _ in range(c["num_sgd_iter"]):
            perm = torch.randperm(n, device=self.device)
            for i in range(nmb):
                idx = perm[i * mbs:(i + 1) * mbs]
                if use_graph:
                    self._sidx.copy_(idx)
                    self._graph.replay()
                    if not self._graph_sync:
                        if self.world > 1:
                            self._allreduce()
                        self.opt.step()
                else:
                    self._eager_step(full, idx)
                steps += 1
        acc = (self.acc / max(steps, 1)).tolist()  # one host sync per update
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
        with torch.no_grad():
            self.model.load_state_dict(w)


class GPURolloutSampler:
    """Samples `fragment` steps from a device-resident vectorised env with on-GPU inference and
    postprocesses with the GAE kernel. Output: a flat SampleBatch of fragment*num_envs rows in HBM.
    Each env step (policy forward, Gumbel-max sampling, env step, buffer writes at a device-side
    step counter) is one HIP-graph replay."""

    def __init__(self, env, model: nn.Module, fragment: int, gamma=0.99, lam=0.95, bf16=True, use_graphs=True):
        self.env = env
        self.model = model
        self.T = fragment
        self.B = env.num_envs
        self.gamma, self.lam, self.bf16 = gamma, lam, bf16
        dev = env.device
        self.device = dev
        obs = env.reset()
        T, B = self.T, self.B
        self.s_obs = obs.clone()
        self.buf_obs = torch.empty((T, B, *obs.shape[1:]), dtype=obs.dtype, device=dev)
        self.buf_act = torch.empty((T, B), dtype=torch.int64, device=dev)
        self.buf_logp = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_vf = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_rew = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.buf_done = torch.empty((T, B), dtype=torch.float32, device=dev)
        with torch.no_grad():
            logits, _ = self._policy(self.s_obs)
        self.buf_logits = torch.empty((T, B, logits.shape[-1]), dtype=torch.float32, device=dev)
        self.t_idx = torch.zeros(1, dtype=torch.int64, device=dev)
        self.graphs = use_graphs and dev.type == "cuda" and not os.environ.get("RMM_NO_GRAPHS")
        self._graph = None

    def _policy(self, obs):
        if self.bf16 and self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, v = self.model(obs)
            return logits.float(), v.float()
        return self.model(obs)

    @torch.no_grad()
    def _step_body(self):
        logits, v = self._policy(self.s_obs)
        d = Categorical(logits)
        a = d.sample()
        t = self.t_idx
        self.buf_obs.index_copy_(0, t, self.s_obs.unsqueeze(0))
        self.buf_act.index_copy_(0, t, a.unsqueeze(0))
        self.buf_logp.index_copy_(0, t, d.logp(a).unsqueeze(0))
        self.buf_vf.index_copy_(0, t, v.unsqueeze(0))
        self.buf_logits.index_copy_(0, t, logits.unsqueeze(0))
        obs, r, done = self.env.step(a)
        self.s_obs.copy_(obs)
        self.buf_rew.index_copy_(0, t, r.unsqueeze(0))
        self.buf_done.index_copy_(0, t, done.unsqueeze(0))
        self.t_idx.add_(1)

    def _capture(self):
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self.t_idx.zero_()
                self._step_body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_body()
        self._graph = g

    @torch.no_grad()
    def sample(self) -> SampleBatch:
        if self.graphs and self._graph is None:
            try:
                self._capture()
            except Exception as e:  # pragma: no cover
                print(f"[GPURolloutSampler] HIP graph capture failed ({e!r}); running eagerly")
                self.graphs = False
                torch.cuda.synchronize(self.device)
        self.t_idx.zero_()
        for _ in range(self.T):
            if self._graph is not None:
                self._graph.replay()
            else:
                self._step_body()
        _, last_v = self._policy(self.s_obs)
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
