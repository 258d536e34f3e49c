"""GPU PPO learner + on-device rollout sampler (the MI355X fast path of RLlib PPO).

Parity: reference rllib/algorithms/ppo/ppo_torch_policy.py (loss: clipped surrogate, clipped
value loss, entropy bonus, KL penalty with adaptive coefficient), rllib/algorithms/ppo/ppo.py
(training_step: sample → standardize advantages → num_sgd_iter × minibatch SGD → update KL),
rllib/execution/multi_gpu_learner_thread.py + train_ops.multi_gpu_train_one_step (multi-GPU
learner).

MI355X design (fast path, ``device.type == "cuda"``):
  * mixed precision with fp32 MASTER weights: the model holds bf16 compute weights (no autocast
    casts per forward); one flat fp32 master / Adam-moment buffer; the whole optimizer step is one
    launch of the K6 kernel, which also rewrites the bf16 weights in place;
  * gradients land in ONE flat bf16 bucket (one multi-segment copy launch, K1) so the data-parallel
    sync is a single RCCL all-reduce per minibatch step over xGMI — the Atari net is ~1M params;
  * minibatch gather + uint8→bf16 NHWC conversion in one launch (K2b), the remaining columns packed
    into one fp32 matrix and gathered in one launch (K2);
  * policy logits + value are ONE [N, A+1] Linear; the whole categorical PPO loss (log-softmax, logp,
    entropy, KL, ratio/clip, value clip, stats accumulated in place) forward and backward are one
    launch each (K5c), reading all per-sample columns from one packed fp32 matrix;
  * the update's minibatch index table is built once (one rand + one sort); the SGD-step graph
    reads its window through a device step counter that also drives Adam's bias correction, so
    replays need no host→device copies;
  * rollout: Gumbel-max sampling + buffer writes at a device-side step counter in one launch (K7);
  * every rollout step and every SGD step is one HIP-graph replay.
The CPU path (rollout workers without GPUs, tests) is plain fp32 PyTorch with the same math.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch
import torch.nn as nn

from ray_memory_management_amd import ops
from ray_memory_management_amd._native import require_hip
from ray_memory_management_amd.rllib.distributions import Categorical, dist_class_for
from ray_memory_management_amd.rllib.sample_batch import SampleBatch

DEFAULT_PPO = dict(
    gamma=0.99, lambda_=0.95, kl_coeff=0.5, kl_target=0.01, clip_param=0.1, vf_clip_param=10.0,
    vf_loss_coeff=1.0, entropy_coeff=0.01, lr=5e-5, train_batch_size=5000, sgd_minibatch_size=500,
    num_sgd_iter=10, grad_clip=None, standardize_advantages=True, use_graphs=True, fused=True,
    allreduce_in_graph=False, adam_betas=(0.9, 0.999), adam_eps=1e-8, weight_decay=0.0,
)

_LOSS_KEYS = (SampleBatch.OBS, SampleBatch.ACTIONS, SampleBatch.ACTION_LOGP, SampleBatch.ACTION_DIST_INPUTS,
              SampleBatch.ADVANTAGES, SampleBatch.VALUE_TARGETS)


def _stream():
    return torch.cuda.current_stream().cuda_stream


class _CatPPOLoss(torch.autograd.Function):
    """K5b: the categorical PPO loss head; forward = stats, backward = d/dlogits, d/dvalues."""

    @staticmethod
    def forward(ctx, logits, values, old_logits, actions, old_logp, adv, vtgt, coef):
        h = require_hip()
        N, A = logits.shape
        stats = torch.zeros(6, dtype=torch.float32, device=logits.device)
        h.ppo_cat_loss(True, logits.data_ptr(), logits.dtype == torch.bfloat16, old_logits.data_ptr(),
                       actions.data_ptr(), old_logp.data_ptr(), adv.data_ptr(), values.data_ptr(),
                       values.dtype == torch.bfloat16, vtgt.data_ptr(), coef.data_ptr(), stats.data_ptr(), 0, 0, 0,
                       N, A, _stream())
        ctx.save_for_backward(logits, values, old_logits, actions, old_logp, adv, vtgt, coef)
        total = stats[5] / N
        ctx.mark_non_differentiable(stats)
        return total, stats

    @staticmethod
    def backward(ctx, g_total, g_stats):
        h = require_hip()
        logits, values, old_logits, actions, old_logp, adv, vtgt, coef = ctx.saved_tensors
        N, A = logits.shape
        g_logits = torch.empty_like(logits)
        g_values = torch.empty_like(values)
        g = g_total.reshape(1).float().contiguous()
        h.ppo_cat_loss(False, logits.data_ptr(), logits.dtype == torch.bfloat16, old_logits.data_ptr(),
                       actions.data_ptr(), old_logp.data_ptr(), adv.data_ptr(), values.data_ptr(),
                       values.dtype == torch.bfloat16, vtgt.data_ptr(), coef.data_ptr(), 0, g.data_ptr(),
                       g_logits.data_ptr(), g_values.data_ptr(), N, A, _stream())
        return g_logits, g_values, None, None, None, None, None, None


class _HeadsPPOLoss(torch.autograd.Function):
    """K5c: PPO loss on the merged [N, A+1] head output with all per-sample columns packed in one
    fp32 matrix [N, A+4] (old logits, old logp, advantage, value target, action). The forward adds
    the 6 stat sums into `acc` in place and returns an (unwritten) scalar handle; the backward
    reads the upstream gradient from device memory, so the whole step is allocation/copy free."""

    @staticmethod
    def forward(ctx, heads, cols, coef, acc, gout):
        N, A1 = heads.shape
        ctx.g_heads = None
        if gout is not None:  # upstream gradient known now: stats AND d/dheads in one launch
            ctx.g_heads = torch.empty_like(heads)
            ctx.gout_ptr = gout.data_ptr()
            require_hip().ppo_heads_loss(True, heads.data_ptr(), cols.data_ptr(), coef.data_ptr(), acc.data_ptr(),
                                         gout.data_ptr(), ctx.g_heads.data_ptr(), N, A1 - 1, _stream())
        else:
            require_hip().ppo_heads_loss(False, heads.data_ptr(), cols.data_ptr(), coef.data_ptr(), acc.data_ptr(),
                                         0, 0, N, A1 - 1, _stream())
        ctx.save_for_backward(heads, cols, coef)
        return torch.empty((), dtype=torch.float32, device=heads.device)

    @staticmethod
    def backward(ctx, g):
        if ctx.g_heads is not None and g.data_ptr() == ctx.gout_ptr:
            return ctx.g_heads, None, None, None, None
        heads, cols, coef = ctx.saved_tensors
        N, A1 = heads.shape
        g_heads = torch.empty_like(heads)
        g = g.float().contiguous()
        require_hip().ppo_heads_loss(True, heads.data_ptr(), cols.data_ptr(), coef.data_ptr(), 0, g.data_ptr(),
                                     g_heads.data_ptr(), N, A1 - 1, _stream())
        return g_heads, None, None, None, None


def ppo_heads_loss(heads, cols, coef, acc, gout=None):
    """Fused PPO loss on a merged head output (see _HeadsPPOLoss). Differentiate the returned
    handle with grad_outputs=<device scalar 1.0>; the loss VALUE is only available through acc[5]/N.
    Passing that same device scalar as `gout` computes the gradient in the forward launch."""
    assert heads.dtype == torch.bfloat16 and heads.is_contiguous() and cols.dtype == torch.float32
    assert cols.shape == (heads.shape[0], heads.shape[1] + 3) and cols.is_contiguous()
    return _HeadsPPOLoss.apply(heads, cols, coef, acc, gout)


def ppo_categorical_loss(logits, values, old_logits, actions, old_logp, adv, vtgt, coef):
    """Fused categorical PPO loss. coef = device tensor [clip, vf_clip, vf_coeff, ent_coeff, kl_coeff].
    Returns (total, stats[6] = sums of -surr, vf, entropy, kl, clipped, total)."""
    return _CatPPOLoss.apply(logits.contiguous(), values.contiguous(), old_logits.contiguous(), actions.contiguous(),
                             old_logp.contiguous(), adv.contiguous(), vtgt.contiguous(), coef)


def ppo_categorical_loss_reference(logits, values, old_logits, actions, old_logp, adv, vtgt, coef):
    clip, vf_clip, vf_coeff, ent_coeff, kl_coeff = [float(x) for x in coef.tolist()]
    d, old = Categorical(logits.float()), Categorical(old_logits.float())
    logp = d.logp(actions)
    ent = d.entropy()
    kl = old.kl(d)
    ratio = torch.exp(logp - old_logp)
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
    vf = torch.clamp((values.float() - vtgt) ** 2, max=vf_clip)
    per = -surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl
    stats = torch.stack([(-surr).sum(), vf.sum(), ent.sum(), kl.sum(), ((ratio - 1).abs() > clip).float().sum(),
                         per.sum()]).detach()
    return per.mean(), stats


class PPOLearner:
    def __init__(self, model: nn.Module, config: Optional[dict] = None, device="cuda", process_group=None,
                 action_space=None):
        self.cfg = {**DEFAULT_PPO, **(config or {})}
        self.device = torch.device(device)
        self.dist_cls = dist_class_for(action_space) if action_space is not None else Categorical
        self.fast = (self.device.type == "cuda" and bool(self.cfg["fused"]) and self.dist_cls is Categorical)
        self.pg = process_group
        self.world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world = torch.distributed.get_world_size(process_group)
        model = model.to(self.device)
        if self.device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:  # identical initial weights: broadcast rank 0's
            with torch.no_grad():
                flat = torch.cat([p.detach().float().reshape(-1) for p in params])
                src = torch.distributed.get_global_rank(process_group, 0) if process_group is not None else 0
                torch.distributed.broadcast(flat, src=src, group=process_group)
                off = 0
                for p in params:
                    p.copy_(flat[off:off + p.numel()].view(p.shape))
                    off += p.numel()
        self.kl_coeff = float(self.cfg["kl_coeff"])
        self.stats: Dict[str, float] = {}
        self._graph = None
        self._static = None
        self._mbs = None
        if self.fast:
            self._init_fast(params)
        else:
            self.params = params
            self.opt = torch.optim.Adam(params, lr=self.cfg["lr"], betas=self.cfg["adam_betas"],
                                        eps=self.cfg["adam_eps"], weight_decay=self.cfg["weight_decay"])
        self.graphs = self.fast and bool(self.cfg["use_graphs"]) and not os.environ.get("RMM_NO_GRAPHS")

    # ------------------------------------------------------------------ fast-path state
    def _init_fast(self, params):
        dev = self.device
        n = sum(p.numel() for p in params)
        self.n_params = n
        # fp32 master + moments (flat), bf16 compute weights (flat; params become views into it)
        self.master = torch.empty(n, dtype=torch.float32, device=dev)
        self.w_bf16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
        off = 0
        self.params = []
        with torch.no_grad():
            for p in params:
                k = p.numel()
                # lay the master out in the param's MEMORY order so one flat kernel updates both
                self.master.as_strided(p.size(), p.stride(), off).copy_(p.detach().float())
                view = self.w_bf16.as_strided(p.size(), p.stride(), off)
                view.copy_(p.detach())
                p.data = view
                self.params.append(p)
                off += k
        self.m1 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m2 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        # each param's slice of the flat bucket: fused backward kernels (K10 trunk, K8b dense) write
        # their gradients there directly and the bucket copy skips them
        off = 0
        for p in self.params:
            p._rmm_grad_out = self.flat_grad.as_strided(p.size(), p.stride(), off)
            off += p.numel()
        b1, b2 = self.cfg["adam_betas"]
        self.hp = torch.tensor([self.cfg["lr"], b1, b2, self.cfg["adam_eps"], self.cfg["weight_decay"], 0.0],
                               dtype=torch.float32, device=dev)
        self.coef = torch.tensor([self.cfg["clip_param"], self.cfg["vf_clip_param"], self.cfg["vf_loss_coeff"],
                                  self.cfg["entropy_coeff"], self.kl_coeff], dtype=torch.float32, device=dev)
        self.acc = torch.zeros(6, device=dev)
        # device counters {minibatch step within the update, Adam step}: the SGD-step graph reads
        # its minibatch indices at idx_all[ctr[0]] and the Adam bias correction from ctr[1]; one
        # add per step advances both, so no host→device copy happens between graph replays.
        self.ctr = torch.zeros(2, dtype=torch.int64, device=dev)
        self._bump_done = torch.zeros(require_hip().bump_done_words(), dtype=torch.int32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.heads_ok = hasattr(self.model, "forward_heads")

    def _opt_step(self):
        h = require_hip()
        if self.world > 1:
            torch.distributed.all_reduce(self.flat_grad, group=self.pg)
        # K6 also advances both device counters {minibatch step, Adam step} from its last workgroup
        h.adam_flat(self.master.data_ptr(), self.m1.data_ptr(), self.m2.data_ptr(), self.flat_grad.data_ptr(), True,
                    self.w_bf16.data_ptr(), self.hp.data_ptr(), 1.0 / self.world, self.n_params, _stream(),
                    step_ctr=self.ctr.data_ptr() + 8, bump=self.ctr.data_ptr(), nbump=2,
                    done=self._bump_done.data_ptr())

    def _fast_step(self, full, with_opt: bool):
        h = require_hip()
        mbs, period = full["mbs"], full["period"]
        ctr = self.ctr
        # K2b: minibatch gather + u8→bf16 NHWC; K2: ONE gather for every per-sample column —
        # both index idx_all at the device step counter
        frames = full["obs"].dtype == torch.uint8 and full["obs"].dim() == 4
        fused = frames and self.heads_ok and getattr(self.model, "fused_trunk_ok", None) is not None \
            and self.model.fused_trunk_ok(full["obs"])
        if fused:  # K10: gather + both convs inside one MFMA kernel
            x = None
        elif frames:
            x = ops.frames_to_nhwc(full["obs"], full["idx"], rows=mbs, ctr=ctr, period=period)
        else:  # vector observations (e.g. CartPole): plain row gather
            x = ops.gather_rows(full["obs"], full["idx"], rows=mbs, ctr=ctr, period=period)
        cols = None if fused else ops.gather_rows(full["cols"], full["idx"], rows=mbs, ctr=ctr, period=period)
        if fused:  # K10 trunk → K13 → K15 (heads + PPO loss + dheads + dpre, cols gathered in place); bwd K12 → K10
            total, h = self.model.forward_frames_ppo(full["obs"], full["cols"], self.coef, self.acc, self._one,
                                                     idx=full["idx"], ctr=ctr, period=period, rows=mbs)
            if total is None:
                cols = ops.gather_rows(full["cols"], full["idx"], rows=mbs, ctr=ctr, period=period)
                from ray_memory_management_amd.rllib.models import dense_heads

                heads = dense_heads(h, self.model.dense_tail, self.model.heads)
                total = ppo_heads_loss(heads, cols, self.coef, self.acc, gout=self._one)  # K5c, fwd+bwd
            grads = list(torch.autograd.grad(total, self.params, grad_outputs=self._one))
        elif self.heads_ok and frames:
            heads = self.model.forward_heads(x, prescaled=True)
            total = ppo_heads_loss(heads, cols, self.coef, self.acc)     # K5c
            grads = list(torch.autograd.grad(total, self.params, grad_outputs=self._one))
        else:
            A = full["A"]
            logits, v = self.model(x, prescaled=True) if frames else self.model(x)
            total, stats = ppo_categorical_loss(logits, v, cols[:, :A], cols[:, A + 3].long(), cols[:, A],
                                                cols[:, A + 1], cols[:, A + 2], self.coef)
            grads = list(torch.autograd.grad(total, self.params))
            self.acc.add_(stats)
        for i, (g, p) in enumerate(zip(grads, self.params)):
            if g.stride() != p.stride() and g.numel() > 1:  # match the flat bucket's memory order
                grads[i] = torch.empty_strided(p.size(), p.stride(), dtype=g.dtype, device=g.device).copy_(g)
        segs = []
        off = 0
        for g, p in zip(grads, self.params):
            nb = g.numel() * 2
            dst = self.flat_grad.data_ptr() + off * 2
            if g.data_ptr() != dst:  # fused backward kernels already wrote into the bucket
                segs.append((g.data_ptr(), dst, nb))
            off += p.numel()
        if segs:
            h.multi_copy(segs, _stream())                    # K1: remaining grads → one flat bucket
        if with_opt:  # otherwise the caller runs _opt_step (all-reduce + Adam + counters) eagerly
            self._opt_step()

    def _pack(self, batch, mbs, nmb):
        """One fp32 column matrix [n, A+4] (old logits, old logp, adv, value target, action) and the
        whole update's minibatch index table [iters * nmb * mbs] (one rand + one sort launch)."""
        A = batch[SampleBatch.ACTION_DIST_INPUTS].shape[-1]
        n = batch.count
        cols = torch.cat([batch[SampleBatch.ACTION_DIST_INPUTS].float(),
                          batch[SampleBatch.ACTION_LOGP].float().unsqueeze(1),
                          batch[SampleBatch.ADVANTAGES].float().unsqueeze(1),
                          batch[SampleBatch.VALUE_TARGETS].float().unsqueeze(1),
                          batch[SampleBatch.ACTIONS].float().reshape(n, 1)], dim=1).contiguous()
        iters = self.cfg["num_sgd_iter"]
        idx = torch.rand(iters, n, device=self.device).argsort(dim=1)[:, :nmb * mbs].reshape(-1).contiguous()
        return {"obs": batch[SampleBatch.OBS].contiguous(), "cols": cols, "idx": idx, "A": A, "mbs": mbs,
                "period": iters * nmb}

    def _capture(self, full):
        in_graph_opt = self.world == 1 or self.cfg["allreduce_in_graph"]
        saved = (self.master.clone(), self.m1.clone(), self.m2.clone(), self.w_bf16.clone(), self.ctr.clone(),
                 self.acc.clone())
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):  # warm up (MIOpen find, allocator) before capture
                self._fast_step(full, in_graph_opt)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._fast_step(full, in_graph_opt)
        for dst, src in zip((self.master, self.m1, self.m2, self.w_bf16, self.ctr, self.acc), saved):
            dst.copy_(src)  # undo warm-up updates
        self._graph = g
        self._graph_opt = in_graph_opt

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
        if not self.fast:
            return self._update_eager(batch, mbs)
        packed = self._pack(batch, mbs, nmb)
        self.acc.zero_()
        self.coef[4].fill_(self.kl_coeff)
        if self.graphs:
            st = self._static
            if st is None or any(st[k].shape != packed[k].shape for k in ("obs", "cols", "idx")) \
                    or st["mbs"] != mbs:
                self._static = st = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in packed.items()}
                self._graph = None
            else:
                for k in ("obs", "cols", "idx"):
                    st[k].copy_(packed[k])
            if self._graph is None:
                try:
                    self._capture(st)
                except Exception as e:  # pragma: no cover - capture unsupported: stay eager
                    print(f"[PPOLearner] HIP graph capture failed ({e!r}); running eagerly")
                    self.graphs = False
                    torch.cuda.synchronize(self.device)
            full = st if self.graphs else packed
        else:
            full = packed
        self.ctr[0:1].zero_()
        steps = 0
        for _ in range(c["num_sgd_iter"] * nmb):
            if self.graphs:
                self._graph.replay()
                if not self._graph_opt:
                    self._opt_step()
            else:
                self._fast_step(full, True)
            steps += 1
        if self.world > 1:  # KL adaptation and stats from the global batch, identical on every rank
            torch.distributed.all_reduce(self.acc, group=self.pg)
            self.acc.mul_(1.0 / self.world)
        acc = (self.acc / float(max(steps, 1) * mbs)).tolist()  # one host sync per update
        return self._finish(acc[0], acc[1], acc[2], acc[3], acc[5], steps)

    def _finish(self, pol, vf, ent, kl_mean, total, steps):
        c = self.cfg
        # adaptive KL coefficient (reference ppo.py UpdateKL)
        if kl_mean > 2.0 * c["kl_target"]:
            self.kl_coeff *= 1.5
        elif kl_mean < 0.5 * c["kl_target"]:
            self.kl_coeff *= 0.5
        self.stats = {"total_loss": total, "policy_loss": pol, "vf_loss": vf, "entropy": ent, "kl": kl_mean,
                      "cur_kl_coeff": self.kl_coeff, "num_sgd_steps": steps}
        return self.stats

    def _update_eager(self, batch, mbs):
        c = self.cfg
        coef = torch.tensor([c["clip_param"], c["vf_clip_param"], c["vf_loss_coeff"], c["entropy_coeff"],
                             self.kl_coeff])
        acc = torch.zeros(6)
        steps = 0
        for _ in range(c["num_sgd_iter"]):
            for mb in batch.minibatches(mbs, shuffle=True):
                logits, v = self.model(mb[SampleBatch.OBS])
                total, stats = ppo_categorical_loss_reference(
                    logits, v, mb[SampleBatch.ACTION_DIST_INPUTS], mb[SampleBatch.ACTIONS],
                    mb[SampleBatch.ACTION_LOGP].float(), mb[SampleBatch.ADVANTAGES].float(),
                    mb[SampleBatch.VALUE_TARGETS].float(), coef)
                self.opt.zero_grad(set_to_none=True)
                total.backward()
                if self.world > 1:
                    for p in self.params:
                        torch.distributed.all_reduce(p.grad, group=self.pg)
                        p.grad.mul_(1.0 / self.world)
                if c["grad_clip"]:
                    nn.utils.clip_grad_norm_(self.params, c["grad_clip"])
                self.opt.step()
                acc += stats.cpu() / mb.count
                steps += 1
        if self.world > 1:
            acc_d = acc.to(self.device)
            torch.distributed.all_reduce(acc_d, group=self.pg)
            acc = acc_d.cpu() / self.world
        acc = (acc / max(steps, 1)).tolist()
        return self._finish(acc[0], acc[1], acc[2], acc[3], acc[5], steps)

    def get_weights(self):
        if self.fast:  # publish the fp32 masters (the bf16 weights are derived)
            out, off = {}, 0
            sd = self.model.state_dict()
            names = {id(p): n for n, p in self.model.named_parameters()}
            for p in self.params:
                out[names[id(p)]] = self.master.as_strided(p.size(), p.stride(), off).detach().cpu().clone()
                off += p.numel()
            for k, v in sd.items():
                out.setdefault(k, v.detach().cpu())
            return out
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        with torch.no_grad():
            if self.fast:
                names = {id(p): n for n, p in self.model.named_parameters()}
                off = 0
                for p in self.params:
                    src = w[names[id(p)]].to(self.device).float()
                    self.master.as_strided(p.size(), p.stride(), off).copy_(src)
                    p.copy_(src)
                    off += p.numel()
            else:
                self.model.load_state_dict(w)


class GPURolloutSampler:
    """Samples `fragment` steps from a device-resident vectorised env with on-GPU inference and
    postprocesses with the GAE kernel. Output: a flat SampleBatch of fragment*num_envs rows in HBM.
    Each env step (policy forward, K7 sampling + buffer writes, env step) is one HIP-graph replay."""

    def __init__(self, env, model: nn.Module, fragment: int, gamma=0.99, lam=0.95, use_graphs=True, seed=0):
        self.env = env
        self.model = model
        self.T = fragment
        self.B = env.num_envs
        self.gamma, self.lam = gamma, lam
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
        self.act_now = torch.zeros(B, dtype=torch.int64, device=dev)
        with torch.no_grad():
            logits, _ = self.model(self.s_obs)
        self.A = logits.shape[-1]
        self.buf_logits = torch.empty((T, B, self.A), dtype=torch.float32, device=dev)
        # device-side {rng counter, rollout row}; both advance by one per step (one add launch)
        self.ctr_t = torch.zeros(2, dtype=torch.int64, device=dev)
        self.ctr = self.ctr_t[0:1]
        self.t_idx = self.ctr_t[1:2]
        self.seed = int(seed) & 0xFFFFFFFF
        self.fast = dev.type == "cuda"
        self.fused_env = self.fast and hasattr(env, "fused_step")
        if self.fused_env:
            self.s_obs = env.frames  # the env's frame stack IS the observation buffer
        self.graphs = use_graphs and self.fast and not os.environ.get("RMM_NO_GRAPHS")
        self._graph = None

    @torch.no_grad()
    def _step_body(self):
        t = self.t_idx
        if self.fast and hasattr(self.model, "forward_sample") and getattr(
                getattr(self.model, "heads", None), "out_features", -1) == self.A + 1 and self.model.forward_sample(
                self.s_obs, t, self.ctr, self.seed, self.buf_act, self.buf_logp, self.buf_vf, self.buf_logits,
                self.act_now):  # K10 → K13 → K16: heads + sampling + row stores in one launch
            a = self.act_now
        elif self.fast:
            if hasattr(self.model, "forward_heads"):  # merged [B, A+1] head read in place (strided)
                hd = self.model.forward_heads(self.s_obs)
                lp, vp, ld = hd.data_ptr(), hd.data_ptr() + self.A * hd.element_size(), hd.stride(0)
                lbf = vbf = hd.dtype == torch.bfloat16
                lds = (ld, ld)
            else:
                logits, v = self.model(self.s_obs)
                logits, v = logits.contiguous(), v.contiguous()
                lp, vp, lbf, vbf, lds = (logits.data_ptr(), v.data_ptr(), logits.dtype == torch.bfloat16,
                                         v.dtype == torch.bfloat16, (self.A, 1))
            require_hip().sample_store(
                lp, lbf, vp, vbf, t.data_ptr(), self.ctr.data_ptr(), self.seed, self.buf_act.data_ptr(),
                self.buf_logp.data_ptr(), self.buf_vf.data_ptr(), self.buf_logits.data_ptr(),
                self.act_now.data_ptr(), self.B, self.A, _stream(), ldl=lds[0], ldv=lds[1])
            a = self.act_now
        else:
            logits, v = self.model(self.s_obs)
            d = Categorical(logits.float())
            a = d.sample()
            self.buf_act.index_copy_(0, t, a.unsqueeze(0))
            self.buf_logp.index_copy_(0, t, d.logp(a).unsqueeze(0))
            self.buf_vf.index_copy_(0, t, v.float().unsqueeze(0))
            self.buf_logits.index_copy_(0, t, logits.float().unsqueeze(0))
        if self.fused_env:  # K9: obs row write + frame-stack step + reward/done + counters in one launch
            self.env.fused_step(a, self.ctr_t, self.buf_obs, self.buf_rew, self.buf_done, self.seed, advance=True)
            return
        else:
            self.buf_obs.index_copy_(0, t, self.s_obs.unsqueeze(0))
            obs, r, done = self.env.step(a)
            self.s_obs.copy_(obs)
            self.buf_rew.index_copy_(0, t, r.unsqueeze(0))
            self.buf_done.index_copy_(0, t, done.unsqueeze(0))
        self.ctr_t.add_(1)

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
        _, last_v = self.model(self.s_obs)
        adv, ret = ops.gae(self.buf_rew, self.buf_vf, self.buf_done, last_v.float(), self.gamma, self.lam)
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
    """One tiny PPO iteration (K7 sampling → K3 GAE → K2/K2b gathers → K5b loss → K6 Adam)."""
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(0)
    env = GPUSyntheticAtariVectorEnv(8, device, num_actions=4)
    learner = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 32, "num_sgd_iter": 1}, device=device,
                         action_space=env.action_space)
    sampler = GPURolloutSampler(env, learner.model, fragment=8)
    batch = sampler.sample()
    stats = learner.update(batch)
    torch.cuda.synchronize()
    return stats
