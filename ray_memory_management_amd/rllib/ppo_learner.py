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
    lr_schedule=None, entropy_coeff_schedule=None, manual_step=True, compute_dtype="bf16",
)

_LOSS_KEYS = (SampleBatch.OBS, SampleBatch.ACTIONS, SampleBatch.ACTION_LOGP, SampleBatch.ACTION_DIST_INPUTS,
              SampleBatch.ADVANTAGES, SampleBatch.VALUE_TARGETS)


def _k13s() -> bool:
    """K13s split-K dense layer with the reduction in its consumer (K15 / K16); RMM_NO_K13S=1 keeps
    K13 (bf16 hidden written by the dense kernel itself), for A/B timing."""
    return os.environ.get("RMM_NO_K13S") is None


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _x3_available() -> bool:
    """The precision-matched learner's split-bf16 kernels (csrc/hip/x3_kernels.hip) are built in;
    RMM_NO_X3=1 sends compute_dtype fp32 back through autograd (MIOpen / hipBLASLt), for A/B only."""
    if os.environ.get("RMM_NO_X3"):
        return False
    try:
        return hasattr(require_hip(), "x3_trunk_fwd")
    except Exception:
        return False



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
    """Data-parallel PPO learner on one device (see module docstring). `comm` selects the
    process group that averages gradients: None → torch.distributed's default group when it is
    initialised (torchrun ranks), a util.collective group name (learner actors), or a Comm."""

    _graph_has_comm = False  # the SGD-step graph contains the gradient all-reduces

    def __init__(self, model: nn.Module, config: Optional[dict] = None, device="cuda", process_group=None,
                 action_space=None, comm=None):
        from ray_memory_management_amd.parallel.comm import as_comm
        from ray_memory_management_amd.rllib.utils.schedules import make_schedule

        self.cfg = {**DEFAULT_PPO, **(config or {})}
        self.device = torch.device(device)
        self.dist_cls = dist_class_for(action_space) if action_space is not None else Categorical
        self.recurrent = bool(getattr(model, "is_recurrent", False))
        self.fast = (self.device.type == "cuda" and bool(self.cfg["fused"]) and self.dist_cls is Categorical
                     and not self.recurrent)
        self.comm = as_comm(comm if comm is not None else process_group)
        self.world = self.comm.world
        model = model.to(self.device)
        if self.device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:  # identical initial weights: broadcast rank 0's (one flat collective)
            with torch.no_grad():
                flat = torch.cat([p.detach().float().reshape(-1) for p in params])
                self.comm.broadcast(flat, 0)
                off = 0
                for p in params:
                    p.copy_(flat[off:off + p.numel()].view(p.shape))
                    off += p.numel()
        self.kl_coeff = float(self.cfg["kl_coeff"])
        self.lr_sched = make_schedule(self.cfg.get("lr_schedule"), self.cfg["lr"])
        self.ent_sched = make_schedule(self.cfg.get("entropy_coeff_schedule"), self.cfg["entropy_coeff"])
        self.timesteps = 0  # global env steps trained (drives the schedules)
        self.stats: Dict[str, float] = {}
        self._graph = None
        self._graphs_split = None
        self._static = None
        self._mbs = None
        self._ingest = None
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
        params = self._bucket_order(params)
        n = sum(p.numel() for p in params)
        self.n_params = n
        # fp32 master + moments (flat), bf16 compute weights (flat; params become views into it)
        # compute_dtype "fp32" (precision-matched with the reference's fp32 PPO): the parameters ARE
        # views of the fp32 master, gradients land in an fp32 bucket, K6 updates the master only
        self.fp32 = str(self.cfg.get("compute_dtype", "bf16")) in ("fp32", "float32")
        self.cdt = torch.float32 if self.fp32 else torch.bfloat16
        self.grad_bf16 = not self.fp32
        self.master = torch.empty(n, dtype=torch.float32, device=dev)
        self.w_bf16 = None if self.fp32 else torch.empty(n, dtype=torch.bfloat16, device=dev)
        off = 0
        self.params = []
        with torch.no_grad():
            for p in params:
                k = p.numel()
                # lay the master out in the param's MEMORY order so one flat kernel updates both
                self.master.as_strided(p.size(), p.stride(), off).copy_(p.detach().float())
                view = (self.master if self.fp32 else self.w_bf16).as_strided(p.size(), p.stride(), off)
                if not self.fp32:
                    view.copy_(p.detach())
                p.data = view
                self.params.append(p)
                off += k
        # fp32 learner on the hand-written kernels: the optimizer keeps a split-bf16 pair (hi + lo) of the
        # fp32 master next to it (K6 writes both planes), which the x3 kernels read (csrc/hip/x3_device.h)
        self.x3 = self.fp32 and _x3_available()
        self.w_x3 = None
        if self.x3:
            from ray_memory_management_amd.ops import x3 as X3

            self.w_x3 = X3.split(self.master)
            self._attach_x3()
        self.m1 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m2 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=self.cdt, device=dev)
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
        # Two copies (parity pair): inside a chained SGD graph step k reads copy k % 2 and its K6 writes
        # the advanced counters into the other copy from one lane (no last-workgroup ticket on the
        # critical path, 1.4 us per step on MI355X, profiles/adam_unroll_r3.txt); the chain's last
        # step leaves them in copy 0 (`self.ctr`), which everything outside the chain uses.
        self._ctrs = torch.zeros(2, 2, dtype=torch.int64, device=dev)
        self.ctr = self._ctrs[0]
        self._par = 0            # copy the next launched step reads
        self._parity = False     # set while capturing a chained graph
        self._parity_last = False
        self._bump_done = torch.zeros(require_hip().bump_done_words(), dtype=torch.int32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.heads_ok = hasattr(self.model, "forward_heads") and not self.fp32  # K5c reads bf16 heads
        # global-norm gradient clipping on the device (K6b → K6 scale pointer), graph-capturable
        self.clip_ws = self.clip_out = None
        if self.cfg["grad_clip"]:
            self.clip_ws = torch.zeros(require_hip().grad_clip_workspace_floats(), dtype=torch.float32, device=dev)
            self.clip_out = torch.ones(2, dtype=torch.float32, device=dev)
        self._manual = self._manual_layout()
        #: flat ranges whose Adam ran ZeRO-1 style (moments current on their owner rank only)
        self._zero1_ranges = set()

    def _wptr(self) -> int:
        """K6's bf16 weight output: the bf16 compute weights, the hi plane of the fp32 learner's split
        pair, or 0 (fp32 learner without the x3 kernels: its parameters are the master)."""
        if self.w_bf16 is not None:
            return self.w_bf16.data_ptr()
        return self.w_x3.hi.data_ptr() if self.w_x3 is not None else 0

    def _wlo(self) -> int:
        """K6's lo-plane output (the split pair's residual), 0 unless the fp32 learner runs the x3 kernels."""
        return self.w_x3.lo.data_ptr() if self.w_x3 is not None else 0

    def _x3_views(self):
        """{parameter name: Pair view} of the flat split pair, in each parameter's memory layout."""
        names = {id(p): n for n, p in self.model.named_parameters()}
        out, off = {}, 0
        for p in self.params:
            out[names[id(p)]] = self.w_x3.as_strided(p.size(), p.stride(), off)
            off += p.numel()
        return out

    def _attach_x3(self):
        """Point the model's fused fp32 path (rollout sampling with the learner's own model) at the pair."""
        if hasattr(self.model, "attach_x3") and getattr(self.model, "nature", False):
            try:
                self.model.attach_x3(self._x3_views())
            except ValueError:
                pass

    def rebind_master(self, flat: torch.Tensor) -> None:
        """Move the fp32 master (the fp32 learner's parameters are views of it) to `flat`, same layout,
        e.g. an HBM object co-located rollout workers alias; K6 keeps updating it in place."""
        if not self.fast or flat.dtype != torch.float32 or flat.numel() != self.n_params \
                or flat.device != self.master.device:
            raise ValueError("rebind_master: flat fp32 buffer of the learner's size on its device expected")
        torch.cuda.synchronize(self.device)
        with torch.no_grad():
            flat.copy_(self.master)
            if self.fp32:
                off = 0
                for p in self.params:
                    p.data = flat.as_strided(p.size(), p.stride(), off)
                    off += p.numel()
        self.master = flat
        self._graph = self._graphs_split = None

    def rebind_x3(self, hi: torch.Tensor, lo: torch.Tensor) -> None:
        """Move the fp32 learner's split pair to (hi, lo) (e.g. HBM objects that co-located rollout
        workers map zero-copy), same layout; captured graphs are dropped (recaptured next update)."""
        from ray_memory_management_amd.ops import x3 as X3

        if self.w_x3 is None:
            raise RuntimeError("rebind_x3 needs the fp32 learner on the x3 kernels")
        for t in (hi, lo):
            if t.dtype != torch.bfloat16 or t.numel() != self.n_params or t.device != self.w_x3.hi.device:
                raise ValueError("rebind_x3: flat bf16 planes of the learner's size on its device expected")
        torch.cuda.synchronize(self.device)
        hi.copy_(self.w_x3.hi)
        lo.copy_(self.w_x3.lo)
        self.w_x3 = X3.Pair(hi, lo)
        self._attach_x3()
        self._graph = self._graphs_split = None

    def _bucket_order(self, params):
        """Flat-bucket order: for the Nature-CNN layout the trunk (conv) parameters first, then
        dense + heads, so the gradient that K12 produces before the trunk backward is ONE contiguous
        tail slice of the bucket (all-reduced while K10 backward runs)."""
        from ray_memory_management_amd.rllib.models import VisionNetwork

        m = self.model
        if isinstance(m, VisionNetwork) and m.nature and m.dense_tail is not None:
            c1, c2 = m.convs[0], m.convs[1]
            order = [c1.weight, c1.bias, c2.weight, c2.bias, m.dense_tail.weight, m.dense_tail.bias,
                     m.heads.weight, m.heads.bias]
            if len(order) == len(params) and {id(p) for p in order} == {id(p) for p in params}:
                return order
        return list(params)

    def _manual_layout(self):
        """The flagship Nature-CNN model runs its SGD step as explicit kernel launches (no autograd):
        K10 fwd → K13 → K15 → K12 → K10 bwd, which lets a multi-rank step all-reduce the dense+heads
        bucket (≈99% of the gradient, ready after K12) WHILE the trunk backward runs. Returns the
        trunk/dense split of the flat bucket, or None when the model does not have that layout."""
        from ray_memory_management_amd.rllib.models import VisionNetwork

        m = self.model
        if self.fp32 and not self.x3:  # fp32 without the split-bf16 kernels: autograd (RMM_NO_X3)
            return None
        if not (self.cfg.get("manual_step", True) and isinstance(m, VisionNetwork) and m.nature
                and m.dense_tail is not None and not os.environ.get("RMM_NO_MANUAL_STEP")):
            return None
        c1, c2 = m.convs[0], m.convs[1]
        order = [c1.weight, c1.bias, c2.weight, c2.bias, m.dense_tail.weight, m.dense_tail.bias, m.heads.weight,
                 m.heads.bias]
        if len(order) != len(self.params) or any(a is not b for a, b in zip(order, self.params)):
            return None
        if not (m.dense_tail.out_features == 256 and m.dense_tail.in_features % 32 == 0
                and 3 <= m.heads.out_features <= 16 and m.dense_tail.weight.is_contiguous()
                and m.heads.weight.is_contiguous()):
            return None
        return sum(p.numel() for p in order[:4])

    def _manual_ok(self, full) -> bool:
        if self.x3:
            return self._manual is not None and self.model.fused_x3_ok(full["obs"])
        return (self._manual is not None and full["obs"].dtype == torch.uint8 and full["mbs"] <= 640
                and self.model.fused_trunk_ok(full["obs"]) and not os.environ.get("RMM_NO_K12")
                and not os.environ.get("RMM_NO_K15"))

    def _manual_ws(self, mbs):
        ws = getattr(self, "_mws", None)
        if ws is not None and ws["mbs"] == mbs:
            return ws
        if self.x3:
            return self._manual_ws_x3(mbs)
        dev, bf = self.device, torch.bfloat16
        A1 = self.model.heads.out_features
        K = self.model.dense_tail.in_features
        ws = {"mbs": mbs, "h1": torch.empty((mbs, 441, 16), dtype=bf, device=dev),
              "h2": torch.empty((mbs, K), dtype=bf, device=dev), "hidden": torch.empty((mbs, 256), dtype=bf, device=dev),
              "dz": torch.empty((mbs, A1), dtype=bf, device=dev), "dpre": torch.empty((mbs, 256), dtype=bf, device=dev),
              "dx": torch.empty((mbs, K), dtype=bf, device=dev),
              "part": torch.empty(require_hip().nature_trunk_partial_floats(mbs), dtype=torch.float32, device=dev)}
        if _k13s():  # K13s: split-K dense layer, K15 sums its fp32 partials (and writes `hidden` for K12)
            ws["S"] = require_hip().dense_fwd_part_slices(mbs, K, 256)
            ws["hpart"] = torch.empty(ws["S"] * mbs * 256, dtype=torch.float32, device=dev)
        self._mws = ws
        return ws

    def _manual_ws_x3(self, mbs):
        """Split-pair activations of the fp32 SGD step (K10x → K13x → K15x → K12x → K10x bwd)."""
        from ray_memory_management_amd.ops import x3 as X3

        dev = self.device
        A1 = self.model.heads.out_features
        K = self.model.dense_tail.in_features
        S = X3.dense_part_slices(mbs, K, 256)
        ws = {"mbs": mbs, "h1": X3.Pair.empty((mbs, 441, 16), dev), "h2": X3.Pair.empty((mbs, K), dev),
              "hid": X3.Pair.empty((mbs, 256), dev), "dz": X3.Pair.empty((mbs, A1), dev),
              "dpre": X3.Pair.empty((mbs, 256), dev), "dx": X3.Pair.empty((mbs, K), dev),
              "dpre1": X3.Pair.empty((mbs, 441, 16), dev), "S": S,
              "hpart": torch.empty(S * mbs * 256, dtype=torch.float32, device=dev),
              "part": torch.empty(X3.trunk_partial_floats(mbs), dtype=torch.float32, device=dev),
              # the minibatch's loss columns, gathered by K10x so K15x reads them without the index chain
              "colsg": torch.empty((mbs, A1 + 3), dtype=torch.float32, device=dev),
              # K15x's loss statistics, one row of running sums per workgroup (no same-word atomics), folded
              # into `acc` once per update (_fold_k15_stats)
              "k15s": torch.zeros((require_hip().x3_heads_ppo_groups(mbs), 8), dtype=torch.float32, device=dev)}
        if self._manual is not None:  # K12x second row part's dense + heads gradients (see _x3_rows)
            ws["grad2"] = torch.empty(self.n_params - self._manual, dtype=torch.float32, device=dev)
        self._mws = ws
        return ws

    def _zero_k15_stats(self):
        ws = getattr(self, "_mws", None)
        if ws is not None and "k15s" in ws:
            ws["k15s"].zero_()

    def _fold_k15_stats(self):
        """Add K15x's per-workgroup loss-statistics rows into `acc` (a fixed-order sum: deterministic, unlike
        the same-word atomics it replaces) and clear them."""
        ws = getattr(self, "_mws", None)
        if ws is not None and "k15s" in ws:
            self.acc.add_(ws["k15s"][:, :6].sum(0))
            ws["k15s"].zero_()

    def _x3_rows(self, mbs) -> int:
        """K12x row parts: 2 when the tail Adam consumes the dense + heads gradients (world of one, no clip)
        and the minibatch has >= 4 chunks of 64 rows. Each column / head workgroup then streams half of
        dpre (its bound); the second part's gradients go to a side slab that the tail Adam adds, so no
        merge runs inside K12x. RMM_X3_K12_ROWS=1: one part."""
        if not self._tail_adam() or (mbs + 63) // 64 < 4 or os.environ.get("RMM_X3_K12_ROWS", "2") == "1":
            return 1
        return 2

    def _x3_fwd_dense_bwd(self, full):
        """fp32 step, first half: K10x fwd → K13x → K15x (loss stats, dheads, dpre) → K12x (dense + heads
        gradients, fp32, into the bucket; dx for the trunk backward)."""
        h = require_hip()
        m = self.model
        P = self._x3_views_cached()
        mbs, period, idx, ctr = full["mbs"], full["period"], full["idx"], self._ctr()
        ws = self._manual_ws(mbs)
        st = _stream()
        K, A1 = m.dense_tail.in_features, m.heads.out_features
        w1, b1, w2, b2 = (P[n] for n in m._X3_NAMES[:4])
        wd, bd, wh, bh = (P[n] for n in m._X3_NAMES[4:])
        cols, colsg = full["cols"], ws["colsg"]
        gather = cols.dtype == torch.float32 and cols.is_contiguous() and cols.shape[1] == colsg.shape[1] \
            and not os.environ.get("RMM_NO_COLS_GATHER")
        h.x3_trunk_fwd(full["obs"].data_ptr(), idx.data_ptr(), ctr.data_ptr(), int(period), int(mbs), w1.ptrs(),
                       list(w1.hi.stride()), b1.ptrs(), w2.ptrs(), list(w2.hi.stride()), b2.ptrs(), ws["h1"].ptrs(),
                       ws["h2"].ptrs(), st, cols=cols.data_ptr() if gather else 0,
                       cols_out=colsg.data_ptr() if gather else 0, ncols=colsg.shape[1] if gather else 0)
        h.x3_dense_fwd_part(ws["h2"].ptrs(), wd.ptrs(), mbs, K, 256, ws["hpart"].data_ptr(), ws["S"], st)
        h.x3_heads_ppo(ws["hpart"].data_ptr(), ws["S"], bd.ptrs(), wh.ptrs(), bh.ptrs(),
                       (colsg if gather else cols).data_ptr(), self.coef.data_ptr(), ws["k15s"].data_ptr(),
                       self._one.data_ptr(), mbs, A1, ws["dz"].ptrs(), ws["dpre"].ptrs(), ws["hid"].ptrs(), st,
                       cidx=0 if gather else idx.data_ptr(), ctr=0 if gather else ctr.data_ptr(), period=int(period),
                       acc_slab=True)
        g = [p._rmm_grad_out for p in self.params]
        rs = self._x3_rows(mbs)
        side = {}
        if rs == 2:  # the second row part's outputs at the same offsets of the side slab
            base, s2 = self.flat_grad.data_ptr() + 4 * self._manual, ws["grad2"].data_ptr()
            side = dict(dw2=s2 + g[4].data_ptr() - base, db2=s2 + g[5].data_ptr() - base,
                        dwh2=s2 + g[6].data_ptr() - base, dbh2=s2 + g[7].data_ptr() - base)
        self._x3_grad2 = ws["grad2"].data_ptr() if rs == 2 else 0
        h.x3_dense_heads_bwd(ws["dz"].ptrs(), A1, ws["hid"].ptrs(), ws["h2"].ptrs(), wd.ptrs(), ws["dpre"].ptrs(), mbs,
                             K, ws["dx"].ptrs(), g[4].data_ptr(), g[5].data_ptr(), g[6].data_ptr(), g[7].data_ptr(), st,
                             rs=rs, **side)

    def _x3_trunk_bwd(self, full):
        """fp32 step, second half: K10x conv2 backward → conv1 weight gradient → reduce (fp32 trunk grads)."""
        h = require_hip()
        m = self.model
        P = self._x3_views_cached()
        ws = self._manual_ws(full["mbs"])
        g = [p._rmm_grad_out for p in self.params]
        w2 = P[m._X3_NAMES[2]]
        ctr = self._ctr().data_ptr()  # this step's counter copy (the tail args advance the parity)
        adam = self._x3_tail_args() if self._tail_adam() else []
        # the dense + heads Adam is final after K12x: fork it onto a side stream beside the trunk backward
        # (parity counters only: the reduce launch advances them into the other copy, never under its reads)
        fork = bool(adam) and adam[13] != 0 and os.environ.get("RMM_X3_DENSE_ADAM_FORK", "0") == "1"
        if fork:
            cur = torch.cuda.current_stream(self.device)
            side = getattr(self, "_adam_stream", None)
            if side is None:
                side = self._adam_stream = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            h.x3_dense_adam(adam, 1.0 / self.world, side.cuda_stream)
        h.x3_trunk_bwd(full["obs"].data_ptr(), full["idx"].data_ptr(), ctr, int(full["period"]),
                       int(full["mbs"]), w2.ptrs(), list(w2.hi.stride()), ws["h1"].ptrs(), ws["h2"].hi.data_ptr(),
                       ws["dx"].ptrs(), ws["dpre1"].ptrs(), ws["part"].data_ptr(), g[0].data_ptr(),
                       list(m.convs[0].weight.stride()), g[1].data_ptr(), g[2].data_ptr(), g[3].data_ptr(), _stream(),
                       adam=adam, grad_scale=1.0 / self.world, dense_separate=fork)
        if fork:
            cur.wait_stream(side)

    def _x3_tail_args(self):
        """Tail Adam of the fp32 learner (world of one): K6 folded into the x3 trunk-reduce launch — the
        reduce workgroups update each trunk parameter as its gradient becomes final, extra workgroups run
        K6's pass over the dense + heads range; both write the fp32 master, the moments and the split
        pair (hi / lo planes), and the launch advances the step counters (same rules as K6)."""
        cur = self._ctr().data_ptr()
        parity = self._parity and not (self._parity_last and self._par == 0)
        nxt = self._ctrs[1 - self._par].data_ptr() if parity else 0
        if parity:
            self._par ^= 1
        return [self.master.data_ptr(), self.m1.data_ptr(), self.m2.data_ptr(), self.flat_grad.data_ptr(),
                self.w_x3.hi.data_ptr(), self.w_x3.lo.data_ptr(), self._manual, self.n_params, self.hp.data_ptr(),
                cur + 8, cur, 2, 0 if parity else self._bump_done.data_ptr(), nxt, getattr(self, "_x3_grad2", 0)]

    def _x3_views_cached(self):
        key = (self.w_x3.hi.data_ptr(), self.w_x3.lo.data_ptr())
        c = getattr(self, "_x3v", None)
        if c is None or c[0] != key:
            c = self._x3v = (key, self._x3_views())
        return c[1]

    def _manual_fwd_dense_bwd(self, full):
        """K10 fwd → K13 → K15 (loss stats + dheads + dpre) → K12: dense+heads grads into the bucket."""
        if self.x3:
            return self._x3_fwd_dense_bwd(full)
        h = require_hip()
        m = self.model
        c1, c2, dl, hd = m.convs[0], m.convs[1], m.dense_tail, m.heads
        mbs, period, idx, ctr = full["mbs"], full["period"], full["idx"], self._ctr()
        ws = self._manual_ws(mbs)
        st = _stream()
        K, A1 = dl.in_features, hd.out_features
        h.nature_trunk_fwd(full["obs"].data_ptr(), idx.data_ptr(), ctr.data_ptr(), int(period), int(mbs),
                           c1.weight.data_ptr(), list(c1.weight.stride()), c1.bias.data_ptr(), c2.weight.data_ptr(),
                           list(c2.weight.stride()), c2.bias.data_ptr(), ws["h1"].data_ptr(), ws["h2"].data_ptr(), st)
        if "hpart" in ws:
            h.dense_fwd_part(ws["h2"].data_ptr(), dl.weight.data_ptr(), mbs, K, 256, ws["hpart"].data_ptr(), ws["S"],
                             st)
            part = dict(hpart=ws["hpart"].data_ptr(), S=ws["S"], hb=dl.bias.data_ptr(), hid_out=ws["hidden"].data_ptr())
        else:
            h.dense_relu_fwd(ws["h2"].data_ptr(), dl.weight.data_ptr(), dl.bias.data_ptr(), mbs, K, 256,
                             ws["hidden"].data_ptr(), st)
            part = {}
        h.dense_heads_ppo(ws["hidden"].data_ptr(), hd.weight.data_ptr(), hd.bias.data_ptr(), full["cols"].data_ptr(),
                          self.coef.data_ptr(), self.acc.data_ptr(), self._one.data_ptr(), mbs, A1,
                          ws["dz"].data_ptr(), ws["dpre"].data_ptr(), st, cidx=idx.data_ptr(), ctr=ctr.data_ptr(),
                          period=int(period), **part)
        g = [p._rmm_grad_out for p in self.params]
        h.dense_heads_bwd(ws["dz"].data_ptr(), A1, hd.weight.data_ptr(), ws["hidden"].data_ptr(), ws["h2"].data_ptr(),
                          dl.weight.data_ptr(), mbs, K, ws["dx"].data_ptr(), g[4].data_ptr(), g[5].data_ptr(),
                          g[6].data_ptr(), g[7].data_ptr(), ws["dpre"].data_ptr(), st, dpre_ready=True,
                          defer_finalize=self._split_fin(),
                          split=self._k12_split(mbs))

    def _manual_trunk_bwd(self, full):
        """K10 backward: trunk grads (conv1/conv2 weights + biases) into the bucket."""
        if self.x3:
            return self._x3_trunk_bwd(full)
        h = require_hip()
        c1, c2 = self.model.convs[0], self.model.convs[1]
        ws = self._manual_ws(full["mbs"])
        g = [p._rmm_grad_out for p in self.params]
        ctr = self._ctr().data_ptr()
        adam, tail = self._tail_adam_args() if self._tail_adam() else ([], [])
        fin = []
        if self._split_fin():  # the deferred K12 finalize (+ Adam) runs in the trunk-reduce launch
            part, rs, groups = self._split_plan(int(full["mbs"]))
            K = self.model.dense_tail.in_features
            # the head group (db, dWh, dbh) through split_finalize_elem; the dense weight through the
            # split-reading Adam tail (see _tail_adam_args)
            fin = [part, rs, groups, K, self.model.heads.out_features,
                   g[4].data_ptr(), g[5].data_ptr(), g[6].data_ptr(), g[7].data_ptr(), K // 32]
        h.nature_trunk_bwd(full["obs"].data_ptr(), full["idx"].data_ptr(), ctr, int(full["period"]),
                           int(full["mbs"]), c2.weight.data_ptr(), list(c2.weight.stride()), ws["h1"].data_ptr(),
                           ws["h2"].data_ptr(), ws["dx"].data_ptr(), ws["part"].data_ptr(), g[0].data_ptr(),
                           list(c1.weight.stride()), g[1].data_ptr(), g[2].data_ptr(), g[3].data_ptr(), _stream(),
                           adam=adam, tail=tail, tail_scale=1.0 / self.world, fin=fin)

    def _split_plan(self, mbs: int):
        """(workspace pointer, rs, groups) of the K12 row split at this minibatch size."""
        return require_hip().dense_split_plan(int(mbs), self.model.dense_tail.in_features, self._k12_split(mbs),
                                              _stream())

    def _k12_split(self, mbs: int) -> int:
        """K12 row-split factor (RMM_K12_SPLIT, read per call so K12 and a deferred finalize agree),
        capped by the minibatch's 64-row chunks. Default 2 under tail Adam (the finalize folds into the
        trunk-reduce launch: K12 15.5 -> 10.9 µs, reduce 9.3 -> 10.4 µs, fused loop 10.76 -> 10.38
        ms/iter, profiles/tail_adam_r4.txt), else 1 (a separate finalize kernel measured no gain)."""
        default = "2" if self._tail_adam() else "1"
        return max(1, min(int(os.environ.get("RMM_K12_SPLIT", default)), (int(mbs) + 63) // 64))

    def _split_fin(self) -> bool:
        """K12 row split (RMM_K12_SPLIT=2: twice the workgroups, half the serial row-chunk chain each)
        with its finalize deferred into the trunk-reduce launch, where each finalized dense / heads
        gradient element goes straight through FusedAdam: no finalize kernel boundary, and the
        bf16-rounded sums equal the finalize kernel's, so the update is bit-identical to split K12 →
        finalize → K6. Needs tail Adam (world of one, no clip)."""
        mbs = getattr(self, "_mws", {}).get("mbs", 0) if isinstance(getattr(self, "_mws", None), dict) else 0
        return self._tail_adam() and self._k12_split(mbs or 640) > 1

    def _tail_adam(self) -> bool:
        """World of one without a global-norm clip: K6 folds into the K10 trunk-reduce LAUNCH — the
        reduce's epilogue applies Adam to the trunk parameters (FusedAdam) while extra workgroups of
        the same launch run K6's pass over the dense + heads range (adam_device.h: the same code as
        K6, so the update is bit-identical). The SGD step loses the K6 launch and the two
        latency-bound passes (trunk partial sums, 28 MB of Adam traffic) overlap: fused loop 10.88 /
        11.04 -> 10.62 / 10.67 ms per iteration on MI355X (profiles/tail_adam_r4.txt). RMM_TAIL_ADAM=0
        restores the separate K6."""
        return (self._manual is not None and self.world == 1 and self.clip_out is None and self._manual % 4 == 0
                and os.environ.get("RMM_TAIL_ADAM", "1") != "0")

    def _tail_adam_args(self):
        """(FusedAdam fields for the trunk range, AdamTail fields for the dense + heads range). In a
        chained graph with parity counters the launch writes the advanced counters into the other
        copy from one lane (as K6 does); otherwise the reduce's last workgroup bumps them in place."""
        cur = self._ctr().data_ptr()
        parity = self._parity and not (self._parity_last and self._par == 0)
        lo = self._manual
        f4, b2 = 4 * lo, 2 * lo
        adam = [self.flat_grad.data_ptr(), self.master.data_ptr(), self.m1.data_ptr(), self.m2.data_ptr(),
                self._wptr(), self.hp.data_ptr(), cur + 8, 0 if parity else cur, 0 if parity else 2,
                0 if parity else self._bump_done.data_ptr()]
        nxt = self._ctrs[1 - self._par].data_ptr() if parity else 0
        if self._split_fin():  # dense weight: Adam on the summed row-split partials (vector pass)
            part, rs, _ = self._split_plan(self._mws["mbs"])
            K = self.model.dense_tail.in_features
            tail = [self.master.data_ptr() + f4, self.m1.data_ptr() + f4, self.m2.data_ptr() + f4,
                    self.flat_grad.data_ptr() + b2, self._wptr() + b2, 256 * K, self.hp.data_ptr(),
                    cur + 8, cur, 2, nxt, part, rs, K]
        else:
            tail = [self.master.data_ptr() + f4, self.m1.data_ptr() + f4, self.m2.data_ptr() + f4,
                    self.flat_grad.data_ptr() + b2, self._wptr() + b2, self.n_params - lo, self.hp.data_ptr(),
                    cur + 8, cur, 2, nxt]
        if parity:
            self._par ^= 1
        return adam, tail

    def _opt_launch(self):
        """[K6b global-norm clip coefficient →] K6 Adam; K6 also advances both device counters
        {minibatch step, Adam step} from its last workgroup. Graph-capturable."""
        h = require_hip()
        if self._zero1_ranges:
            self._zero1_sync()
        scale_ptr = 0
        if self.clip_out is not None:
            h.grad_clip_coef(self.flat_grad.data_ptr(), self.grad_bf16, self.n_params, 1.0 / self.world,
                             float(self.cfg["grad_clip"]), self.clip_ws.data_ptr(), self.clip_out.data_ptr(),
                             _stream())
            scale_ptr = self.clip_out.data_ptr()
        cur = self._ctr()
        args = (self.master.data_ptr(), self.m1.data_ptr(), self.m2.data_ptr(), self.flat_grad.data_ptr(),
                self.grad_bf16, self._wptr(), self.hp.data_ptr(), 1.0 / self.world, self.n_params, _stream())
        if self._parity and not (self._parity_last and self._par == 0):
            # chained graph: advance into the other copy from one lane (see __init__)
            h.adam_flat(*args, step_ctr=cur.data_ptr() + 8, bump=cur.data_ptr(), nbump=2, scale_ptr=scale_ptr,
                        bump_next=self._ctrs[1 - self._par].data_ptr(), wlo=self._wlo())
            self._par ^= 1
        else:  # in place: the last workgroup advances the counters after every workgroup read them
            h.adam_flat(*args, step_ctr=cur.data_ptr() + 8, bump=cur.data_ptr(), nbump=2,
                        done=self._bump_done.data_ptr(), scale_ptr=scale_ptr, wlo=self._wlo())

    def _peer_in_graph(self) -> bool:
        """The communicator's collectives are plain kernels with no host step (PeerComm): they can
        sit inside a chained multi-step SGD graph."""
        return self.world > 1 and bool(getattr(self.comm, "in_graph", False)) \
            and os.environ.get("RMM_PEER_IN_GRAPH", "1") != "0"

    def _peer_mode(self) -> str:
        """How a peer-comm SGD step reduces its bucket (RMM_PEER_MODE overrides):
        ``fork`` (default when every rank has its own GPU): the dense+heads bucket (≈99% of the bytes,
        final after K12) is all-reduced on the comm stream WHILE the trunk backward runs on the compute
        stream; then the small trunk bucket; Adam after both;
        ``one`` (default when ranks share a GPU, where the overlap only contends for the same CUs):
        one all-reduce of the whole bucket after both backwards."""
        m = os.environ.get("RMM_PEER_MODE")
        if m in ("one", "fork"):
            return m
        return "one" if getattr(self.comm, "shared_device", True) else "fork"

    def _zero1(self) -> bool:
        """Multi-rank optimizer step ZeRO-1 style (PeerComm.allreduce_adam_on): each rank reduces its
        1/W of the fp32 gradient bucket over the peers, applies Adam to it and all-gathers the updated
        masters, in ONE launch per bucket — instead of an all-reduce of the whole bucket followed by
        every rank running the same full Adam (K6). Same bits as all-reduce -> K6 (peer self-test).
        Not with global-norm clipping (the norm needs the whole summed gradient first).
        RMM_PEER_ZERO1=0 restores all-reduce -> K6."""
        return (self._manual is not None and self.world > 1 and self.clip_out is None and self._wptr() != 0
                and getattr(self.comm, "zero1_ready", False) and os.environ.get("RMM_PEER_ZERO1", "1") != "0")

    def _zero1_adam(self, lo: int, hi: int, stream, last: bool):
        """Fused reduce-scatter + Adam + all-gather over flat elements [lo, hi) on `stream`; the last
        launch of the step advances the counters (parity copy in a chained graph, else the ticket)."""
        cur = self._ctr().data_ptr()
        wlo = self._wlo()
        kw = dict(master=self.master.data_ptr() + 4 * lo, m1=self.m1.data_ptr() + 4 * lo,
                  m2=self.m2.data_ptr() + 4 * lo, whi=self._wptr() + 2 * lo, wlo=wlo + 2 * lo if wlo else 0,
                  hp=self.hp.data_ptr(), grad_scale=1.0 / self.world, step_ctr=cur + 8)
        if last:
            kw.update(bump=cur, nbump=2)
            if self._parity and not (self._parity_last and self._par == 0):
                kw["bump_next"] = self._ctrs[1 - self._par].data_ptr()
                self._par ^= 1
            else:
                kw["done"] = self._bump_done.data_ptr()
        self.comm.allreduce_adam_on(self.flat_grad[lo:hi], stream, **kw)
        self._zero1_ranges.add((lo, hi))

    def _zero1_sync(self):
        """Before any non-ZeRO Adam: replicate the moments the ZeRO-1 steps kept on their owners."""
        for lo, hi in sorted(self._zero1_ranges):
            self.comm.replicate_moments(self.flat_grad.dtype, hi - lo, self.m1.data_ptr() + 4 * lo,
                                        self.m2.data_ptr() + 4 * lo)
        self._zero1_ranges.clear()

    def _manual_peer_step(self, full):
        """One multi-rank SGD step with the peer-memory all-reduce (eager or under capture): every
        rank issues the same all-reduce sequence, so the device epoch counters stay in step."""
        mode = self._peer_mode()
        if self._zero1():
            n, t = self.n_params, self._manual
            self._manual_fwd_dense_bwd(full)
            cap = torch.cuda.current_stream(self.device)
            if mode == "fork":  # the dense + heads Adam (final after K12) overlaps the trunk backward
                cs = self.comm.stream
                cs.wait_stream(cap)
                self._zero1_adam(t, n, cs, last=False)
                self._manual_trunk_bwd(full)
                cap.wait_stream(cs)  # one communicator: the two launches may not overlap
                self._zero1_adam(0, t, cap, last=True)
            else:
                self._manual_trunk_bwd(full)
                self._zero1_adam(0, n, cap, last=True)
            return
        self._manual_fwd_dense_bwd(full)
        if mode == "fork":
            cap = torch.cuda.current_stream(self.device)
            cs = self.comm.stream
            cs.wait_stream(cap)
            self.comm.allreduce_on(self.flat_grad[self._manual:], cs)
            self._manual_trunk_bwd(full)
            # the two all-reduces share the peer kernel's per-workgroup epoch counters (and staging
            # parity): the trunk one may only start once the dense one has finished
            cap.wait_stream(cs)
            self.comm.allreduce_on(self.flat_grad[:self._manual], cap)
        else:
            self._manual_trunk_bwd(full)
            self.comm.allreduce(self.flat_grad)
        self._opt_launch()

    def _ctr(self):
        """The device counter copy the step being launched / captured reads."""
        return self._ctrs[self._par]

    def _opt_step(self):
        if self.world > 1:
            self.comm.allreduce(self.flat_grad)
        self._opt_launch()

    def _fast_step(self, full, with_opt: bool):
        h = require_hip()
        mbs, period = full["mbs"], full["period"]
        ctr = self._ctr()
        # K2b: minibatch gather + u8→bf16 NHWC; K2: ONE gather for every per-sample column —
        # both index idx_all at the device step counter
        frames = full["obs"].dtype == torch.uint8 and full["obs"].dim() == 4
        fused = frames and self.heads_ok and getattr(self.model, "fused_trunk_ok", None) is not None \
            and self.model.fused_trunk_ok(full["obs"])
        if fused:  # K10: gather + both convs inside one MFMA kernel
            x = None
        elif frames:
            x = ops.frames_to_nhwc(full["obs"], full["idx"], rows=mbs, ctr=ctr, period=period, dtype=self.cdt)
        else:  # vector observations (e.g. CartPole): plain row gather
            x = ops.gather_rows(full["obs"], full["idx"], rows=mbs, ctr=ctr, period=period)
        cols = None if fused else ops.gather_rows(full["cols"], full["idx"], rows=mbs, ctr=ctr, period=period)
        if fused:  # K10 trunk → K13 → K15 (heads + PPO loss + dheads + dpre, cols gathered in place); bwd K12 → K10
            total, trunk = self.model.forward_frames_ppo(full["obs"], full["cols"], self.coef, self.acc, self._one,
                                                         idx=full["idx"], ctr=ctr, period=period, rows=mbs)
            if total is None:
                cols = ops.gather_rows(full["cols"], full["idx"], rows=mbs, ctr=ctr, period=period)
                from ray_memory_management_amd.rllib.models import dense_heads

                heads = dense_heads(trunk, self.model.dense_tail, self.model.heads)
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
            esz = self.flat_grad.element_size()
            nb = g.numel() * esz
            dst = self.flat_grad.data_ptr() + off * esz
            if g.data_ptr() != dst:  # fused backward kernels already wrote into the bucket
                segs.append((g.data_ptr(), dst, nb))
            off += p.numel()
        if segs:
            h.multi_copy(segs, _stream())                    # K1: remaining grads → one flat bucket
        if with_opt:  # otherwise the caller runs _opt_step (all-reduce + Adam + counters) eagerly
            self._opt_step()

    # ------------------------------------------------------------------ one SGD step (any mode)
    def _step_eager(self, full):
        """One minibatch step without graphs: manual kernels (overlapped all-reduce) or autograd."""
        if self._manual_ok(full) and self._peer_in_graph():
            self._manual_peer_step(full)
        elif self._manual_ok(full):
            self._manual_fwd_dense_bwd(full)
            if self.world > 1:
                self._manual_trunk_bwd(full)
                self.comm.allreduce(self.flat_grad)  # one collective, same stream: no fork / join
            else:
                self._manual_trunk_bwd(full)
                if self._tail_adam():
                    return
            self._opt_launch()
        else:
            self._fast_step(full, True)

    def _make_cols(self, batch):
        """One fp32 column matrix [n, A+4] (old logits, old logp, adv, value target, action)."""
        n = batch.count
        return torch.cat([batch[SampleBatch.ACTION_DIST_INPUTS].float(),
                          batch[SampleBatch.ACTION_LOGP].float().unsqueeze(1),
                          batch[SampleBatch.ADVANTAGES].float().unsqueeze(1),
                          batch[SampleBatch.VALUE_TARGETS].float().unsqueeze(1),
                          batch[SampleBatch.ACTIONS].float().reshape(n, 1)], dim=1).contiguous()

    def _pack(self, obs, cols, A, mbs, nmb):
        """The whole update's minibatch index table [iters * nmb * mbs] (one rand + one sort)."""
        n = obs.shape[0]
        iters = self.cfg["num_sgd_iter"]
        idx = torch.rand(iters, n, device=self.device).argsort(dim=1)[:, :nmb * mbs].reshape(-1).contiguous()
        return {"obs": obs.contiguous(), "cols": cols, "idx": idx, "A": A, "mbs": mbs, "period": iters * nmb}

    def _dbg(self, what: str):
        """RMM_CAPTURE_DEBUG=1: synchronise and log each capture / replay phase (fault hunting:
        the last line in the process log names the phase whose kernels faulted)."""
        if os.environ.get("RMM_CAPTURE_DEBUG"):
            import sys

            torch.cuda.synchronize(self.device)
            print(f"[ppo-learner pid {os.getpid()}] {what} ok (w_bf16 {self._wptr():#x})", file=sys.stderr, flush=True)

    def _capture(self, full):
        self._dbg("capture: start")
        wx = (self.w_x3.hi, self.w_x3.lo) if self.w_x3 is not None else (None, None)
        saved = (self.master.clone(), self.m1.clone(), self.m2.clone(),
                 self.w_bf16.clone() if self.w_bf16 is not None else None, self.ctr.clone(),
                 self.acc.clone(), *(t.clone() if t is not None else None for t in wx))
        manual = self._manual_ok(full)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):  # warm up (MIOpen find, allocator, RCCL communicator) before capture
                self._step_eager(full)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._dbg("capture: eager warm-up steps")
        self._graph = self._graphs_split = None
        self._graph_has_comm = False
        self._chain = 1
        if self.world == 1 or self.cfg["allreduce_in_graph"] or self._peer_in_graph():
            # world of one: `chain` consecutive SGD steps per graph (the device counters index each
            # step's minibatch and Adam step) — consecutive replays of a one-step graph leave ~8 µs
            # idle between them on MI355X (profiles/sgd_chain_r3.txt), a chained graph none.
            # Multi-rank with the peer-memory all-reduce (parallel/comm.py:PeerComm): the same chain,
            # with the bucket all-reduce kernel inside every step (no host between SGD steps)
            peer = self.world > 1 and self._peer_in_graph()
            chain = self._sgd_chain(int(full["period"])) if (self.world == 1 or peer) else 1
            self._graph_has_comm = self.world > 1
            self._parity = manual and chain > 1 and os.environ.get("RMM_CTR_PARITY", "1") != "0"
            self._par = 0
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for k in range(chain):
                        self._parity_last = k == chain - 1
                        if manual and peer:
                            self._manual_peer_step(full)
                        elif manual:
                            self._manual_fwd_dense_bwd(full)
                            if self.world > 1:
                                self.comm.allreduce(self.flat_grad[self._manual:])
                            self._manual_trunk_bwd(full)
                            if self.world > 1:
                                self.comm.allreduce(self.flat_grad[:self._manual])
                            if not self._tail_adam():
                                self._opt_launch()
                        else:
                            self._fast_step(full, True)
            finally:
                par, self._par = self._par, 0
                self._parity = self._parity_last = False
            if par != 0:
                raise RuntimeError("chained SGD graph must leave the step counters in copy 0")
            self._graph = g
            self._chain = chain
        elif manual:
            # multi-rank default: forward + both backwards in one graph, ONE all-reduce of the whole
            # flat bucket on the same stream, Adam graph. A fork onto a comm stream and the join
            # back cost ~16 us inside a graph and ~35 us eagerly on MI355X
            # (benchmarks/stream_fork_cost.py, profiles/stream_fork_r3.txt) — more than the 24 us
            # trunk backward it would hide the dense-bucket all-reduce behind
            ga, gc = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                self._manual_fwd_dense_bwd(full)
                self._manual_trunk_bwd(full)
            with torch.cuda.graph(gc):
                self._opt_launch()
            self._graphs_split = (ga, None, gc)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._fast_step(full, False)
            self._graph = g
        self._dbg("capture: graphs captured")
        for dst, src in zip((self.master, self.m1, self.m2, self.w_bf16, self.ctr, self.acc, *wx), saved):
            if dst is not None:
                dst.copy_(src)  # undo warm-up updates
        self._dbg("capture: state restored")

    def _sgd_chain(self, total: int) -> int:
        """SGD steps captured per graph (world of one): the largest divisor of the update's step
        count that is <= RMM_SGD_CHAIN (default 25)."""
        cap = max(1, int(os.environ.get("RMM_SGD_CHAIN", "25")))
        return max(d for d in range(1, min(cap, max(total, 1)) + 1) if total % d == 0)

    def _replay(self):
        if self._graphs_split is not None and self._graphs_split[1] is None:
            ga, _, gc = self._graphs_split
            ga.replay()
            self.comm.allreduce(self.flat_grad)
            gc.replay()
        elif self.world > 1 and not self.cfg["allreduce_in_graph"] and not self._graph_has_comm:
            self._graph.replay()
            self._opt_step()
        else:
            self._graph.replay()

    def _apply_schedules(self):
        lr = float(self.lr_sched(self.timesteps))
        ent = float(self.ent_sched(self.timesteps))
        if self.fast:
            self.hp[0].fill_(lr)
            self.coef[3].fill_(ent)
        else:
            for g in self.opt.param_groups:
                g["lr"] = lr
        self.cur_lr, self.cur_entropy_coeff = lr, ent

    # ------------------------------------------------------------------ update
    def update(self, batch: SampleBatch) -> Dict[str, float]:
        """num_sgd_iter epochs of shuffled minibatch SGD over a (device-resident) batch."""
        c = self.cfg
        if self.recurrent:
            return self._update_seq(batch)
        if c["standardize_advantages"]:
            a = batch[SampleBatch.ADVANTAGES].float()
            batch[SampleBatch.ADVANTAGES] = (a - a.mean()) / a.std(unbiased=False).clamp_min(1e-4)
        if not self.fast:
            self._apply_schedules()
            return self._update_eager(batch, min(c["sgd_minibatch_size"], batch.count))
        A = batch[SampleBatch.ACTION_DIST_INPUTS].shape[-1]
        return self._update_tables(batch[SampleBatch.OBS], self._make_cols(batch), A)

    def update_fragments(self, frags) -> Dict[str, float]:
        """Train on rollout fragments straight from the object store (postprocess_on_learner):
        K17 ingest (DMA + GAE + advantage standardisation on the GPU), then the SGD epochs."""
        from ray_memory_management_amd.rllib.execution.sample_ingest import (SampleIngest, fragment_dims,
                                                                              fragments_to_batch_cpu)

        c = self.cfg
        A = fragment_dims(frags[0])[2]
        if not self.fast:
            obs, cols = fragments_to_batch_cpu(frags, c["gamma"], c["lambda_"], c["standardize_advantages"])
            batch = SampleBatch({SampleBatch.OBS: obs, SampleBatch.ACTION_DIST_INPUTS: cols[:, :A],
                                 SampleBatch.ACTION_LOGP: cols[:, A], SampleBatch.ADVANTAGES: cols[:, A + 1],
                                 SampleBatch.VALUE_TARGETS: cols[:, A + 2], SampleBatch.ACTIONS: cols[:, A + 3].long()})
            self._apply_schedules()
            return self._update_eager(batch, min(c["sgd_minibatch_size"], batch.count))
        if self._ingest is None:
            self._ingest = SampleIngest(self.device, c["gamma"], c["lambda_"])
        obs, cols = self._ingest.ingest(frags, standardize=c["standardize_advantages"])
        return self._update_tables(obs, cols, A, persistent=True)

    def _update_tables(self, obs, cols, A, persistent=False):
        """`persistent`: obs / cols are the ingest's long-lived device buffers (rewritten in place
        every update, same shape), so the captured graphs read them directly instead of a static
        copy — no 141 MB D2D copy of the frames per update."""
        c = self.cfg
        n = obs.shape[0]
        mbs = min(c["sgd_minibatch_size"], n)
        nmb = max(n // mbs, 1)
        self._apply_schedules()
        packed = self._pack(obs, cols, A, mbs, nmb)
        self.acc.zero_()
        self.coef[4].fill_(self.kl_coeff)
        if self.graphs:
            st = self._static
            if st is None or any(st[k].shape != packed[k].shape for k in ("obs", "cols", "idx")) \
                    or st["mbs"] != mbs:
                keep = ("obs", "cols") if persistent else ()
                self._static = st = {k: (v.clone() if torch.is_tensor(v) and k not in keep else v)
                                     for k, v in packed.items()}
                self._graph = self._graphs_split = None
            else:
                for k in ("obs", "cols", "idx"):
                    if st[k].data_ptr() != packed[k].data_ptr():
                        st[k].copy_(packed[k])
            if self._graph is None and self._graphs_split is None:
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
        self._zero_k15_stats()  # after any capture: its warm-up steps wrote the slab too
        steps, total = 0, c["num_sgd_iter"] * nmb
        chain = getattr(self, "_chain", 1) if self.graphs and self._graph is not None else 1
        if total % chain:  # not expected: the chain divides the period it was captured for
            raise RuntimeError(f"SGD graph chains {chain} steps, update has {total}")
        while steps < total:
            if self.graphs:
                self._replay()
            else:
                self._step_eager(full)
            steps += chain
        self._dbg(f"update: {steps} SGD steps")
        self._fold_k15_stats()
        if self.world > 1:  # KL adaptation and stats from the global batch, identical on every rank
            self.comm.allreduce(self.acc)
            self.acc.mul_(1.0 / self.world)
        acc = (self.acc / float(max(steps, 1) * mbs)).tolist()  # one host sync per update
        if self.world > 1 and hasattr(self.comm, "check"):
            self.comm.check()  # a peer all-reduce that timed out (dead peer) fails the update here
        self.timesteps += n * self.world
        st = self._finish(acc[0], acc[1], acc[2], acc[3], acc[5], steps)
        if self.clip_out is not None:
            st["grad_gnorm"] = float(self.clip_out[1])
        return st

    def _finish(self, pol, vf, ent, kl_mean, total, steps):
        c = self.cfg
        # adaptive KL coefficient (reference ppo.py UpdateKL)
        if kl_mean > 2.0 * c["kl_target"]:
            self.kl_coeff *= 1.5
        elif kl_mean < 0.5 * c["kl_target"]:
            self.kl_coeff *= 0.5
        self.stats = {"total_loss": total, "policy_loss": pol, "vf_loss": vf, "entropy": ent, "kl": kl_mean,
                      "cur_kl_coeff": self.kl_coeff, "num_sgd_steps": steps, "cur_lr": self.cur_lr,
                      "entropy_coeff": self.cur_entropy_coeff}
        return self.stats

    def _update_eager(self, batch, mbs):
        c = self.cfg
        coef = torch.tensor([c["clip_param"], c["vf_clip_param"], c["vf_loss_coeff"], self.cur_entropy_coeff,
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
                self.opt.zero_grad(set_to_none=False)
                total.backward()
                if self.world > 1:  # one flat collective per step
                    for p in self.params:
                        if p.grad is None:
                            p.grad = torch.zeros_like(p)
                    flat = torch.cat([p.grad.reshape(-1) for p in self.params])
                    self.comm.allreduce(flat)
                    flat.mul_(1.0 / self.world)
                    off = 0
                    for p in self.params:
                        p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                        off += p.numel()
                if c["grad_clip"]:
                    nn.utils.clip_grad_norm_(self.params, c["grad_clip"])
                self.opt.step()
                acc += stats.cpu() / mb.count
                steps += 1
        if self.world > 1:
            acc_d = acc.to(self.device)
            self.comm.allreduce(acc_d)
            acc = acc_d.cpu() / self.world
        acc = (acc / max(steps, 1)).tolist()
        self.timesteps += batch.count * self.world
        return self._finish(acc[0], acc[1], acc[2], acc[3], acc[5], steps)

    def _update_seq(self, batch) -> Dict[str, float]:
        """PPO over fixed-length sequences (LSTM / attention models, rllib/recurrent_net.py):
        minibatches are whole sequences (sgd_minibatch_size // max_seq_len of them), each re-run
        from its recorded state_in with `resets` at episode starts; padded steps (seq_lens) are
        masked out of every mean. Reference: ppo_torch_policy.py loss with sequence_mask /
        reduce_mean_valid."""
        from ray_memory_management_amd.rllib.policy.rnn_sequencing import PREV_ACTIONS, PREV_REWARDS, RESETS, \
            SEQ_LENS, state_key

        c = self.cfg
        dev = self.device
        t = lambda k: torch.as_tensor(batch[k], device=dev)  # noqa: E731
        seq_lens = t(SEQ_LENS).long()
        S = int(seq_lens.shape[0])
        rows = int(torch.as_tensor(batch[SampleBatch.OBS]).shape[0])
        L = rows // S
        obs = t(SampleBatch.OBS)
        obs = obs.reshape((S, L) + tuple(obs.shape[1:]))
        mask = (torch.arange(L, device=dev).unsqueeze(0) < seq_lens.unsqueeze(1))          # [S, L]
        cols = {k: t(k).reshape((S, L) + tuple(t(k).shape[1:])) for k in (
            SampleBatch.ACTIONS, SampleBatch.ACTION_LOGP, SampleBatch.ACTION_DIST_INPUTS, SampleBatch.ADVANTAGES,
            SampleBatch.VALUE_TARGETS, RESETS)}
        pa = t(PREV_ACTIONS).reshape((S, L) + tuple(t(PREV_ACTIONS).shape[1:])) if PREV_ACTIONS in batch else None
        pr = t(PREV_REWARDS).reshape(S, L) if PREV_REWARDS in batch else None
        states = []
        k = 0
        while state_key(k) in batch:
            states.append(t(state_key(k)).float())
            k += 1
        adv = cols[SampleBatch.ADVANTAGES].float()
        if c["standardize_advantages"]:
            m = mask.float()
            mu = (adv * m).sum() / m.sum()
            sd = (((adv - mu) ** 2 * m).sum() / m.sum()).sqrt().clamp_min(1e-4)
            adv = (adv - mu) / sd
        self._apply_schedules()
        clip, vf_clip, vf_coeff = c["clip_param"], c["vf_clip_param"], c["vf_loss_coeff"]
        n_mb = max(1, int(c["sgd_minibatch_size"]) // max(L, 1))
        acc = torch.zeros(6, device=dev)
        steps, valid_total = 0, 0.0
        for _ in range(c["num_sgd_iter"]):
            perm = torch.randperm(S, device=dev)
            for i in range(0, S, n_mb):
                idx = perm[i:i + n_mb]
                m = mask[idx].float()
                nv = m.sum().clamp_min(1.0)
                logits, values, _ = self.model.seq(obs[idx], [s[idx] for s in states], cols[RESETS][idx],
                                                   None if pa is None else pa[idx], None if pr is None else pr[idx])
                d = self.dist_cls(logits.float())
                old = self.dist_cls(cols[SampleBatch.ACTION_DIST_INPUTS][idx].float())
                logp = d.logp(cols[SampleBatch.ACTIONS][idx])
                ratio = torch.exp(logp - cols[SampleBatch.ACTION_LOGP][idx].float())
                a_mb = adv[idx]
                surr = torch.min(a_mb * ratio, a_mb * torch.clamp(ratio, 1 - clip, 1 + clip))
                vf = torch.clamp((values.float() - cols[SampleBatch.VALUE_TARGETS][idx].float()) ** 2, max=vf_clip)
                ent = d.entropy()
                kl = old.kl(d)
                per = -surr + vf_coeff * vf - self.cur_entropy_coeff * ent + self.kl_coeff * kl
                loss = (per * m).sum() / nv
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if self.world > 1:
                    for p in self.params:
                        if p.grad is None:
                            p.grad = torch.zeros_like(p)
                    flat = torch.cat([p.grad.reshape(-1) for p in self.params])
                    self.comm.allreduce(flat)
                    flat.mul_(1.0 / self.world)
                    off = 0
                    for p in self.params:
                        p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                        off += p.numel()
                if c["grad_clip"]:
                    nn.utils.clip_grad_norm_(self.params, c["grad_clip"])
                self.opt.step()
                with torch.no_grad():
                    acc += torch.stack([((-surr) * m).sum(), (vf * m).sum(), (ent * m).sum(), (kl * m).sum(),
                                        (((ratio - 1).abs() > clip).float() * m).sum(), (per * m).sum()])
                valid_total += float(nv)
                steps += 1
        if self.world > 1:
            self.comm.allreduce(acc)
            acc.mul_(1.0 / self.world)
        a = (acc / max(valid_total, 1.0)).tolist()
        self.timesteps += int(mask.sum()) * self.world
        return self._finish(a[0], a[1], a[2], a[3], a[5], steps)

    def get_weights(self, numpy: bool = False):
        """fp32 weights keyed like the model's state_dict (ONE device→host copy of the flat masters
        on the fast path). numpy=True returns contiguous ndarrays (zero-copy through the store)."""
        sd = self.model.state_dict()
        out = {}
        if self.fast:  # publish the fp32 masters (the bf16 weights are derived)
            flat = self.master.detach().cpu()
            names = {id(p): n for n, p in self.model.named_parameters()}
            off = 0
            for p in self.params:
                out[names[id(p)]] = flat.as_strided(p.size(), p.stride(), off).contiguous()
                off += p.numel()
        for k, v in sd.items():
            if k not in out:
                out[k] = v.detach().float().cpu().contiguous() if v.is_floating_point() else v.detach().cpu()
        if numpy:
            return {k: v.numpy() for k, v in out.items()}
        return out

    def rebind_bf16(self, flat: torch.Tensor) -> None:
        """Move the bf16 compute weights (and every parameter view) to `flat`: same layout, e.g. an
        HBM object of the GPU object store that co-located rollout workers map zero-copy. Captured
        graphs hold the old pointers, so they are dropped (recaptured by the next update)."""
        if not self.fast or self.w_bf16 is None:
            raise RuntimeError("rebind_bf16 needs the fused bf16 learner")
        if flat.dtype != torch.bfloat16 or flat.numel() != self.n_params or flat.device != self.w_bf16.device:
            raise ValueError("rebind_bf16: flat bf16 buffer of the learner's size on its device expected")
        torch.cuda.synchronize(self.device)
        with torch.no_grad():
            flat.copy_(self.w_bf16)
            off = 0
            for p in self.params:
                p.data = flat.as_strided(p.size(), p.stride(), off)
                off += p.numel()
        self.w_bf16 = flat
        self._graph = self._graphs_split = None

    def set_weights(self, w):
        with torch.no_grad():
            w = {k: torch.as_tensor(v) for k, v in w.items()}
            if self.fast:
                names = {id(p): n for n, p in self.model.named_parameters()}
                off = 0
                for p in self.params:
                    src = w[names[id(p)]].to(self.device).float()
                    self.master.as_strided(p.size(), p.stride(), off).copy_(src)
                    p.copy_(src)
                    off += p.numel()
                if self.w_x3 is not None:  # the kernels' split pair follows the master (in place: aliases stay valid)
                    from ray_memory_management_amd.ops import x3 as X3

                    X3.split(self.master, out=self.w_x3)
            else:
                self.model.load_state_dict(w)


def bootstrap_value(model, obs):
    """Value of the observation after a fragment's last step ([B]): the model's fused value-only
    forward when it has one, else the plain forward's value column."""
    fv = getattr(model, "forward_value", None)
    return fv(obs) if fv is not None else model(obs)[1]


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
        heads = getattr(self.model, "heads", None)
        if getattr(heads, "out_features", 0) >= 2:  # [A logits | value]: no probe forward (MIOpen's solver
            self.A = heads.out_features - 1          # search for a torch fp32 conv costs ~2.5 ms at start-up)
        else:
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
    def run_fragment(self):
        """Step the env `fragment` times into the rollout buffers (one graph replay per step)."""
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

    @torch.no_grad()
    def sample(self) -> SampleBatch:
        self.run_fragment()
        last_v = bootstrap_value(self.model, self.s_obs)
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
