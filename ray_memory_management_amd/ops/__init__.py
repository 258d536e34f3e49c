"""Hand-written CDNA4 ops (``csrc/hip/kernels.hip``) with torch-tensor front ends.

CUDA(ROCm) tensors always go to the native HIP kernels — if the ``_hip`` extension is
missing on a GPU box these raise instead of silently falling back. CPU tensors (e.g. rollout
workers without a GPU) use the equivalent torch/numpy math.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ray_memory_management_amd._native import hip_ext, require_hip

__all__ = [
    "multi_copy", "pack_tensors", "unpack_tensors", "concat", "gather_rows", "gae", "vtrace",
    "compress", "decompress", "ppo_loss", "hip_available",
]


def hip_available() -> bool:
    return hip_ext() is not None


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def multi_copy(pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> None:
    """Copy src→dst for many contiguous same-device tensor pairs in ONE kernel launch."""
    if not pairs:
        return
    dev = pairs[0][0].device
    if dev.type != "cuda":
        for s, d in pairs:
            d.view(-1).view(torch.uint8).copy_(s.reshape(-1).view(torch.uint8))
        return
    h = require_hip()
    segs = []
    for s, d in pairs:
        if not (s.is_contiguous() and d.is_contiguous()):
            raise ValueError("multi_copy needs contiguous tensors")
        nb = s.numel() * s.element_size()
        if d.numel() * d.element_size() < nb:
            raise ValueError("multi_copy: destination too small")
        segs.append((s.data_ptr(), d.data_ptr(), nb))
    h.multi_copy(segs, _stream(pairs[0][0]))


def _align(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


def pack_tensors(tensors: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, list]:
    """Serialize a list of tensors into one contiguous uint8 buffer (256 B aligned parts).

    Returns (buffer, layout) with layout = [(offset, nbytes, dtype, shape), ...]."""
    layout, off = [], 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        layout.append((off, nb, t.dtype, tuple(t.shape)))
        off = _align(off + nb)
    dev = tensors[0].device if tensors else torch.device("cpu")
    buf = torch.empty(max(off, 1), dtype=torch.uint8, device=dev)
    pairs = []
    for t, (o, nb, _, _) in zip(tensors, layout):
        if nb:
            pairs.append((t.contiguous(), buf[o:o + nb]))
    multi_copy(pairs)
    return buf, layout


def unpack_tensors(buf: torch.Tensor, layout: list, copy: bool = False) -> List[torch.Tensor]:
    """Inverse of pack_tensors. Zero-copy views unless copy=True (one launch for all parts)."""
    views = []
    for o, nb, dt, shape in layout:
        views.append(buf[o:o + nb].view(dt).view(shape) if nb else torch.empty(shape, dtype=dt, device=buf.device))
    if not copy:
        return views
    outs = [torch.empty_like(v) for v in views]
    multi_copy([(v, o) for v, o in zip(views, outs) if v.numel()])
    return outs


def concat(tensors: Sequence[torch.Tensor], dim: int = 0) -> torch.Tensor:
    """Concatenate along dim 0 with one multi-segment copy launch (sample-batch concat)."""
    if dim != 0 or not tensors or tensors[0].device.type != "cuda":
        return torch.cat(list(tensors), dim=dim)
    t0 = tensors[0]
    rest = t0.shape[1:]
    for t in tensors:
        if t.shape[1:] != rest or t.dtype != t0.dtype or t.device != t0.device:
            raise ValueError("concat: shape/dtype/device mismatch")
    n = sum(t.shape[0] for t in tensors)
    out = torch.empty((n, *rest), dtype=t0.dtype, device=t0.device)
    pairs, r = [], 0
    for t in tensors:
        k = t.shape[0]
        if k:
            pairs.append((t.contiguous(), out[r:r + k]))
        r += k
    multi_copy(pairs)
    return out


def _counter_window(idx, rows, ctr, period):
    """CPU semantics of the device-counter gathers: the rows-long window of idx at ctr[0] % period."""
    k = int(ctr.reshape(-1)[0]) % max(int(period), 1)
    return idx.reshape(-1)[k * rows:(k + 1) * rows]


def gather_rows(x: torch.Tensor, idx: torch.Tensor, rows: int = None, ctr: torch.Tensor = None,
                period: int = 1) -> torch.Tensor:
    """out[i] = x[idx[i]] over dim 0 (minibatch gather).

    With a device counter `ctr` (int64 tensor, element 0 is read by the kernel) the indices are
    idx[(ctr[0] % period) * rows : ... + rows] — a HIP graph walks a whole epoch's index table
    without host-side copies between replays."""
    if ctr is not None and rows is None:
        raise ValueError("gather_rows: rows is required with ctr")
    if x.device.type != "cuda":
        return x[_counter_window(idx, rows, ctr, period) if ctr is not None else idx]
    h = require_hip()
    x = x.contiguous()
    idx = idx.to(device=x.device, dtype=torch.int64).contiguous()
    n = idx.numel() if rows is None else int(rows)
    if ctr is not None:
        assert ctr.dtype == torch.int64 and ctr.device == x.device and idx.numel() >= n * period
    out = torch.empty((n, *x.shape[1:]), dtype=x.dtype, device=x.device)
    row_bytes = x[0].numel() * x.element_size() if x.shape[0] else 0
    if n and row_bytes:
        h.gather_rows(x.data_ptr(), idx.data_ptr(), out.data_ptr(), n, row_bytes, _stream(x),
                      ctr=ctr.data_ptr() if ctr is not None else 0, period=int(period))
    return out


def frames_to_nhwc(x: torch.Tensor, idx: torch.Tensor = None, scale: float = 1.0 / 255.0, rows: int = None,
                   ctr: torch.Tensor = None, period: int = 1, dtype=torch.bfloat16) -> torch.Tensor:
    """uint8 frames [B, C, H, W] (rows optionally gathered by `idx`, or by the device-counter
    window of idx as in gather_rows) → scaled `dtype` (bf16, or fp32 for the precision-matched
    learner), returned as a [B', C, H, W] tensor in channels_last memory (what the NHWC conv
    kernels consume), one pass."""
    if ctr is not None and (rows is None or idx is None):
        raise ValueError("frames_to_nhwc: idx and rows are required with ctr")
    if dtype not in (torch.bfloat16, torch.float32):
        raise ValueError(f"frames_to_nhwc: bf16 or fp32 output, not {dtype}")
    if x.device.type != "cuda":
        if ctr is not None:
            idx = _counter_window(idx, rows, ctr, period)
        y = x[idx] if idx is not None else x
        return (y.float() * scale).to(dtype).contiguous(memory_format=torch.channels_last)
    h = require_hip()
    x = x.contiguous()
    B0, C, H, W = x.shape
    B = int(rows) if rows is not None else (idx.numel() if idx is not None else B0)
    out = torch.empty((B, H, W, C), dtype=dtype, device=x.device)
    if idx is not None:
        idx = idx.to(device=x.device, dtype=torch.int64).contiguous()
    if ctr is not None:
        assert ctr.dtype == torch.int64 and ctr.device == x.device and idx.numel() >= B * period
    if B:
        fn = h.frames_to_nhwc_bf16 if dtype == torch.bfloat16 else h.frames_to_nhwc_f32
        fn(x.data_ptr(), idx.data_ptr() if idx is not None else 0, out.data_ptr(), B, C, H, W, float(scale),
           _stream(x), ctr=ctr.data_ptr() if ctr is not None else 0, period=int(period))
    return out.permute(0, 3, 1, 2)


def gae_reference(rewards, values, dones, last_values, gamma: float, lam: float):
    """Plain fp32 torch GAE over time-major [T, B] tensors (also the CPU path)."""
    T = rewards.shape[0]
    dt = torch.promote_types(rewards.dtype, torch.float32)
    adv = torch.empty(rewards.shape, dtype=dt, device=rewards.device)
    a = torch.zeros(last_values.shape, dtype=dt, device=rewards.device)
    vnext = last_values.to(dt)
    for t in range(T - 1, -1, -1):
        nd = 1.0 - dones[t].to(dt)
        delta = rewards[t].to(dt) + gamma * vnext * nd - values[t].to(dt)
        a = delta + gamma * lam * nd * a
        adv[t] = a
        vnext = values[t].to(dt)
    return adv, adv + values.to(dt)


def gae(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor, last_values: torch.Tensor,
        gamma: float = 0.99, lam: float = 0.95) -> Tuple[torch.Tensor, torch.Tensor]:
    """Generalized advantage estimation on time-major [T, B] tensors.

    Returns (advantages, value_targets). Parity: reference
    rllib/evaluation/postprocessing.py:compute_advantages (use_gae=True)."""
    if rewards.device.type != "cuda":
        return gae_reference(rewards, values, dones, last_values, gamma, lam)
    h = require_hip()
    T, B = rewards.shape
    f = lambda t: t.to(torch.float32).contiguous()  # noqa: E731
    r, v, d, lv = f(rewards), f(values), f(dones), f(last_values).reshape(B)
    adv = torch.empty((T, B), dtype=torch.float32, device=r.device)
    ret = torch.empty_like(adv)
    h.gae(r.data_ptr(), v.data_ptr(), d.data_ptr(), lv.data_ptr(), adv.data_ptr(), ret.data_ptr(),
          T, B, float(gamma), float(lam), _stream(r))
    return adv, ret


def vtrace_reference(behaviour_logp, target_logp, rewards, values, dones, bootstrap, gamma: float,
                     clip_rho: float = 1.0, clip_pg_rho: float = 1.0, lam: float = 1.0):
    """Plain fp32 torch V-trace over time-major [T, B] tensors (also the CPU path). Parity:
    reference rllib/algorithms/impala/vtrace_torch.py:from_importance_weights."""
    f = lambda t: t.to(torch.float32)  # noqa: E731
    rho = torch.exp(f(target_logp) - f(behaviour_logp))
    disc = gamma * (1.0 - f(dones))
    v = f(values)
    boot = f(bootstrap).reshape(-1)
    v_tp1 = torch.cat([v[1:], boot.unsqueeze(0)], 0)
    crho = torch.clamp(rho, max=clip_rho) if clip_rho is not None else rho
    deltas = crho * (f(rewards) + disc * v_tp1 - v)
    cs = lam * torch.clamp(rho, max=1.0)
    acc = torch.zeros_like(boot)
    out = torch.empty_like(v)
    for t in range(v.shape[0] - 1, -1, -1):
        acc = deltas[t] + disc[t] * cs[t] * acc
        out[t] = acc
    vs = out + v
    vs_tp1 = torch.cat([vs[1:], boot.unsqueeze(0)], 0)
    prho = torch.clamp(rho, max=clip_pg_rho) if clip_pg_rho is not None else rho
    return vs, prho * (f(rewards) + disc * vs_tp1 - v)


def vtrace(behaviour_logp, target_logp, rewards, values, dones, bootstrap, gamma: float = 0.99,
           clip_rho: float = 1.0, clip_pg_rho: float = 1.0, lam: float = 1.0):
    """V-trace targets (vs, pg_advantages) over time-major [T, B] tensors; no gradient flows
    through them. CUDA tensors run the K18 kernel (one launch for the whole recursion)."""
    if rewards.device.type != "cuda":
        return vtrace_reference(behaviour_logp, target_logp, rewards, values, dones, bootstrap, gamma, clip_rho,
                                clip_pg_rho, lam)
    h = require_hip()
    T, B = rewards.shape
    f = lambda t: t.detach().to(torch.float32).contiguous()  # noqa: E731
    bl, tl, r, v, d, bt = (f(behaviour_logp), f(target_logp), f(rewards), f(values), f(dones),
                           f(bootstrap).reshape(B))
    for x in (bl, tl, v, d):
        if tuple(x.shape) != (T, B) or x.device != r.device:
            raise ValueError("vtrace: all [T, B] inputs must match rewards' shape and device")
    vs = torch.empty((T, B), dtype=torch.float32, device=r.device)
    pg = torch.empty_like(vs)
    inf = float("inf")
    h.vtrace(bl.data_ptr(), tl.data_ptr(), r.data_ptr(), v.data_ptr(), d.data_ptr(), bt.data_ptr(), T, B,
             float(gamma), inf if clip_rho is None else float(clip_rho),
             inf if clip_pg_rho is None else float(clip_pg_rho), float(lam), vs.data_ptr(), pg.data_ptr(), _stream(r))
    return vs, pg


_BITS = {torch.bfloat16: 16, torch.float16: 16, torch.float32: 32, torch.int16: 16, torch.int32: 32}


def compress(x: torch.Tensor) -> torch.Tensor:
    """Lossless CDNA4 block compression of a 16/32-bit tensor; returns a uint8 device tensor."""
    h = require_hip()
    bits = _BITS.get(x.dtype)
    if bits is None or x.device.type != "cuda":
        raise ValueError("compress: needs a cuda tensor of a 16/32-bit dtype")
    x = x.contiguous()
    n = x.numel()
    out = torch.empty(h.compress_bound(n, bits), dtype=torch.uint8, device=x.device)
    ws = torch.empty(h.compress_workspace(n), dtype=torch.uint8, device=x.device)
    sz = h.compress(x.data_ptr(), n, bits, out.data_ptr(), ws.data_ptr(), _stream(x))
    return out[:sz]


def decompress(buf: torch.Tensor, n: int, dtype: torch.dtype, shape=None) -> torch.Tensor:
    h = require_hip()
    bits = _BITS[dtype]
    out = torch.empty(n, dtype=dtype, device=buf.device)
    ws = torch.empty(h.compress_workspace(n), dtype=torch.uint8, device=buf.device)
    buf = buf.contiguous()
    h.decompress(buf.data_ptr(), out.data_ptr(), n, bits, ws.data_ptr(), _stream(buf))
    return out.view(shape) if shape is not None else out


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logp_new, logp_old, adv, v_new, v_tgt, ent, clip, vf_clip, vf_coeff, ent_coeff):
        h = require_hip()
        f = lambda t: t.detach().to(torch.float32).contiguous().reshape(-1)  # noqa: E731
        ln, lo, a, vn, vt, en = f(logp_new), f(logp_old), f(adv), f(v_new), f(v_tgt), f(ent)
        n = ln.numel()
        g_logp, g_v, g_ent = torch.empty_like(ln), torch.empty_like(ln), torch.empty_like(ln)
        stats = torch.empty(4, dtype=torch.float32, device=ln.device)
        h.ppo_loss(ln.data_ptr(), lo.data_ptr(), a.data_ptr(), vn.data_ptr(), vt.data_ptr(), en.data_ptr(),
                   g_logp.data_ptr(), g_v.data_ptr(), g_ent.data_ptr(), stats.data_ptr(), n,
                   float(clip), float(vf_clip), float(vf_coeff), float(ent_coeff), _stream(ln))
        ctx.save_for_backward(g_logp, g_v, g_ent)
        ctx.shapes = (logp_new.shape, v_new.shape, ent.shape)
        ctx.dtypes = (logp_new.dtype, v_new.dtype, ent.dtype)
        means = stats / n
        total = means[0] + vf_coeff * means[1] - ent_coeff * means[2]
        return total, means.detach()

    @staticmethod
    def backward(ctx, g_total, g_means):
        g_logp, g_v, g_ent = ctx.saved_tensors
        s = ctx.shapes
        dt = ctx.dtypes
        return ((g_logp * g_total).view(s[0]).to(dt[0]), None, None, (g_v * g_total).view(s[1]).to(dt[1]),
                None, (g_ent * g_total).view(s[2]).to(dt[2]), None, None, None, None)


def ppo_loss_reference(logp_new, logp_old, adv, v_new, v_tgt, ent, clip, vf_clip, vf_coeff, ent_coeff):
    ratio = torch.exp(logp_new.float() - logp_old.float())
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
    vf = torch.pow(v_new.float() - v_tgt.float(), 2.0)
    vf_c = torch.clamp(vf, 0, vf_clip)
    total = torch.mean(-surr + vf_coeff * vf_c - ent_coeff * ent.float())
    clip_frac = ((ratio - 1).abs() > clip).float().mean()
    means = torch.stack([(-surr).mean(), vf_c.mean(), ent.float().mean(), clip_frac]).detach()
    return total, means


def ppo_loss(logp_new, logp_old, adv, v_new, v_tgt, ent, clip=0.2, vf_clip=10.0, vf_coeff=1.0, ent_coeff=0.0):
    """Fused PPO loss: returns (total_loss, [policy_loss, vf_loss, entropy, clip_frac])."""
    if logp_new.device.type != "cuda":
        return ppo_loss_reference(logp_new, logp_old, adv, v_new, v_tgt, ent, clip, vf_clip, vf_coeff, ent_coeff)
    return _PPOLoss.apply(logp_new, logp_old, adv, v_new, v_tgt, ent, clip, vf_clip, vf_coeff, ent_coeff)
