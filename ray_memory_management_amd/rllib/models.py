"""Policy/value networks. Parity: reference rllib/models/torch/{fcnet,visionnet}.py and
rllib/models/utils.py:get_filter_config (84x84 Atari filters [[16,8,4],[32,4,2],[256,11,1]])."""
from __future__ import annotations

import os
from typing import List, Sequence

import torch
import torch.nn as nn


class _ConvBiasReLUFn(torch.autograd.Function):
    """MIOpen conv (no bias) + fused bias/ReLU epilogue (K8); backward: fused ReLU mask + bias grad
    (deterministic two-pass reduction, K8) then MIOpen data/weight grads."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        y = torch.convolution(x, w, None, stride, padding, (1, 1), False, (0, 0), 1)
        if not y.is_contiguous(memory_format=torch.channels_last):
            y = y.contiguous(memory_format=torch.channels_last)
        N, C, H, W = y.shape
        h.bias_relu_fwd(y.data_ptr(), b.data_ptr(), N * H * W, C, True, torch.cuda.current_stream().cuda_stream)
        ctx.save_for_backward(x, w, y)
        ctx.conf = (stride, padding)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        x, w, y = ctx.saved_tensors
        stride, padding = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        N, C, H, W = y.shape
        M = N * H * W
        dpre = torch.empty_like(dy)
        db = torch.empty(C, dtype=y.dtype, device=y.device)
        partial = torch.empty(h.bias_relu_bwd_partials(M) * C, dtype=torch.float32, device=y.device)
        h.bias_relu_bwd(dy.data_ptr(), y.data_ptr(), dpre.data_ptr(), db.data_ptr(), partial.data_ptr(), M, C, True,
                        torch.cuda.current_stream().cuda_stream)
        dx, dw, _ = torch.ops.aten.convolution_backward(
            dpre, x, w, None, stride, padding, (1, 1), False, (0, 0), 1,
            (ctx.needs_input_grad[0], ctx.needs_input_grad[1], False))
        return dx, dw, db, None, None


def _dbg_sync(what: str) -> None:
    """RMM_KERNEL_SYNC_DEBUG=1 (fault hunting): synchronise after a launch and log it, so the last line a
    faulting process printed names the kernel. Never while a HIP graph is being captured."""
    if os.environ.get("RMM_KERNEL_SYNC_DEBUG") and not torch.cuda.is_current_stream_capturing():
        import sys

        torch.cuda.synchronize()
        print(f"[kernel-sync pid {os.getpid()}] {what} ok", file=sys.stderr, flush=True)


class _NatureTrunkFn(torch.autograd.Function):
    """K10: both Nature-CNN convs (+bias/ReLU, + the u8 frame gather/scale) as ONE MFMA kernel
    forward and one kernel (+ a deterministic partial-sum reduce) backward — see
    csrc/hip/conv_kernels.hip. Input: u8 frames [N,4,84,84] and optional minibatch indices (with a
    device step counter window, as ops.gather_rows). Output: h2 [rows, 11*11*32] bf16 (NHWC flatten)."""

    @staticmethod
    def forward(ctx, obs, idx, ctr, period, rows, w1, b1, w2, b2):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        dev = obs.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        train = any(ctx.needs_input_grad[5:9])  # grad mode is off inside forward(): ask ctx
        h2 = torch.empty((rows, 11 * 11 * 32), dtype=torch.bfloat16, device=dev)
        h1 = torch.empty((rows, 441, 16), dtype=torch.bfloat16, device=dev) if train else None
        h.nature_trunk_fwd(obs.data_ptr(), idx.data_ptr() if idx is not None else 0,
                           ctr.data_ptr() if ctr is not None else 0, int(period), int(rows), w1.data_ptr(),
                           list(w1.stride()), b1.data_ptr(), w2.data_ptr(), list(w2.stride()), b2.data_ptr(),
                           h1.data_ptr() if h1 is not None else 0, h2.data_ptr(), stream)
        if train:
            ctx.save_for_backward(obs, idx, ctr, w1, w2, h1, h2)
            ctx.conf = (int(period), int(rows))
            ctx.gout = tuple(_grad_out(t) for t in (w1, b1, w2, b2))
        return h2

    @staticmethod
    def backward(ctx, dh2):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        obs, idx, ctr, w1, w2, h1, h2 = ctx.saved_tensors
        period, rows = ctx.conf
        dh2 = dh2.contiguous()
        dev = obs.device
        part = torch.empty(h.nature_trunk_partial_floats(rows), dtype=torch.float32, device=dev)
        g1, gb1, g2, gb2 = ctx.gout
        dw1 = g1 if g1 is not None else torch.empty_strided(w1.size(), w1.stride(), dtype=w1.dtype, device=dev)
        dw2 = g2 if g2 is not None else torch.empty_strided(w2.size(), w2.stride(), dtype=w2.dtype, device=dev)
        db1 = gb1 if gb1 is not None else torch.empty(16, dtype=w1.dtype, device=dev)
        db2 = gb2 if gb2 is not None else torch.empty(32, dtype=w2.dtype, device=dev)
        assert dw1.stride() == w1.stride() and dw2.stride() == w2.stride()
        h.nature_trunk_bwd(obs.data_ptr(), idx.data_ptr() if idx is not None else 0,
                           ctr.data_ptr() if ctr is not None else 0, period, rows, w2.data_ptr(), list(w2.stride()),
                           h1.data_ptr(), h2.data_ptr(), dh2.data_ptr(), part.data_ptr(), dw1.data_ptr(),
                           list(w1.stride()), db1.data_ptr(), dw2.data_ptr(), db2.data_ptr(),
                           torch.cuda.current_stream(dev).cuda_stream)
        return None, None, None, None, None, dw1, db1, dw2, db2


def _grad_out(p):
    """Optional preallocated gradient buffer of a parameter (e.g. its view into the PPO learner's
    flat gradient bucket): backward kernels write the gradient there directly, no copy."""
    return getattr(p, "_rmm_grad_out", None)


class _DenseFn(torch.autograd.Function):
    """y = act(x Wᵀ + b) for the PPO dense layers on the bf16 GPU path. Forward: one hipBLASLt GEMM
    with the bias(+ReLU) epilogue. Backward: K8b mask + bias column-sum in one launch, dW GEMM
    written straight into the parameter's gradient buffer when it has one, dX GEMM."""

    @staticmethod
    def forward(ctx, x, w, b, relu):
        y = torch._addmm_activation(b, x, w.t()) if relu else torch.addmm(b, x, w.t())
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.relu = relu
        ctx.gout = (_grad_out(w), _grad_out(b))
        return y

    @staticmethod
    def backward(ctx, dy):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        M, C = dy.shape
        gw, gb = ctx.gout
        db = gb if gb is not None else torch.empty(C, dtype=dy.dtype, device=dy.device)
        stream = torch.cuda.current_stream(dy.device).cuda_stream
        if ctx.relu:
            dpre = torch.empty_like(dy)
            h.mask_colsum(dy.data_ptr(), y.data_ptr(), dpre.data_ptr(), db.data_ptr(), M, C, True, stream)
        else:
            dpre = dy
            h.mask_colsum(dy.data_ptr(), 0, 0, db.data_ptr(), M, C, False, stream)
        if gw is not None:
            torch.mm(dpre.t(), x, out=gw)
            dw = gw
        else:
            dw = dpre.t() @ x
        dx = dpre @ w if ctx.needs_input_grad[0] else None
        return dx, dw, db, None


class _DenseHeadsFn(torch.autograd.Function):
    """hidden = ReLU(x Wᵀ + b); heads = hidden Whᵀ + bh. Forward: K13 (small-M MFMA GEMM with the
    bias+ReLU epilogue) and K14 (one wave per row) for the 5-wide head. Backward: ONE K12 launch (csrc/hip/dense_kernels.hip) for dx, dW, db, dWh, dbh,
    writing parameter gradients straight into their gradient buffers when they have one."""

    @staticmethod
    def forward(ctx, x, w, b, wh, bh):
        from ray_memory_management_amd._native import require_hip

        M, K = x.shape
        hidden = torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device)
        require_hip().dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, w.shape[0], hidden.data_ptr(),
                                     torch.cuda.current_stream(x.device).cuda_stream)  # K13
        heads = torch.empty((M, wh.shape[0]), dtype=x.dtype, device=x.device)
        require_hip().dense_heads_fwd(hidden.data_ptr(), wh.data_ptr(), bh.data_ptr(), M, wh.shape[0],
                                      heads.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)  # K14
        ctx.save_for_backward(x, w, wh, hidden)
        ctx.gout = tuple(_grad_out(t) for t in (w, b, wh, bh))
        return heads

    @staticmethod
    def backward(ctx, dheads):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        x, w, wh, hidden = ctx.saved_tensors
        dheads = dheads.contiguous()
        M, K = x.shape
        A1 = wh.shape[0]
        dev = x.device

        def out(g, like):
            return g if g is not None else torch.empty_like(like, memory_format=torch.contiguous_format)

        gw, gb, gwh, gbh = ctx.gout
        dw = out(gw, w)
        db = gb if gb is not None else torch.empty(w.shape[0], dtype=w.dtype, device=dev)
        dwh = out(gwh, wh)
        dbh = gbh if gbh is not None else torch.empty(A1, dtype=wh.dtype, device=dev)
        assert dw.is_contiguous() and dwh.is_contiguous()
        dx = torch.empty_like(x)
        dpre = torch.empty_like(hidden)  # scratch: (dheads Wh) ⊙ [hidden > 0]
        h.dense_heads_bwd(dheads.data_ptr(), A1, wh.data_ptr(), hidden.data_ptr(), x.data_ptr(), w.data_ptr(), M, K,
                          dx.data_ptr(), dw.data_ptr(), db.data_ptr(), dwh.data_ptr(), dbh.data_ptr(), dpre.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
        return dx, dw, db, dwh, dbh


class _DenseHeadsPPOFn(torch.autograd.Function):
    """PPO loss of heads(ReLU(layer(x))) for the fused learner step. Forward: K13 dense + ONE K15
    launch (head GEMM, loss statistics into `acc`, d/dheads and dpre for the backward, with the
    upstream gradient `gout` — a device scalar — known up front). Backward: K12 without its dpre
    pre-kernel. Returns an (unwritten) scalar handle; differentiate it with grad_outputs=gout."""

    @staticmethod
    def forward(ctx, x, w, b, wh, bh, cols, coef, acc, gout, cidx=None, ctr=None, period=1):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        M, K = x.shape
        A1 = wh.shape[0]
        stream = torch.cuda.current_stream(x.device).cuda_stream
        hidden = torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device)
        h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, w.shape[0], hidden.data_ptr(), stream)  # K13
        dz = torch.empty((M, A1), dtype=x.dtype, device=x.device)
        dpre = torch.empty_like(hidden)
        h.dense_heads_ppo(hidden.data_ptr(), wh.data_ptr(), bh.data_ptr(), cols.data_ptr(), coef.data_ptr(),
                          acc.data_ptr(), gout.data_ptr(), M, A1, dz.data_ptr(), dpre.data_ptr(), stream,
                          cidx=cidx.data_ptr() if cidx is not None else 0,
                          ctr=ctr.data_ptr() if ctr is not None else 0, period=int(period))  # K15
        ctx.save_for_backward(x, w, wh, hidden, dz, dpre)
        ctx.gout = tuple(_grad_out(t) for t in (w, b, wh, bh))
        ctx.gout_ptr = gout.data_ptr()
        return torch.empty((), dtype=torch.float32, device=x.device)

    @staticmethod
    def backward(ctx, g):
        from ray_memory_management_amd._native import require_hip

        if g.data_ptr() != ctx.gout_ptr:
            raise RuntimeError("dense_heads_ppo: differentiate with grad_outputs=<the gout scalar of the forward>")
        h = require_hip()
        x, w, wh, hidden, dz, dpre = ctx.saved_tensors
        M, K = x.shape
        A1 = wh.shape[0]
        dev = x.device
        gw, gb, gwh, gbh = ctx.gout
        dw = gw if gw is not None else torch.empty_like(w, memory_format=torch.contiguous_format)
        db = gb if gb is not None else torch.empty(w.shape[0], dtype=w.dtype, device=dev)
        dwh = gwh if gwh is not None else torch.empty_like(wh, memory_format=torch.contiguous_format)
        dbh = gbh if gbh is not None else torch.empty(A1, dtype=wh.dtype, device=dev)
        dx = torch.empty_like(x)
        h.dense_heads_bwd(dz.data_ptr(), A1, wh.data_ptr(), hidden.data_ptr(), x.data_ptr(), w.data_ptr(), M, K,
                          dx.data_ptr(), dw.data_ptr(), db.data_ptr(), dwh.data_ptr(), dbh.data_ptr(), dpre.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream, dpre_ready=True)
        return dx, dw, db, dwh, dbh, None, None, None, None, None, None, None


def dense_heads_ppo_ok(x, layer: nn.Linear, heads: nn.Linear) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and layer.weight.dtype == torch.bfloat16
            and heads.weight.dtype == torch.bfloat16 and layer.out_features == 256 and layer.in_features % 32 == 0
            and 3 <= heads.out_features <= 16 and x.shape[0] <= 640 and layer.bias is not None
            and heads.bias is not None and layer.weight.is_contiguous() and heads.weight.is_contiguous()
            and not os.environ.get("RMM_NO_K12") and not os.environ.get("RMM_NO_K15"))


def dense_heads_ppo(x, layer: nn.Linear, heads: nn.Linear, cols, coef, acc, gout, idx=None, ctr=None,
                    period: int = 1):
    """Fused PPO loss handle over heads(ReLU(layer(x))) (see _DenseHeadsPPOFn). With `idx` the loss
    columns are read in place as cols[idx[...]] (the device-counter window of ops.gather_rows)."""
    M = x.shape[0]
    assert cols.dtype == torch.float32 and cols.is_contiguous() and cols.dim() == 2
    assert cols.shape[1] == heads.out_features + 3
    if idx is None:
        assert cols.shape[0] == M
    else:
        assert idx.dtype == torch.int64 and idx.is_contiguous() and idx.numel() >= M * (period if ctr is not None else 1)
        assert ctr is None or (ctr.dtype == torch.int64 and ctr.device == x.device)
    return _DenseHeadsPPOFn.apply(x.contiguous(), layer.weight, layer.bias, heads.weight, heads.bias, cols, coef, acc,
                                  gout, idx, ctr, period)


def dense_heads(x, layer: nn.Linear, heads: nn.Linear):
    """heads(ReLU(layer(x))) with the fused K12 backward on the bf16 GPU path."""
    ok = (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and layer.weight.dtype == torch.bfloat16
          and heads.weight.dtype == torch.bfloat16 and layer.out_features == 256 and layer.in_features % 32 == 0
          and heads.out_features <= 16 and x.shape[0] <= 640 and layer.bias is not None and heads.bias is not None
          and layer.weight.is_contiguous() and heads.weight.is_contiguous() and not os.environ.get("RMM_NO_K12"))
    if not ok:
        return dense(dense(x, layer, True), heads, False)
    return _DenseHeadsFn.apply(x.contiguous(), layer.weight, layer.bias, heads.weight, heads.bias)


def dense(x, layer: nn.Linear, relu: bool):
    if (x.is_cuda and x.dtype == torch.bfloat16 and layer.weight.dtype == torch.bfloat16 and x.dim() == 2
            and layer.bias is not None):
        return _DenseFn.apply(x.contiguous(), layer.weight, layer.bias, relu)
    y = layer(x)
    return torch.relu(y) if relu else y


def nature_trunk(obs, w1, b1, w2, b2, idx=None, ctr=None, period: int = 1, rows: int = None):
    """Fused Nature-CNN trunk on u8 frames (see _NatureTrunkFn). Checks shapes on the host before
    launching the hand-written kernel."""
    if obs.dtype != torch.uint8 or obs.dim() != 4 or tuple(obs.shape[1:]) != (4, 84, 84) or not obs.is_contiguous():
        raise ValueError(f"nature_trunk: need contiguous u8 frames [N,4,84,84], got {tuple(obs.shape)} {obs.dtype}")
    if tuple(w1.shape) != (16, 4, 8, 8) or tuple(w2.shape) != (32, 16, 4, 4) or b1.numel() != 16 or b2.numel() != 32:
        raise ValueError("nature_trunk: weights must be conv 4->16 8x8 and 16->32 4x4")
    if any(t.dtype != torch.bfloat16 for t in (w1, b1, w2, b2)):
        raise ValueError("nature_trunk: bf16 weights required")
    if idx is None:
        rows = obs.shape[0] if rows is None else rows
        if rows > obs.shape[0]:
            raise ValueError("nature_trunk: rows > frames")
    else:
        if idx.dtype != torch.int64 or not idx.is_contiguous() or rows is None:
            raise ValueError("nature_trunk: idx must be contiguous int64 and rows given")
        if idx.numel() < rows * (period if ctr is not None else 1):
            raise ValueError("nature_trunk: index table shorter than rows * period")
        if ctr is not None and (ctr.dtype != torch.int64 or ctr.device != obs.device):
            raise ValueError("nature_trunk: ctr must be an int64 device tensor")
    return _NatureTrunkFn.apply(obs, idx, ctr, period, rows, w1, b1.contiguous(), w2, b2.contiguous())


class ConvReLU(nn.Conv2d):
    """Conv2d followed by ReLU. On MI355X (bf16 NHWC) the bias add + ReLU and its backward run as
    fused HIP kernels around the MIOpen convolution."""

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16 and self.bias is not None
                and self.out_channels % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
                and not torch.is_autocast_enabled()):
            return _ConvBiasReLUFn.apply(x, self.weight, self.bias, self.stride, self.padding)
        return torch.relu(super().forward(x))


def _act(name):
    return {"relu": nn.ReLU, "tanh": nn.Tanh, "elu": nn.ELU, "swish": nn.SiLU, "silu": nn.SiLU}[name]()


class FullyConnectedNetwork(nn.Module):
    def __init__(self, obs_dim: int, num_outputs: int, hiddens: Sequence[int] = (256, 256), activation="tanh",
                 vf_share_layers: bool = False):
        super().__init__()
        self.vf_share_layers = vf_share_layers

        def mlp():
            layers, d = [], obs_dim
            for h in hiddens:
                layers += [nn.Linear(d, h), _act(activation)]
                d = h
            return nn.Sequential(*layers), d

        self.body, d = mlp()
        self.logits = nn.Linear(d, num_outputs)
        if vf_share_layers:
            self.value = nn.Linear(d, 1)
        else:
            self.vf_body, dv = mlp()
            self.value = nn.Linear(dv, 1)
        nn.init.orthogonal_(self.logits.weight, 0.01)
        nn.init.zeros_(self.logits.bias)

    def forward(self, obs):
        obs = obs.to(self.logits.weight.dtype).flatten(1)  # fp32 on CPU, bf16 on the GPU fast path
        h = self.body(obs)
        v = self.value(h if self.vf_share_layers else self.vf_body(obs))
        return self.logits(h), v.squeeze(-1)


class VisionNetwork(nn.Module):
    """RLlib's default Atari conv stack with a shared value head (vf_share_layers=True).

    Input: uint8 frames [B, 4, 84, 84] (channels-first) or [B, 84, 84, 4]; scaled by 1/255 in the
    first layer. Uses channels_last memory format so MIOpen picks NHWC kernels on gfx950."""

    def __init__(self, num_outputs: int, in_channels: int = 4,
                 filters: List[list] = ((16, 8, 4), (32, 4, 2), (256, 11, 1)), in_hw: int = 84):
        super().__init__()
        layers = []
        c = in_channels
        hw = in_hw
        self.dense_tail = None
        for i, (out, k, s) in enumerate(filters):
            last = i == len(filters) - 1
            pad = 0 if last else _same_pad(hw, k, s)
            if last and pad == 0 and k == hw:
                # A "valid" conv whose kernel covers the whole feature map is a dense layer:
                # run it as one GEMM on the NHWC-flattened map (hipBLASLt, MFMA) instead of an
                # implicit-GEMM conv (MIOpen picks a 2 TFLOP/s kernel for its backward on gfx950).
                self.dense_tail = nn.Linear(c * k * k, out)
                hw = 1
            else:
                layers.append(ConvReLU(c, out, k, s, padding=pad))
                hw = (hw + 2 * pad - k) // s + 1
            c = out
        self.out_hw = hw
        self.convs = nn.Sequential(*layers)
        # the exact RLlib 84x84 Atari stack runs as the fused K10 kernel on the GPU bf16 path
        self.nature = (in_hw == 84 and in_channels == 4 and len(layers) == 2 and self.dense_tail is not None
                       and [(l.in_channels, l.out_channels, l.kernel_size, l.stride, l.padding) for l in layers]
                       == [(4, 16, (8, 8), (4, 4), (2, 2)), (16, 32, (4, 4), (2, 2), (2, 2))])
        self.num_outputs = num_outputs
        # policy logits and the (shared-trunk) value head are ONE Linear of width A+1: one GEMM
        # forward/backward, and the fused loss (K5c) / sampler (K7) read both columns in place.
        self.heads = nn.Linear(c, num_outputs + 1)
        with torch.no_grad():
            w = torch.empty(num_outputs, c)
            nn.init.orthogonal_(w, 0.01)
            self.heads.weight[:num_outputs].copy_(w)
            self.heads.bias[:num_outputs].zero_()

    def forward(self, obs, prescaled: bool = False):
        """Returns (logits [B, A], value [B]) — strided views of the merged head output."""
        h = self.forward_heads(obs, prescaled)
        return h[:, :self.num_outputs], h[:, self.num_outputs]

    def forward_heads(self, obs, prescaled: bool = False):
        """obs: uint8 frames [B,C,H,W] / [B,H,W,C], or (prescaled=True) an already scaled bf16/fp32
        [B,C,H,W] tensor such as ops.frames_to_nhwc() returns. Returns heads [B, A+1]."""
        if prescaled:
            return self._trunk(obs)
        if obs.shape[-1] in (1, 3, 4) and obs.shape[1] not in (1, 3, 4):
            obs = obs.permute(0, 3, 1, 2)
        bf16_path = obs.is_cuda and obs.dtype == torch.uint8 and obs.is_contiguous() and (
            torch.is_autocast_enabled() or self.heads.weight.dtype == torch.bfloat16)
        if bf16_path and self.fused_trunk_ok(obs):
            return self.forward_frames(obs)
        if bf16_path:
            from ray_memory_management_amd import ops

            x = ops.frames_to_nhwc(obs)  # fused u8->bf16 scale + NCHW->NHWC (kernel K2b)
        else:
            x = obs.to(self.heads.weight.dtype if not torch.is_autocast_enabled() else torch.float32) * (1.0 / 255.0)
            x = x.contiguous(memory_format=torch.channels_last)
        return self._trunk(x)

    def fused_trunk_ok(self, obs) -> bool:
        return (self.nature and obs.is_cuda and obs.dtype == torch.uint8 and obs.dim() == 4
                and tuple(obs.shape[1:]) == (4, 84, 84) and obs.is_contiguous()
                and self.heads.weight.dtype == torch.bfloat16 and not torch.is_autocast_enabled()
                and not os.environ.get("RMM_NO_FUSED_TRUNK"))

    # ------------------------------------------------------------ precision-matched (fp32) fused path
    # The fp32 policy keeps fp32 parameters; its fused kernels (K10x / K13x / K16x, csrc/hip/x3_kernels.hip)
    # read every weight as a split bf16 pair hi + lo (rllib/ops/x3.py). The owner attaches the pairs:
    # the PPO learner attaches views of the flat pair its optimizer rewrites after every step, a rollout
    # worker its own pair buffers (copied weights, refresh_x3) or views of the learner's live pair
    # (zero-copy shared weights).
    _X3_NAMES = ("convs.0.weight", "convs.0.bias", "convs.1.weight", "convs.1.bias", "dense_tail.weight",
                 "dense_tail.bias", "heads.weight", "heads.bias")

    def attach_x3(self, pairs) -> None:
        """pairs: {parameter name: ops.x3.Pair} for the 8 Nature-CNN parameters (or None to detach)."""
        if pairs is not None and set(pairs) != set(self._X3_NAMES):
            raise ValueError(f"attach_x3 needs pairs for {self._X3_NAMES}")
        self._x3 = pairs

    def refresh_x3(self) -> None:
        """(Re)split the fp32 parameters into this model's own pair buffers (after a weight copy)."""
        from ray_memory_management_amd.ops import x3

        params = dict(self.named_parameters())
        own = getattr(self, "_x3_own", None)
        if own is None or any(own[n].hi.shape != params[n].shape for n in self._X3_NAMES):
            own = self._x3_own = {n: x3.split_like(params[n]) for n in self._X3_NAMES}
        else:
            for n in self._X3_NAMES:
                p = params[n].detach()
                own[n].hi.copy_(p.to(torch.bfloat16))
                own[n].lo.copy_((p - own[n].hi.float()).to(torch.bfloat16))
        self._x3 = own

    def x3_pairs(self):
        return getattr(self, "_x3", None)

    def fused_x3_ok(self, obs) -> bool:
        """The fp32 policy's fused path applies: Nature-CNN layout, u8 frames, fp32 weights with attached pairs."""
        return (self.nature and getattr(self, "_x3", None) is not None and obs.is_cuda and obs.dtype == torch.uint8
                and obs.dim() == 4 and tuple(obs.shape[1:]) == (4, 84, 84) and obs.is_contiguous()
                and self.heads.weight.dtype == torch.float32 and 3 <= self.heads.out_features <= 16
                and self.dense_tail.out_features == 256 and self.dense_tail.in_features == 3872
                and not os.environ.get("RMM_NO_X3"))

    @torch.no_grad()
    def forward_sample_x3(self, obs, t_ptr, ctr, seed, act, logp, vf, lout, act_now, done=None, push=None) -> bool:
        """fp32 rollout step: K10x trunk (push mode when given) → K13x split-K → K16x (fp32 head row,
        Gumbel-max sampling, rollout-row stores, optional step advance). Same contract as forward_sample."""
        from ray_memory_management_amd._native import require_hip
        from ray_memory_management_amd.ops import x3

        if not self.fused_x3_ok(obs) or (push is not None and len(push) == 3):
            return False
        P = self._x3
        hip = require_hip()
        B = obs.shape[0]
        dev = obs.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        ws = getattr(self, "_x3_ws", None)
        if ws is None or ws["B"] != B:
            S = x3.dense_part_slices(B, 3872, 256)
            ws = self._x3_ws = {"B": B, "h2": x3.Pair.empty((B, 3872), dev), "S": S,
                                "hpart": torch.empty(S * B * 256, dtype=torch.float32, device=dev)}
        w1, b1, w2, b2 = (P[n] for n in self._X3_NAMES[:4])
        if push is not None:
            nf, rows = push[:2]
            hip.x3_trunk_fwd_push(obs.data_ptr(), int(nf), rows.data_ptr() if rows is not None else 0,
                                  t_ptr.data_ptr(), B, w1.ptrs(), list(w1.hi.stride()), b1.ptrs(), w2.ptrs(),
                                  list(w2.hi.stride()), b2.ptrs(), ws["h2"].ptrs(), stream)
        else:
            x3.trunk_fwd(obs, w1, b1, w2, b2, h2=ws["h2"])
        hip.x3_dense_fwd_part(ws["h2"].ptrs(), P["dense_tail.weight"].ptrs(), B, 3872, 256, ws["hpart"].data_ptr(),
                              ws["S"], stream)
        hip.x3_heads_sample(ws["hpart"].data_ptr(), ws["S"], P["dense_tail.bias"].ptrs(), P["heads.weight"].ptrs(),
                            P["heads.bias"].ptrs(), t_ptr.data_ptr(), ctr.data_ptr(), seed, act.data_ptr(),
                            logp.data_ptr(), vf.data_ptr(), lout.data_ptr(),
                            act_now.data_ptr() if hasattr(act_now, "data_ptr") else int(act_now), B,
                            self.heads.out_features, stream, done=done.data_ptr() if done is not None else 0)
        return True

    def forward_frames(self, obs, idx=None, ctr=None, period: int = 1, rows: int = None):
        """u8 frames (optionally gathered by a minibatch index window) → heads [rows, A+1], with both
        convs in the fused K10 kernel."""
        c1, c2 = self.convs[0], self.convs[1]
        h = nature_trunk(obs, c1.weight, c1.bias, c2.weight, c2.bias, idx=idx, ctr=ctr, period=period, rows=rows)
        return dense_heads(h, self.dense_tail, self.heads)

    @torch.no_grad()
    def forward_sample(self, obs, t_ptr, ctr, seed, act, logp, vf, lout, act_now, done=None, push=None) -> bool:
        """Rollout step: K10 trunk → K13s (split-K partials) → K16 (partial sum + bias + ReLU, head GEMM +
        Gumbel-max sampling + rollout-row stores,
        same sampling stream as sample_store). Returns False (nothing launched) when not applicable.
        With `done` (a zeroed int32 device counter) K16 also advances *t_ptr and *ctr by one.
        With `push` = (new-frame pointer [B,84,84] u8, rollout rows [T,B,4,84,84] u8 or None), `obs`
        is the env's device frame stack: K10 shifts it by one, appends the new frames and stores row
        *t_ptr itself (K19 folded into the trunk launch) — also when the fused step does not apply
        (then only the push runs and False is returned)."""
        from ray_memory_management_amd._native import require_hip

        if self.fused_x3_ok(obs) and not (push is not None and len(push) == 3):
            return self.forward_sample_x3(obs, t_ptr, ctr, seed, act, logp, vf, lout, act_now, done=done, push=push)
        B = obs.shape[0]
        layer, heads = self.dense_tail, self.heads
        if not (self.fused_trunk_ok(obs) and heads.out_features >= 3 and heads.out_features <= 16
                and layer is not None and layer.out_features == 256 and layer.in_features % 32 == 0
                and layer.bias is not None and heads.bias is not None and layer.weight.is_contiguous()
                and heads.weight.is_contiguous() and not os.environ.get("RMM_NO_K16")):
            if push is not None:
                if len(push) == 3:
                    raise RuntimeError("band-mode push needs the fused rollout step")
                nf, rows = push
                require_hip().frame_push(obs.data_ptr(), int(nf), rows.data_ptr() if rows is not None else 0,
                                         t_ptr.data_ptr(), B, obs.shape[2] * obs.shape[3],
                                         torch.cuda.current_stream(obs.device).cuda_stream)
            return False

        c1, c2 = self.convs[0], self.convs[1]
        hip = require_hip()
        stream = torch.cuda.current_stream(obs.device).cuda_stream
        if push is not None and len(push) == 3 and push[2] == "rows":
            # band mode: 4 workgroups per frame; the frame stack is rollout row t-1 (mod T)
            nf, rows, _ = push
            h = torch.empty((B, 11 * 11 * 32), dtype=torch.bfloat16, device=obs.device)
            hip.nature_trunk_fwd_push_rows(rows.data_ptr(), rows.shape[0], int(nf), t_ptr.data_ptr(), B,
                                           c1.weight.data_ptr(), list(c1.weight.stride()), c1.bias.data_ptr(),
                                           c2.weight.data_ptr(), list(c2.weight.stride()), c2.bias.data_ptr(),
                                           h.data_ptr(), stream)
        elif push is not None:
            nf, rows = push[:2]
            h = torch.empty((B, 11 * 11 * 32), dtype=torch.bfloat16, device=obs.device)
            hip.nature_trunk_fwd_push(obs.data_ptr(), int(nf), rows.data_ptr() if rows is not None else 0,
                                      t_ptr.data_ptr(), B, c1.weight.data_ptr(), list(c1.weight.stride()),
                                      c1.bias.data_ptr(), c2.weight.data_ptr(), list(c2.weight.stride()),
                                      c2.bias.data_ptr(), h.data_ptr(), stream)
            _dbg_sync(f"K10 push (W1 {c1.weight.data_ptr():#x} b1 {c1.bias.data_ptr():#x} W2 {c2.weight.data_ptr():#x})")
        else:
            h = nature_trunk(obs, c1.weight, c1.bias, c2.weight, c2.bias)
        if os.environ.get("RMM_NO_K13S") is None:  # K13s: split-K partials, summed in K16's prologue
            S = hip.dense_fwd_part_slices(B, h.shape[1], 256)
            hpart = torch.empty(S * B * 256, dtype=torch.float32, device=h.device)
            hip.dense_fwd_part(h.data_ptr(), layer.weight.data_ptr(), B, h.shape[1], 256, hpart.data_ptr(), S, stream)
            _dbg_sync(f"K13s (W {layer.weight.data_ptr():#x})")
            hidden_ptr, part = 0, dict(hpart=hpart.data_ptr(), S=S, hb=layer.bias.data_ptr())
        else:
            hidden = torch.empty((B, 256), dtype=h.dtype, device=h.device)
            hip.dense_relu_fwd(h.data_ptr(), layer.weight.data_ptr(), layer.bias.data_ptr(), B, h.shape[1], 256,
                               hidden.data_ptr(), stream)  # K13
            hidden_ptr, part = hidden.data_ptr(), {}
        hip.dense_heads_sample(hidden_ptr, heads.weight.data_ptr(), heads.bias.data_ptr(), t_ptr.data_ptr(),
                               ctr.data_ptr(), seed, act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(),
                               act_now.data_ptr() if hasattr(act_now, "data_ptr") else int(act_now), B,
                               heads.out_features, stream,
                               done.data_ptr() if done is not None else 0, **part)  # K16 (act_now: maybe device-mapped host)
        _dbg_sync(f"K16 (Wh {heads.weight.data_ptr():#x} bh {heads.bias.data_ptr():#x})")
        return True

    @torch.no_grad()
    def forward_value(self, obs):
        """Value head only ([B] fp32), e.g. the bootstrap value after a rollout fragment. On the fused
        paths this is one sampling step (K10 → K13 → K16, bf16 or x3) into scratch rows — the value
        column is what the step stores; otherwise the plain forward (a torch fp32 conv there runs
        MIOpen's naive kernel on gfx950, ≈0.3 ms for 50 frames)."""
        if obs.is_cuda and (self.fused_x3_ok(obs) or self.fused_trunk_ok(obs)):
            B, A = obs.shape[0], self.heads.out_features - 1
            sc = getattr(self, "_value_scratch", None)
            if sc is None or sc["B"] != B or sc["dev"] != obs.device:
                dev = obs.device
                sc = self._value_scratch = {
                    "B": B, "dev": dev, "t": torch.zeros(1, dtype=torch.int64, device=dev),
                    "ctr": torch.zeros(1, dtype=torch.int64, device=dev),
                    "act": torch.empty((1, B), dtype=torch.int64, device=dev),
                    "logp": torch.empty((1, B), dtype=torch.float32, device=dev),
                    "vf": torch.empty((1, B), dtype=torch.float32, device=dev),
                    "logits": torch.empty((1, B, A), dtype=torch.float32, device=dev),
                    "act_now": torch.empty(B, dtype=torch.int64, device=dev)}
            if self.forward_sample(obs, sc["t"], sc["ctr"], 0, sc["act"], sc["logp"], sc["vf"], sc["logits"],
                                   sc["act_now"]):
                return sc["vf"][0].clone()
        return self(obs)[1].float()

    def forward_frames_ppo(self, obs, cols, coef, acc, gout, idx=None, ctr=None, period: int = 1,
                           rows: int = None):
        """forward_frames fused with the PPO loss (K10 trunk → K13 → K15); `cols` is the FULL loss-column
        table, read through the same index window as the frames. Returns (loss handle, trunk output),
        handle None when the K15 path does not apply (caller falls back to dense_heads + K5c)."""
        c1, c2 = self.convs[0], self.convs[1]
        h = nature_trunk(obs, c1.weight, c1.bias, c2.weight, c2.bias, idx=idx, ctr=ctr, period=period, rows=rows)
        if not dense_heads_ppo_ok(h, self.dense_tail, self.heads):
            return None, h
        return dense_heads_ppo(h, self.dense_tail, self.heads, cols, coef, acc, gout, idx=idx, ctr=ctr,
                               period=period), h

    def _trunk(self, x):
        h = self.convs(x)
        if self.dense_tail is not None:
            # NHWC memory: permute+reshape is a view, the GEMM reads the map in place
            h = torch.relu(self.dense_tail(h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)))
        else:
            if h.shape[-1] != 1 or h.shape[-2] != 1:
                h = torch.nn.functional.adaptive_avg_pool2d(h, 1)
            h = h.flatten(1)
        return self.heads(h)


def _same_pad(hw, k, s):
    """Symmetric padding giving TF "same" output size ceil(hw/s) (RLlib SlimConv2d)."""
    out = -(-hw // s)
    total = max((out - 1) * s + k - hw, 0)
    return -(-total // 2)


def build_model(obs_space, action_space, model_config=None) -> nn.Module:
    model_config = model_config or {}
    from ray_memory_management_amd.rllib.recurrent_net import build_sequence_model, wants_sequence_model

    if model_config.get("custom_model"):  # a registered ModelV2 (ModelCatalog), behind (logits, value)
        if wants_sequence_model(model_config):
            raise ValueError("use_lstm / use_attention wrap the built-in networks; a custom_model must implement "
                             "its own memory (ModelV2 state) instead")
        from ray_memory_management_amd.rllib.modelv2 import build_custom_model

        return build_custom_model(obs_space, action_space, model_config)
    n = getattr(action_space, "n", None)
    if n is None:
        n = 2 * int(torch.tensor(action_space.shape).prod())  # diag-gaussian mean+logstd
    if wants_sequence_model(model_config):  # reference catalog.py:492: LSTM / attention wrapper
        from ray_memory_management_amd.rllib.modelv2 import MODEL_DEFAULTS

        return build_sequence_model(obs_space, action_space, n, {**MODEL_DEFAULTS, **model_config})
    if hasattr(obs_space, "spaces"):  # Dict / Tuple observations (reference complex_input_net.py)
        from ray_memory_management_amd.rllib.complex_input_net import ComplexInputNetwork

        return ComplexInputNetwork(obs_space, n, model_config)
    shape = tuple(obs_space.shape)
    if len(shape) == 3:
        in_ch = shape[0] if shape[0] in (1, 3, 4) and shape[-1] not in (1, 3, 4) else shape[-1]
        filters = model_config.get("conv_filters") or ((16, 8, 4), (32, 4, 2), (256, 11, 1))
        filters = [(f[0], f[1] if isinstance(f[1], int) else f[1][0], f[2] if isinstance(f[2], int) else f[2][0])
                   for f in filters]
        hw = shape[1] if shape[0] == in_ch else shape[0]
        return VisionNetwork(n, in_ch, filters, in_hw=hw)
    obs_dim = int(torch.tensor(shape).prod()) if shape else 1
    return FullyConnectedNetwork(obs_dim, n, model_config.get("fcnet_hiddens", (256, 256)),
                                 model_config.get("fcnet_activation", "tanh"),
                                 model_config.get("vf_share_layers", False))


# ModelV2 API surface (reference rllib/models/__init__.py)
from ray_memory_management_amd.rllib.modelv2 import (  # noqa: E402,F401
    MODEL_DEFAULTS, ActionDistribution, ModelCatalog, ModelV2, Preprocessor, TorchCategorical, TorchDiagGaussian,
    TorchModelV2, get_preprocessor)

# sequence / composite-input networks (reference rllib/models/torch/{recurrent_net,attention_net,
# complex_input_net}.py)
from ray_memory_management_amd.rllib.recurrent_net import (  # noqa: E402,F401
    GTrXLNet, LSTMWrapper, SeqNet as RecurrentNetwork)
from ray_memory_management_amd.rllib.complex_input_net import ComplexInputNetwork  # noqa: E402,F401

AttentionWrapper = GTrXLNet
