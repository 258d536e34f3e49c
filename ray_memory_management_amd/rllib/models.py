"""Policy/value networks. Parity: reference rllib/models/torch/{fcnet,visionnet}.py and
rllib/models/utils.py:get_filter_config (84x84 Atari filters [[16,8,4],[32,4,2],[256,11,1]])."""
from __future__ import annotations

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
        if bf16_path:
            from ray_memory_management_amd import ops

            x = ops.frames_to_nhwc(obs)  # fused u8->bf16 scale + NCHW->NHWC (kernel K2b)
        else:
            x = obs.to(self.heads.weight.dtype if not torch.is_autocast_enabled() else torch.float32) * (1.0 / 255.0)
            x = x.contiguous(memory_format=torch.channels_last)
        return self._trunk(x)

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
    n = getattr(action_space, "n", None)
    if n is None:
        n = 2 * int(torch.tensor(action_space.shape).prod())  # diag-gaussian mean+logstd
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
