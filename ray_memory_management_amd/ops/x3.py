"""Split-bf16 ("bf16x3") tensors for the precision-matched (fp32) PPO path.

An fp32 tensor travels to the x3 kernels (csrc/hip/x3_kernels.hip) as a pair of bf16 planes
``hi = RNE(x)``, ``lo = RNE(x - hi)`` (x = hi + lo to ~17 significant bits); products are
hi*hi + hi*lo + lo*hi on the bf16 MFMA with fp32 accumulation, because gfx950's fp32 MFMA runs at
1/16 of the bf16 rate and it has no TF32 (csrc/hip/x3_device.h). These helpers allocate pairs, split
and join them, and launch the kernels after checking shapes on the host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch


@dataclass
class Pair:
    """Two bf16 planes of the same shape: the split of one fp32 tensor."""
    hi: torch.Tensor
    lo: torch.Tensor

    @staticmethod
    def empty(shape, device) -> "Pair":
        return Pair(torch.empty(shape, dtype=torch.bfloat16, device=device),
                    torch.empty(shape, dtype=torch.bfloat16, device=device))

    @staticmethod
    def zeros(shape, device) -> "Pair":
        return Pair(torch.zeros(shape, dtype=torch.bfloat16, device=device),
                    torch.zeros(shape, dtype=torch.bfloat16, device=device))

    def ptrs(self) -> Tuple[int, int]:
        return (self.hi.data_ptr(), self.lo.data_ptr())

    def float(self) -> torch.Tensor:
        return self.hi.float() + self.lo.float()

    @property
    def shape(self):
        return self.hi.shape

    def view(self, *shape) -> "Pair":
        return Pair(self.hi.view(*shape), self.lo.view(*shape))

    def as_strided(self, size, stride, offset) -> "Pair":
        return Pair(self.hi.as_strided(size, stride, offset), self.lo.as_strided(size, stride, offset))


NONE = (0, 0)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def split(x: torch.Tensor, out: Optional[Pair] = None) -> Pair:
    """fp32 tensor -> Pair (on the GPU: one kernel; elsewhere: the same rounding in torch)."""
    x = x.detach().float().contiguous()
    if out is None:
        out = Pair.empty(x.shape, x.device)
    if x.is_cuda:
        from ray_memory_management_amd._native import require_hip

        require_hip().x3_split(x.data_ptr(), out.hi.data_ptr(), out.lo.data_ptr(), x.numel(), _stream(x))
    else:
        out.hi.copy_(x.to(torch.bfloat16))
        out.lo.copy_((x - out.hi.float()).to(torch.bfloat16))
    return out


def split_like(x: torch.Tensor) -> Pair:
    """Split keeping x's strides (weights in channels-last memory order)."""
    x = x.detach().float()
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return Pair(hi, lo)


def _check_frames(obs):
    if obs.dtype != torch.uint8 or obs.dim() != 4 or tuple(obs.shape[1:]) != (4, 84, 84) or not obs.is_contiguous():
        raise ValueError(f"x3 trunk: need contiguous u8 frames [N,4,84,84], got {tuple(obs.shape)} {obs.dtype}")


def _check_trunk_weights(w1: Pair, b1: Pair, w2: Pair, b2: Pair):
    if tuple(w1.shape) != (16, 4, 8, 8) or tuple(w2.shape) != (32, 16, 4, 4) or b1.hi.numel() != 16 \
            or b2.hi.numel() != 32:
        raise ValueError("x3 trunk: weights must be conv 4->16 8x8 and 16->32 4x4")
    for p in (w1, b1, w2, b2):
        if p.hi.dtype != torch.bfloat16 or p.lo.dtype != torch.bfloat16 or p.hi.stride() != p.lo.stride():
            raise ValueError("x3 trunk: weight pairs must be bf16 planes with equal strides")


def trunk_fwd(obs, w1: Pair, b1: Pair, w2: Pair, b2: Pair, idx=None, ctr=None, period: int = 1,
              rows: Optional[int] = None, h1: Optional[Pair] = None, h2: Optional[Pair] = None) -> Tuple[Pair, Pair]:
    """K10x forward: u8 frames (optionally gathered by a device-counter index window) -> (h1, h2) pairs."""
    from ray_memory_management_amd._native import require_hip

    _check_frames(obs)
    _check_trunk_weights(w1, b1, w2, b2)
    if idx is None:
        rows = obs.shape[0] if rows is None else rows
        if rows > obs.shape[0]:
            raise ValueError("x3 trunk: rows > frames")
    elif rows is None or idx.dtype != torch.int64 or idx.numel() < rows * (period if ctr is not None else 1):
        raise ValueError("x3 trunk: idx must be int64 with rows * period entries and rows given")
    dev = obs.device
    h2 = h2 if h2 is not None else Pair.empty((rows, 11 * 11 * 32), dev)
    if tuple(h2.shape) != (rows, 3872) or (h1 is not None and tuple(h1.shape) != (rows, 441, 16)):
        raise ValueError("x3 trunk: output shapes")
    require_hip().x3_trunk_fwd(obs.data_ptr(), idx.data_ptr() if idx is not None else 0,
                               ctr.data_ptr() if ctr is not None else 0, int(period), int(rows), w1.ptrs(),
                               list(w1.hi.stride()), b1.ptrs(), w2.ptrs(), list(w2.hi.stride()), b2.ptrs(),
                               h1.ptrs() if h1 is not None else NONE, h2.ptrs(), _stream(obs))
    return h1, h2


def trunk_partial_floats(rows: int) -> int:
    from ray_memory_management_amd._native import require_hip

    return int(require_hip().x3_trunk_partial_floats(int(rows)))


def trunk_bwd(obs, w2: Pair, h1: Pair, h2: Pair, dh2: Pair, dpre1: Pair, partial: torch.Tensor, dw1, db1, dw2, db2,
              w1_strides, idx=None, ctr=None, period: int = 1, rows: Optional[int] = None) -> None:
    """K10x backward (two launches + reduce): fp32 dW1 / db1 / dW2 / db2 written in the weights' memory order."""
    from ray_memory_management_amd._native import require_hip

    _check_frames(obs)
    rows = obs.shape[0] if rows is None else rows
    if tuple(h1.shape) != (rows, 441, 16) or tuple(h2.shape) != (rows, 3872) or tuple(dh2.shape) != (rows, 3872) \
            or tuple(dpre1.shape) != (rows, 441, 16):
        raise ValueError("x3 trunk bwd: activation shapes")
    if partial.numel() < trunk_partial_floats(rows) or partial.dtype != torch.float32:
        raise ValueError("x3 trunk bwd: partial workspace too small")
    for t in (dw1, db1, dw2, db2):
        if t.dtype != torch.float32:
            raise ValueError("x3 trunk bwd: fp32 gradients")
    require_hip().x3_trunk_bwd(obs.data_ptr(), idx.data_ptr() if idx is not None else 0,
                               ctr.data_ptr() if ctr is not None else 0, int(period), int(rows), w2.ptrs(),
                               list(w2.hi.stride()), h1.ptrs(), h2.hi.data_ptr(), dh2.ptrs(), dpre1.ptrs(),
                               partial.data_ptr(), dw1.data_ptr(), list(w1_strides), db1.data_ptr(), dw2.data_ptr(),
                               db2.data_ptr(), _stream(obs))


def dense_part_slices(M: int, K: int, N: int = 256) -> int:
    from ray_memory_management_amd._native import require_hip

    return int(require_hip().x3_dense_fwd_part_slices(int(M), int(K), int(N)))


def dense_fwd_part(x: Pair, w: Pair, part: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, int]:
    """K13x: fp32 partials [S, M, N] of x Wᵀ (sum over S, + bias, ReLU happen in the consumer)."""
    from ray_memory_management_amd._native import require_hip

    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K or K % 32 or N % 32 or not x.hi.is_contiguous() or not w.hi.is_contiguous():
        raise ValueError("x3 dense: x [M,K], w [N,K] contiguous, K % 32 == 0, N % 32 == 0")
    S = dense_part_slices(M, K, N)
    if part is None:
        part = torch.empty(S * M * N, dtype=torch.float32, device=x.hi.device)
    if part.numel() < S * M * N:
        raise ValueError("x3 dense: partial buffer too small")
    require_hip().x3_dense_fwd_part(x.ptrs(), w.ptrs(), M, K, N, part.data_ptr(), S, _stream(x.hi))
    return part, S
