"""Sequence models for RLlib policies: the LSTM wrapper and the GTrXL attention wrapper.

Parity: reference rllib/models/torch/recurrent_net.py:116 (LSTMWrapper: a memory on top of the
default network's features, ``lstm_cell_size``, ``lstm_use_prev_action`` / ``lstm_use_prev_reward``,
``max_seq_len``), rllib/models/torch/attention_net.py:37 (GTrXLNet: input projection, L units of
[layer-normed relative multi-head attention over memory + GRU gate, position-wise MLP + GRU gate],
per-unit memory of past unit inputs) and :260 (AttentionWrapper: GTrXL on top of the default
network's features plus previous actions / rewards), rllib/models/catalog.py:492-519 (wrapping when
``use_lstm`` / ``use_attention`` is set).

Design (framework-native, not the reference's ragged layout): training sequences have ONE fixed
length ``L = max_seq_len``. A rollout fragment of T steps per env is cut into ceil(T / L) sequences
per env with the recurrent state recorded at every sequence start; an episode boundary inside a
sequence is a ``resets`` flag (the state returns to its initial value before that step; attention
masks every key from before it) instead of a cut + padding. Every minibatch is then a dense
[S, L] block: fixed shapes for the learner, no per-episode Python loop, and sequences carry state
across episode-free fragment boundaries exactly as the rollout did.

Interface of a sequence model (``is_recurrent = True``):
  * ``initial_state(batch, device)`` → list of state tensors;
  * ``step(obs, state, prev_a, prev_r)`` → (logits, value, new_state), one env step for B envs;
  * ``seq(obs, state_in, resets, prev_a, prev_r)`` with [S, L, ...] inputs → (logits [S, L, A],
    values [S, L], state_out);
  * ``forward(obs)`` → (logits, value) from the initial state (stateless callers).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn


def _act(name):
    from ray_memory_management_amd.rllib.models import _act as a

    return a(name)


# ------------------------------------------------------------------------------------------ trunks
class FCTrunk(nn.Module):
    def __init__(self, obs_dim: int, hiddens, activation: str):
        super().__init__()
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), _act(activation)]
            d = h
        self.net = nn.Sequential(*layers)
        self.out_dim = d

    def forward(self, obs):
        return self.net(obs.reshape(obs.shape[0], -1).float())


class _FeaturesOf(nn.Module):
    def __init__(self, net):
        super().__init__()
        self.net = net
        self.out_dim = net.out_dim

    def forward(self, obs):
        return self.net.features(obs)


def build_trunk(obs_space, cfg: Dict):
    """The feature network a memory sits on (reference: the default model built with
    num_outputs=None): conv stack for images, ComplexInputNetwork for Dict / Tuple spaces,
    fcnet_hiddens MLP otherwise."""
    if hasattr(obs_space, "spaces"):
        from ray_memory_management_amd.rllib.complex_input_net import ComplexInputNetwork

        return _FeaturesOf(ComplexInputNetwork(obs_space, 0, cfg))
    shape = tuple(obs_space.shape or ())
    if len(shape) == 3:
        from ray_memory_management_amd.rllib.complex_input_net import ConvTrunk

        filters = cfg.get("conv_filters")
        if filters is None and max(shape) == 84:
            filters = [(16, 8, 4), (32, 4, 2), (256, 11, 1)]
        scale = 1.0 / 255.0 if np.dtype(getattr(obs_space, "dtype", np.float32)) == np.uint8 else 1.0
        return ConvTrunk(shape, filters, cfg.get("conv_activation", "relu"), scale)
    obs_dim = int(np.prod(shape)) if shape else 1
    return FCTrunk(obs_dim, list(cfg.get("fcnet_hiddens") or [256, 256]), cfg.get("fcnet_activation", "tanh"))


# ------------------------------------------------------------------------------------------ base
class SeqNet(nn.Module):
    is_recurrent = True

    def __init__(self, obs_space, action_space, num_outputs: int, cfg: Dict, use_prev_action: bool,
                 use_prev_reward: bool):
        super().__init__()
        self.max_seq_len = int(cfg.get("max_seq_len", 20))
        self.num_outputs = int(num_outputs)
        self.discrete = hasattr(action_space, "n")
        self.act_in = int(action_space.n) if self.discrete else int(np.prod(action_space.shape))
        self.use_prev_action, self.use_prev_reward = bool(use_prev_action), bool(use_prev_reward)
        self.trunk = build_trunk(obs_space, cfg)
        self.in_dim = self.trunk.out_dim + (self.act_in if self.use_prev_action else 0) + (
            1 if self.use_prev_reward else 0)

    def _encode(self, obs, prev_a=None, prev_r=None):
        """[N, ...] → [N, in_dim]: trunk features (+ previous action one-hot / vector, reward)."""
        parts = [self.trunk(obs)]
        N = parts[0].shape[0]
        if self.use_prev_action:
            if prev_a is None:
                parts.append(parts[0].new_zeros(N, self.act_in))
            elif self.discrete:
                parts.append(torch.nn.functional.one_hot(prev_a.reshape(N).long().clamp_min(0), self.act_in)
                             .to(parts[0].dtype))
            else:
                parts.append(prev_a.reshape(N, self.act_in).to(parts[0].dtype))
        if self.use_prev_reward:
            parts.append((prev_r.reshape(N, 1) if prev_r is not None else parts[0].new_zeros(N, 1)).to(parts[0].dtype))
        return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]

    def _encode_seq(self, obs, prev_a, prev_r):
        S, L = obs.shape[:2]
        flat = lambda x: None if x is None else x.reshape((S * L,) + tuple(x.shape[2:]))  # noqa: E731
        return self._encode(flat(obs), flat(prev_a), flat(prev_r)).reshape(S, L, -1)

    def forward(self, obs):
        B = obs.shape[0]
        logits, v, _ = self.step(obs, self.initial_state(B, obs.device))
        return logits, v

    def reset_state(self, state: List[torch.Tensor], done_mask) -> List[torch.Tensor]:
        """States of envs whose episode ended (done_mask [B] bool) back to the initial state."""
        keep = (~torch.as_tensor(done_mask, dtype=torch.bool, device=state[0].device)).to(state[0].dtype)
        return [s * keep.reshape((-1,) + (1,) * (s.dim() - 1)) for s in state]


# ------------------------------------------------------------------------------------------ LSTM
class LSTMWrapper(SeqNet):
    """reference rllib/models/torch/recurrent_net.py:116: LSTM(cell) over the trunk features, then
    the logits and value branches on the LSTM output. State = [h, c], each [B, cell]."""

    def __init__(self, obs_space, action_space, num_outputs: int, cfg: Dict):
        super().__init__(obs_space, action_space, num_outputs, cfg, cfg.get("lstm_use_prev_action", False),
                         cfg.get("lstm_use_prev_reward", False))
        self.cell = int(cfg.get("lstm_cell_size", 256))
        self.lstm = nn.LSTM(self.in_dim, self.cell, batch_first=True)
        self.logits = nn.Linear(self.cell, self.num_outputs)
        self.value = nn.Linear(self.cell, 1)
        nn.init.orthogonal_(self.logits.weight, 0.01)
        nn.init.zeros_(self.logits.bias)

    def initial_state(self, batch: int, device=None):
        dev = device if device is not None else self.logits.weight.device
        return [torch.zeros(batch, self.cell, device=dev), torch.zeros(batch, self.cell, device=dev)]

    def step(self, obs, state, prev_a=None, prev_r=None):
        x = self._encode(obs, prev_a, prev_r).unsqueeze(1)
        h, c = state
        y, (h, c) = self.lstm(x, (h.unsqueeze(0).contiguous(), c.unsqueeze(0).contiguous()))
        y = y[:, 0]
        return self.logits(y), self.value(y).squeeze(-1), [h[0], c[0]]

    def seq(self, obs, state_in, resets, prev_a=None, prev_r=None):
        x = self._encode_seq(obs, prev_a, prev_r)
        S, L = x.shape[:2]
        r = resets.to(x.dtype)
        h = state_in[0] * (1 - r[:, 0:1])
        c = state_in[1] * (1 - r[:, 0:1])
        if L == 1 or not bool((r[:, 1:] > 0).any()):
            y, (hn, cn) = self.lstm(x, (h.unsqueeze(0).contiguous(), c.unsqueeze(0).contiguous()))
            hn, cn = hn[0], cn[0]
        else:  # an episode ends inside some sequence: step, resetting those rows' state
            h, c = h.unsqueeze(0).contiguous(), c.unsqueeze(0).contiguous()
            ys = []
            for t in range(L):
                if t:
                    keep = (1 - r[:, t]).reshape(1, S, 1)
                    h, c = h * keep, c * keep
                yt, (h, c) = self.lstm(x[:, t:t + 1], (h, c))
                ys.append(yt)
            y = torch.cat(ys, dim=1)
            hn, cn = h[0], c[0]
        return self.logits(y), self.value(y).squeeze(-1), [hn, cn]


# ------------------------------------------------------------------------------------------ GTrXL
class GRUGate(nn.Module):
    """GTrXL gating layer (Parisotto et al. 2019, eq. 5-8): r = σ(W_r y + U_r x),
    z = σ(W_z y + U_z x - b_g), h = tanh(W_g y + U_g (r ⊙ x)), out = (1 - z) ⊙ x + z ⊙ h, with x
    the residual stream and y the sub-layer output; b_g > 0 starts the unit near the identity."""

    def __init__(self, dim: int, init_bias: float = 2.0):
        super().__init__()
        self.w = nn.Linear(dim, 3 * dim, bias=False)
        self.u_rz = nn.Linear(dim, 2 * dim, bias=False)
        self.u_g = nn.Linear(dim, dim, bias=False)
        self.bias = nn.Parameter(torch.full((dim,), float(init_bias)))

    def forward(self, x, y):
        wr, wz, wg = self.w(y).chunk(3, dim=-1)
        ur, uz = self.u_rz(x).chunk(2, dim=-1)
        r = torch.sigmoid(wr + ur)
        z = torch.sigmoid(wz + uz - self.bias)
        h = torch.tanh(wg + self.u_g(r * x))
        return (1 - z) * x + z * h


def _sinusoid(n: int, dim: int, device, dtype):
    pos = torch.arange(n, device=device, dtype=torch.float32).unsqueeze(1)
    inv = torch.exp(torch.arange(0, dim, 2, device=device, dtype=torch.float32) * (-math.log(10000.0) / dim))
    pe = torch.zeros(n, dim, device=device)
    pe[:, 0::2] = torch.sin(pos * inv)
    pe[:, 1::2] = torch.cos(pos * inv[: dim // 2])
    return pe.to(dtype)


class RelMultiHeadAttention(nn.Module):
    """Transformer-XL relative multi-head attention (Dai et al. 2019): scores
    (q + u)·k + (q + v)·R[dist], R = projected sinusoid of the query-key distance, input layer norm,
    ReLU output projection (reference rllib/models/torch/modules/relative_multi_head_attention.py)."""

    def __init__(self, dim: int, heads: int, head_dim: int):
        super().__init__()
        self.h, self.d = heads, head_dim
        self.ln = nn.LayerNorm(dim)
        self.qkv = nn.Linear(dim, 3 * heads * head_dim, bias=False)
        self.pos = nn.Linear(dim, heads * head_dim, bias=False)
        self.u = nn.Parameter(torch.zeros(heads, head_dim))
        self.v = nn.Parameter(torch.zeros(heads, head_dim))
        self.out = nn.Linear(heads * head_dim, dim, bias=False)
        nn.init.xavier_uniform_(self.u)
        nn.init.xavier_uniform_(self.v)

    def forward(self, x, mem, allowed):
        """x [S, L, dim] queries (the current steps), mem [S, M, dim], allowed [S, L, M + L] bool."""
        S, L, D = x.shape
        M = mem.shape[1]
        K = M + L
        h = self.ln(torch.cat([mem, x], dim=1))
        q, k, v = self.qkv(h).view(S, K, 3, self.h, self.d).unbind(2)
        q = q[:, M:]
        R = self.pos(_sinusoid(K, D, x.device, x.dtype)).view(K, self.h, self.d)  # by distance 0..K-1
        content = torch.einsum("slhd,skhd->shlk", q + self.u, k)
        by_dist = torch.einsum("slhd,khd->shlk", q + self.v, R)
        dist = (M + torch.arange(L, device=x.device)).unsqueeze(1) - torch.arange(K, device=x.device).unsqueeze(0)
        pos_score = by_dist.gather(3, dist.clamp(min=0).expand(S, self.h, L, K))
        score = (content + pos_score) * (1.0 / math.sqrt(self.d))
        score = score.masked_fill(~allowed.unsqueeze(1), float("-inf"))
        attn = torch.softmax(score, dim=-1)
        o = torch.einsum("shlk,skhd->slhd", attn, v).reshape(S, L, self.h * self.d)
        return torch.relu(self.out(o))


class GTrXLUnit(nn.Module):
    def __init__(self, dim, heads, head_dim, mlp_dim, gate_bias):
        super().__init__()
        self.mha = RelMultiHeadAttention(dim, heads, head_dim)
        self.gate1 = GRUGate(dim, gate_bias)
        self.mlp = nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, mlp_dim, bias=False), nn.ReLU(),
                                 nn.Linear(mlp_dim, dim, bias=False), nn.ReLU())
        self.gate2 = GRUGate(dim, gate_bias)

    def forward(self, x, mem, allowed):
        x = self.gate1(x, self.mha(x, mem, allowed))
        return self.gate2(x, self.mlp(x))


class GTrXLNet(SeqNet):
    """reference rllib/models/torch/attention_net.py:37 (GTrXLNet) + :260 (AttentionWrapper):
    trunk features (+ previous action / reward) → Linear(attention_dim) → L GTrXL units → logits
    and value branches. State = [memory of unit 0, .., memory of unit L-1, valid length]: unit i's
    memory holds its INPUTS at the last M steps [B, M, dim]; `valid length` [B] is how many of them
    belong to the current episode (older rows are masked: an episode never attends across its
    start, in rollouts and in training alike)."""

    def __init__(self, obs_space, action_space, num_outputs: int, cfg: Dict):
        na = int(cfg.get("attention_use_n_prev_actions", 0) or 0)
        nr = int(cfg.get("attention_use_n_prev_rewards", 0) or 0)
        if na > 1 or nr > 1:
            raise ValueError("attention_use_n_prev_actions / _rewards > 1 are not supported (use 0 or 1)")
        super().__init__(obs_space, action_space, num_outputs, cfg, na == 1, nr == 1)
        self.dim = int(cfg.get("attention_dim", 64))
        self.units = int(cfg.get("attention_num_transformer_units", 1))
        self.mem_inference = int(cfg.get("attention_memory_inference", 50))
        self.mem_training = int(cfg.get("attention_memory_training", 50))
        self.inp = nn.Linear(self.in_dim, self.dim)
        self.blocks = nn.ModuleList([
            GTrXLUnit(self.dim, int(cfg.get("attention_num_heads", 1)), int(cfg.get("attention_head_dim", 32)),
                      int(cfg.get("attention_position_wise_mlp_dim", 32)),
                      float(cfg.get("attention_init_gru_gate_bias", 2.0))) for _ in range(self.units)])
        self.logits = nn.Linear(self.dim, self.num_outputs)
        self.value = nn.Linear(self.dim, 1)
        nn.init.orthogonal_(self.logits.weight, 0.01)
        nn.init.zeros_(self.logits.bias)

    def initial_state(self, batch: int, device=None):
        dev = device if device is not None else self.logits.weight.device
        return [torch.zeros(batch, self.mem_inference, self.dim, device=dev) for _ in range(self.units)] + [
            torch.zeros(batch, device=dev)]

    @staticmethod
    def _allowed(valid, resets, M: int, L: int):
        """[S, L, M + L] attention mask: causal, same episode segment, memory rows of this episode."""
        S = resets.shape[0]
        dev = resets.device
        seg_q = torch.cumsum(resets.long(), dim=1)                       # [S, L] segment of each step
        seg_k = torch.cat([torch.zeros(S, M, dtype=torch.long, device=dev), seg_q], dim=1)
        same = seg_q.unsqueeze(2) == seg_k.unsqueeze(1)                  # [S, L, K]
        j = torch.arange(M + L, device=dev)
        q = (M + torch.arange(L, device=dev)).unsqueeze(1)
        # causal, and at most M steps back: exactly the window a rollout step sees (its M-row memory +
        # itself), so training re-computes the rollout's outputs instead of attending further back
        causal = (j.unsqueeze(0) <= q) & (q - j.unsqueeze(0) <= M)   # [L, K]
        mem_ok = (j.unsqueeze(0) >= (M - valid.long().clamp(0, M)).unsqueeze(1)) | (j.unsqueeze(0) >= M)  # [S, K]
        return same & causal.unsqueeze(0) & mem_ok.unsqueeze(1)

    def _run(self, x, mems, valid, resets):
        """x [S, L, in_dim]; mems: per-unit [S, M, dim]; returns (out [S, L, dim], new mems, new valid)."""
        S, L = x.shape[:2]
        M = mems[0].shape[1]
        allowed = self._allowed(valid, resets, M, L)
        h = self.inp(x)
        new_mems = []
        for blk, mem in zip(self.blocks, mems):
            new_mems.append(torch.cat([mem, h], dim=1)[:, -M:])
            h = blk(h, mem, allowed)
        r = resets.to(torch.long)
        if bool(r.any()):
            last = torch.where(r.any(1), (L - 1) - torch.argmax(r.flip(1), dim=1), torch.full_like(r[:, 0], -1))
            nv = torch.where(last >= 0, (L - last).to(valid.dtype), valid + L)
        else:
            nv = valid + L
        return h, new_mems, nv.clamp(max=M)

    def step(self, obs, state, prev_a=None, prev_r=None):
        x = self._encode(obs, prev_a, prev_r).unsqueeze(1)
        mems, valid = state[:-1], state[-1]
        h, new_mems, nv = self._run(x, mems, valid, torch.zeros(x.shape[0], 1, device=x.device))
        h = h[:, 0]
        return self.logits(h), self.value(h).squeeze(-1), new_mems + [nv]

    def seq(self, obs, state_in, resets, prev_a=None, prev_r=None):
        x = self._encode_seq(obs, prev_a, prev_r)
        mems, valid = state_in[:-1], state_in[-1]
        M = min(self.mem_training, mems[0].shape[1])  # training memory: the most recent M rows
        mems = [m[:, -M:] for m in mems]
        valid = valid.clamp(max=M)
        h, new_mems, nv = self._run(x, mems, valid, resets)
        return self.logits(h), self.value(h).squeeze(-1), new_mems + [nv]

    def reset_state(self, state, done_mask):
        return super().reset_state(state, done_mask)


# ------------------------------------------------------------------------------------------ catalog
def wants_sequence_model(cfg: Optional[Dict]) -> bool:
    cfg = cfg or {}
    return bool(cfg.get("use_lstm") or cfg.get("use_attention"))


def build_sequence_model(obs_space, action_space, num_outputs: int, cfg: Dict) -> SeqNet:
    """reference rllib/models/catalog.py:492-519: wrap the default network in an LSTM or attention
    memory when the model config asks for one (not both)."""
    if cfg.get("use_lstm") and cfg.get("use_attention"):
        raise ValueError("use_lstm and use_attention are mutually exclusive")
    if cfg.get("use_attention"):
        return GTrXLNet(obs_space, action_space, num_outputs, cfg)
    return LSTMWrapper(obs_space, action_space, num_outputs, cfg)


def is_recurrent(model) -> bool:
    return bool(getattr(model, "is_recurrent", False))
