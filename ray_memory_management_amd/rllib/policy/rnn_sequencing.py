"""Sequence utilities for recurrent / attention policies.

Parity: reference rllib/policy/rnn_sequencing.py — ``chop_into_sequences`` (:219: cut a flat batch
into per-episode sequences of at most max_seq_len, zero-pad them, keep the state at each sequence
start), ``pad_batch_to_sequences_of_same_size`` (:34: the same applied to a SampleBatch in place,
adding ``seq_lens``) and ``add_time_dimension`` ([B*T, ...] → [B, T, ...]).

The framework's own rollout → learner path uses the fixed-length layout of
``fragment_to_sequences``: a time-major fragment [T, n] becomes n * ceil(T / L) sequences of
exactly L steps (the last one per env zero-padded when L does not divide T), with the recurrent
state recorded by the rollout at every sequence start and a ``resets`` flag where an episode
begins inside a sequence (see rllib/recurrent_net.py). Both layouts are exposed; the reference
functions stay available for user code and custom policies.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

SEQ_LENS = "seq_lens"
RESETS = "resets"
PREV_ACTIONS = "prev_actions"
PREV_REWARDS = "prev_rewards"


def state_key(i: int) -> str:
    return f"state_in_{i}"


def chop_into_sequences(*, feature_columns: Sequence, state_columns: Sequence, max_seq_len: int,
                        episode_ids=None, unroll_ids=None, agent_indices=None, dynamic_max: bool = True,
                        shuffle: bool = False, seq_lens=None, states_already_reduced_to_init: bool = False,
                        **_unused):
    """Returns (padded feature columns [num_seqs * max_len, ...], initial states [num_seqs, ...],
    seq_lens [num_seqs]). A sequence ends where the episode / unroll / agent id changes or after
    `max_seq_len` rows; with `dynamic_max` the padded length is the longest sequence found."""
    n = len(feature_columns[0]) if len(feature_columns) else len(state_columns[0])
    if seq_lens is None or len(seq_lens) == 0:
        ids = [np.asarray(x) for x in (episode_ids, unroll_ids, agent_indices) if x is not None]
        lens, cur = [], 0
        for i in range(n):
            new = i > 0 and any(a[i] != a[i - 1] for a in ids)
            if i > 0 and (new or cur == max_seq_len):
                lens.append(cur)
                cur = 0
            cur += 1
        if n:
            lens.append(cur)
        seq_lens = np.asarray(lens, dtype=np.int32)
    else:
        seq_lens = np.asarray(seq_lens, dtype=np.int32)
    max_len = int(seq_lens.max()) if dynamic_max and len(seq_lens) else int(max_seq_len)
    starts = np.concatenate([[0], np.cumsum(seq_lens)[:-1]]).astype(np.int64)
    feats = []
    for col in feature_columns:
        col = np.asarray(col)
        out = np.zeros((len(seq_lens) * max_len,) + col.shape[1:], dtype=col.dtype)
        for s, (st, ln) in enumerate(zip(starts, seq_lens)):
            out[s * max_len:s * max_len + ln] = col[st:st + ln]
        feats.append(out)
    states = []
    for col in state_columns:
        col = np.asarray(col)
        states.append(col[:len(seq_lens)] if states_already_reduced_to_init else col[starts])
    if shuffle:
        perm = np.random.permutation(len(seq_lens))
        feats = [f.reshape((len(seq_lens), max_len) + f.shape[1:])[perm].reshape(f.shape) for f in feats]
        states = [s[perm] for s in states]
        seq_lens = seq_lens[perm]
    return feats, states, seq_lens


def pad_batch_to_sequences_of_same_size(batch, max_seq_len: int, shuffle: bool = False,
                                        batch_divisibility_req: int = 1, feature_keys: Optional[List[str]] = None,
                                        view_requirements=None, _enable_new_api_stack: bool = False, **_unused):
    """In place: chop `batch` (a SampleBatch with eps_id and state_in_* columns) into padded
    sequences; sets batch['seq_lens'] and replaces state_in_* by the per-sequence initial states."""
    if batch_divisibility_req > 1 and batch.count % batch_divisibility_req == 0 and not any(
            k.startswith("state_in_") for k in batch):
        return
    state_keys = sorted((k for k in batch if k.startswith("state_in_")), key=lambda k: int(k.rsplit("_", 1)[1]))
    if feature_keys is None:
        feature_keys = [k for k in batch if not k.startswith("state_") and k != SEQ_LENS]
    feats, states, lens = chop_into_sequences(
        feature_columns=[batch[k] for k in feature_keys], state_columns=[batch[k] for k in state_keys],
        max_seq_len=max_seq_len, episode_ids=batch.get("eps_id"), unroll_ids=batch.get("unroll_id"),
        agent_indices=batch.get("agent_index"), dynamic_max=True, shuffle=shuffle,
        seq_lens=batch.get(SEQ_LENS))
    for k, v in zip(feature_keys, feats):
        dict.__setitem__(batch, k, v)
    for k, v in zip(state_keys, states):
        dict.__setitem__(batch, k, v)
    dict.__setitem__(batch, SEQ_LENS, lens)
    batch.count = len(feats[0]) if feats else 0
    batch.max_seq_len = int(lens.max()) if len(lens) else max_seq_len
    batch.zero_padded = True


def add_time_dimension(padded_inputs, *, max_seq_len: Optional[int] = None, framework: str = "torch",
                       time_major: bool = False, seq_lens=None):
    """[B * T, ...] → [B, T, ...] (or [T, B, ...] when time_major), T = max_seq_len or the padded
    length implied by seq_lens."""
    n = padded_inputs.shape[0]
    if seq_lens is not None:
        B = len(seq_lens)
        T = n // B
    else:
        T = int(max_seq_len)
        B = n // T
    out = padded_inputs.reshape((B, T) + tuple(padded_inputs.shape[1:]))
    if time_major:
        out = out.swapaxes(0, 1) if isinstance(out, np.ndarray) else out.transpose(0, 1)
    return out


def sequence_mask(seq_lens, maxlen: Optional[int] = None):
    """[B, maxlen] bool: step t of sequence b is real (t < seq_lens[b])."""
    import torch

    lens = torch.as_tensor(seq_lens)
    maxlen = int(maxlen or int(lens.max()))
    return torch.arange(maxlen, device=lens.device).unsqueeze(0) < lens.unsqueeze(1)


def fragment_to_sequences(cols: Dict[str, np.ndarray], dones: np.ndarray, states: List[np.ndarray], L: int,
                          ep_start: Optional[np.ndarray] = None):
    """Time-major fragment → fixed-length sequences.

    cols: name → [T, n, ...] arrays; dones [T, n]; states: per state component, the snapshots the
    rollout took at t = 0, L, 2L, ... → [ceil(T / L), n, ...]; ep_start [n] bool: env i began a
    new episode at t = 0 (its state at t = 0 is the initial one anyway, the flag makes attention
    mask its memory). Returns (columns [S * L, ...] with S = n * ceil(T / L) in env-major sequence
    order, state_in list [S, ...], seq_lens [S], resets [S * L])."""
    T, n = dones.shape
    C = -(-T // L)
    pad = C * L - T

    def seqs(x):
        x = np.asarray(x)
        if pad:
            x = np.concatenate([x, np.zeros((pad,) + x.shape[1:], dtype=x.dtype)], axis=0)
        x = x.reshape((C, L, n) + x.shape[2:])            # [C, L, n, ...]
        x = np.moveaxis(x, 2, 0)                          # [n, C, L, ...]
        return np.ascontiguousarray(x.reshape((n * C * L,) + x.shape[3:]))

    out = {k: seqs(v) for k, v in cols.items()}
    resets = np.zeros((T, n), np.float32)
    resets[1:] = dones[:-1]
    if ep_start is not None:
        resets[0] = np.asarray(ep_start, np.float32)
    state_in = []
    for s in states:
        s = np.asarray(s)                                 # [C, n, ...]
        state_in.append(np.ascontiguousarray(np.moveaxis(s, 1, 0).reshape((n * C,) + s.shape[2:])))
    seq_lens = np.full((n, C), L, np.int32)
    if pad:
        seq_lens[:, -1] = L - pad
    return out, state_in, seq_lens.reshape(-1), seqs(resets)
