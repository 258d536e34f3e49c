"""Sample-batch GPU ingest: rollout fragments from the object store → the learner's loss tables.

Parity: reference rllib/execution/rollout_ops.py (concat of worker batches) +
rllib/evaluation/postprocessing.py:compute_gae_for_sample_batch (GAE, bootstrapped on truncation)
+ rllib/algorithms/ppo/ppo.py:training_step (standardize advantages) +
rllib/policy/torch_policy.py:load_batch_into_buffer (host → device copy of the train batch).

A *fragment* is what one rollout worker returns for one `sample()` call when postprocessing is left
to the learner (``postprocess_on_learner=True``):

* ``obs``    uint8 [T*n, C, H, W] frames, time-major rows (row = t*n + env);
* ``_raw``   fp32 [T*n, A+5] = [logits(A) | logp | vf pred | reward | done | action];
* ``_boot``  fp32 [n] bootstrap values V(s_T).

The fragment's numpy arrays are zero-copy views into the node's shared-memory object store. On the
learner GPU, :class:`SampleIngest` DMAs every fragment's two tables straight from the store into one
device table each (the concat is the DMA's destination offset; store chunks are hipHostRegister'ed
on first use so every later copy is a page-locked transfer), then ONE K17 launch computes GAE per
(fragment, env) column and writes the PPO loss-column table, and K17b standardises the advantages.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

RAW_EXTRA = 5  # logp, vf, reward, done, action after the A logits


def pack_fragment(obs: np.ndarray, logits: np.ndarray, logp: np.ndarray, vf: np.ndarray, rew: np.ndarray,
                  done: np.ndarray, actions: np.ndarray, boot: np.ndarray):
    """Worker side: time-major [T, n, ...] buffers → a fragment SampleBatch (see module doc)."""
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    T, n = rew.shape
    A = logits.shape[-1]
    raw = np.empty((T * n, A + RAW_EXTRA), dtype=np.float32)
    raw[:, :A] = logits.reshape(T * n, A)
    raw[:, A] = logp.reshape(-1)
    raw[:, A + 1] = vf.reshape(-1)
    raw[:, A + 2] = rew.reshape(-1)
    raw[:, A + 3] = done.reshape(-1)
    raw[:, A + 4] = actions.reshape(-1)
    return SampleBatch({"obs": obs.reshape((T * n,) + obs.shape[2:]), "_raw": raw,
                        "_boot": np.ascontiguousarray(boot, dtype=np.float32)})


def is_fragment(b) -> bool:
    return "_raw" in b and "_boot" in b


def fragment_dims(b) -> Tuple[int, int, int]:
    """(T, n, A) of a fragment."""
    n = int(b["_boot"].shape[0])
    rows = int(b["_raw"].shape[0])
    return rows // n, n, int(b["_raw"].shape[1]) - RAW_EXTRA


def pack_fragment_device(obs, logits, logp, vf, rew, done, actions, boot):
    """GPU rollout worker side: time-major device buffers → a fragment of CUDA tensors (the raw
    table is built on the GPU; returned as task output the tensors go to the HBM object store)."""
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    T, n = rew.shape
    A = logits.shape[-1]
    raw = torch.cat([logits.reshape(T * n, A).float(), logp.reshape(-1, 1).float(), vf.reshape(-1, 1).float(),
                     rew.reshape(-1, 1).float(), done.reshape(-1, 1).float(), actions.reshape(-1, 1).float()], 1)
    return SampleBatch({"obs": obs.reshape((T * n,) + tuple(obs.shape[2:])), "_raw": raw.contiguous(),
                        "_boot": boot.reshape(n).float().contiguous()})


def fragments_to_batch_cpu(frags: Sequence, gamma: float, lam: float, standardize: bool = True):
    """Reference (fp32 torch) ingest: fragments → (obs, cols[N, A+4]) on the CPU. Used by the CPU
    learner path and as the numerics oracle of the GPU kernels."""
    from ray_memory_management_amd import ops

    obs, cols = [], []
    for b in frags:
        T, n, A = fragment_dims(b)
        raw = torch.as_tensor(np.asarray(b["_raw"])).view(T, n, A + RAW_EXTRA)
        adv, ret = ops.gae_reference(raw[..., A + 2], raw[..., A + 1], raw[..., A + 3],
                                     torch.as_tensor(np.asarray(b["_boot"])), gamma, lam)
        c = torch.cat([raw[..., :A + 1], adv.unsqueeze(-1), ret.unsqueeze(-1), raw[..., A + 4:A + 5]], dim=-1)
        cols.append(c.reshape(T * n, A + 4))
        obs.append(torch.as_tensor(np.asarray(b["obs"])))
    cols = torch.cat(cols)
    if standardize:
        a = cols[:, -3]
        cols[:, -3] = (a - a.mean()) / a.std(unbiased=False).clamp_min(1e-4)
    return torch.cat(obs), cols


class SampleIngest:
    """Device-side ingest of rollout fragments for one learner GPU (see module docstring)."""

    def __init__(self, device, gamma: float, lam: float):
        self.device = torch.device(device)
        self.gamma, self.lam = float(gamma), float(lam)
        self._obs = None
        self._raw = None
        self._cols = None
        self._boot = None
        self._stats = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._seg_registered = set()
        self.bytes_ingested = 0
        self.bytes_registered = 0

    def _buf(self, name, shape, dtype):
        t = getattr(self, name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            setattr(self, name, t)
        return t

    def _register_store(self, h):
        from ray_memory_management_amd._private import worker as _w

        w = _w.global_worker
        if w is None or getattr(w, "store", None) is None:
            return
        base = w.store.base_address()
        if base not in self._seg_registered:
            h.host_register_segment(base, w.store.mapped_size())
            self._seg_registered.add(base)

    def ingest(self, frags: Sequence, standardize: bool = True):
        """Returns (obs [N, ...] u8, cols [N, A+4] fp32) resident on the learner GPU."""
        from ray_memory_management_amd._native import require_hip

        if self.device.type != "cuda":
            return fragments_to_batch_cpu(frags, self.gamma, self.lam, standardize)
        h = require_hip()
        self._register_store(h)
        dims = [fragment_dims(b) for b in frags]
        A = dims[0][2]
        if any(d[2] != A for d in dims):
            raise ValueError("ingest: fragments disagree on the action dimension")
        on_dev = torch.is_tensor(frags[0]["obs"])
        obs_shape = tuple(frags[0]["obs"].shape[1:])
        N = sum(T * n for T, n, _ in dims)
        nb = sum(n for _, n, _ in dims)
        obs = self._buf("_obs", (N,) + obs_shape, torch.uint8)
        raw = self._buf("_raw", (N, A + RAW_EXTRA), torch.float32)
        boot = self._buf("_boot", (nb,), torch.float32)
        cols = self._buf("_cols", (N, A + 4), torch.float32)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        table = np.zeros((len(frags), 3), dtype=np.int64)  # IngestBlock: row0 | (T, n) | (boot0, pad)
        row = bo = 0
        orow = obs.stride(0)
        segs = []
        for i, (b, (T, n, _)) in enumerate(zip(frags, dims)):
            rows = T * n
            if on_dev:  # GPU rollout fragments: zero-copy IPC views of the producer's HBM objects
                o, r, bt = b["obs"], b["_raw"], b["_boot"]
                if o.dtype != torch.uint8 or tuple(o.shape[1:]) != obs_shape or not o.is_contiguous():
                    raise ValueError("ingest: fragments must carry contiguous uint8 frames of one shape")
                if r.dtype != torch.float32 or bt.dtype != torch.float32:
                    raise ValueError("ingest: _raw/_boot must be float32")
                segs += [(o.data_ptr(), obs.data_ptr() + row * orow, o.numel()),
                         (r.contiguous().data_ptr(), raw.data_ptr() + row * raw.stride(0) * 4, r.numel() * 4),
                         (bt.contiguous().data_ptr(), boot.data_ptr() + bo * 4, bt.numel() * 4)]
                self.bytes_ingested += o.numel() + r.numel() * 4
            else:
                o = np.asarray(b["obs"])
                r = np.asarray(b["_raw"])
                bt = np.asarray(b["_boot"])
                if o.dtype != np.uint8 or tuple(o.shape[1:]) != obs_shape or not o.flags.c_contiguous:
                    raise ValueError("ingest: fragments must carry contiguous uint8 frames of one shape")
                if r.dtype != np.float32 or not r.flags.c_contiguous or bt.dtype != np.float32:
                    raise ValueError("ingest: _raw/_boot must be contiguous float32")
                self.bytes_registered += h.h2d_from_segment(obs.data_ptr() + row * orow, o.ctypes.data, o.nbytes,
                                                            stream)
                self.bytes_registered += h.h2d_from_segment(raw.data_ptr() + row * raw.stride(0) * 4, r.ctypes.data,
                                                            r.nbytes, stream)
                h.memcpy_async(boot.data_ptr() + bo * 4, bt.ctypes.data, bt.nbytes, stream)
                self.bytes_ingested += o.nbytes + r.nbytes
            table[i, 0] = row
            table[i, 1] = (T & 0xFFFFFFFF) | (n << 32)
            table[i, 2] = bo
            row += rows
            bo += n
        if segs:  # K1: every device-side fragment column into the learner tables, one launch
            h.multi_copy(segs, stream)
        key = table.tobytes()
        if getattr(self, "_blocks_key", None) != key:  # the fragment layout rarely changes: upload once
            self._blocks = torch.from_numpy(table.view(np.uint8).reshape(-1)).to(self.device, non_blocking=False)
            self._blocks_key = key
        blocks = self._blocks
        self._stats.zero_()
        h.ingest_gae(raw.data_ptr(), boot.data_ptr(), blocks.data_ptr(), len(frags), A, self.gamma, self.lam,
                     cols.data_ptr(), self._stats.data_ptr(), stream)
        if standardize:
            h.standardize_col(cols.data_ptr(), N, A + 4, A + 1, self._stats.data_ptr(), stream)
        if not on_dev:  # the host fragments (store views) may be released once the DMAs drained
            torch.cuda.current_stream(self.device).synchronize()
        # device fragments: their HBM objects stay referenced by the caller (the update call's arguments)
        # until the update's final stats readback, so the copies need no host wait here
        return obs, cols


def split_for_learners(refs: List, num_learners: int) -> List[List]:
    """Round-robin assignment of rollout-worker outputs to learner actors (each learner trains on
    its own shard, gradients are averaged: data-parallel PPO)."""
    return [refs[k::num_learners] for k in range(num_learners)]
