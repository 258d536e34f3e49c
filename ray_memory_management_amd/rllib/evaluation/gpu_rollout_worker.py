"""GPU rollout worker: a RolloutWorker whose vectorised env AND policy inference live on its GPU.

Role parity: reference rllib/evaluation/rollout_worker.py with ``num_gpus_per_worker > 0`` (the
policy runs on the worker's GPU). MI355X design: the synthetic Atari env is device-resident
(K9 env step), every env step is ONE HIP-graph replay of K10 trunk → K13 dense → K16 heads +
Gumbel sampling + rollout-row stores, so a 100-step fragment of 50 envs takes a few ms. The
fragment (time-major frames + a packed fp32 row table + bootstrap values) is returned as CUDA
tensors: the runtime's serializer puts each into this process's HBM object store and the learner
on the same GPU reads them zero-copy through hipIPC (GAE runs on the learner, K17).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np


class GPURolloutWorker:
    def __init__(self, env_creator=None, config: Optional[Dict] = None, worker_index: int = 0,
                 num_workers: int = 0, policy_config: Optional[Dict] = None, seed: Optional[int] = None):
        import torch

        from ray_memory_management_amd._native import require_hip
        from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
        from ray_memory_management_amd.rllib.models import build_model
        from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler

        if not torch.cuda.is_available():
            raise RuntimeError("GPURolloutWorker needs a GPU (num_gpus_per_worker > 0)")
        require_hip()
        self.config = dict(config or {})
        self.worker_index = worker_index
        ec = dict(self.config.get("env_config") or {})
        base_seed = seed if seed is not None else self.config.get("seed")
        s = (int(base_seed or 0) * 1000 + worker_index) & 0x7FFFFFFF
        self.device = torch.device("cuda:0")
        torch.cuda.set_device(0)
        n = int(self.config.get("num_envs_per_worker", 1))
        self.env = GPUSyntheticAtariVectorEnv(n, self.device, num_actions=int(ec.get("num_actions", 4)),
                                              episode_len=int(ec.get("episode_len", 1000)), seed=s)
        torch.manual_seed(s)
        model = build_model(self.env.observation_space, self.env.action_space, self.config.get("model") or {})
        # bf16 inference weights in the layout the fused kernels read
        self.model = model.to(self.device).to(torch.bfloat16).to(memory_format=torch.channels_last)
        self.T = int(self.config.get("rollout_fragment_length", 200))
        self.sampler = GPURolloutSampler(self.env, self.model, fragment=self.T, seed=s)
        self._ep_len = np.zeros(n, dtype=np.int64)
        self._completed: List[tuple] = []
        self._sample_time = 0.0

    def sample(self):
        import time

        import torch

        from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment_device

        t0 = time.perf_counter()
        S = self.sampler
        with torch.no_grad():
            S.run_fragment()
            _, last_v = self.model(S.s_obs)
            frag = pack_fragment_device(S.buf_obs, S.buf_logits, S.buf_logp, S.buf_vf, S.buf_rew, S.buf_done,
                                        S.buf_act, last_v)
        self._sample_time += time.perf_counter() - t0
        return frag

    def set_weights(self, weights, global_vars=None):
        import torch

        with torch.no_grad():
            sd = self.model.state_dict()
            for k, v in weights.items():
                if k in sd:
                    sd[k].copy_(torch.as_tensor(np.asarray(v)).to(sd[k].dtype), non_blocking=False)

    def get_weights(self, policies=None):
        return {k: v.detach().float().cpu().numpy() for k, v in self.model.state_dict().items()}

    def get_metrics(self) -> List[tuple]:
        out, self._completed = self._completed, []
        return out

    def sample_time(self):
        return self._sample_time

    def apply(self, fn, *args):
        return fn(self, *args)

    def stop(self):
        pass
