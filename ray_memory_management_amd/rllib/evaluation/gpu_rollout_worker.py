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


class HybridRolloutWorker(GPURolloutWorker):
    """CPU rollout worker whose env steps on the CPU and whose policy runs on its (fractional) GPU.

    Role parity: reference rllib/evaluation/rollout_worker.py with ``num_gpus_per_worker > 0`` and
    a CPU env (the policy is placed on the worker's GPU). MI355X design: each env step is ONE
    HIP-graph replay — pinned-host → HBM observation copy, K10 trunk → K13 dense → K16 heads +
    Gumbel sampling + rollout-row stores (the frame row included), action copy back to pinned
    host — then a single stream sync and the CPU vector-env step. The frames each step uploads for
    inference stay in HBM as the fragment's observation rows, so the fragment is returned as CUDA
    tensors (``pack_fragment_device``): it lands in this process's HBM object store and the learner
    on the same GPU reads it zero-copy via hipIPC — no 28 KB/frame host round trip at the learner.
    """

    def __init__(self, env_creator=None, config: Optional[Dict] = None, worker_index: int = 0,
                 num_workers: int = 0, policy_config: Optional[Dict] = None, seed: Optional[int] = None):
        import torch

        from ray_memory_management_amd._native import require_hip
        from ray_memory_management_amd.rllib.env import make_vector_env
        from ray_memory_management_amd.rllib.models import build_model

        if not torch.cuda.is_available():
            raise RuntimeError("HybridRolloutWorker needs a GPU (num_gpus_per_worker > 0)")
        require_hip()
        self.config = dict(config or {})
        self.worker_index = worker_index
        ec = dict(self.config.get("env_config") or {})
        base_seed = seed if seed is not None else self.config.get("seed")
        s = (int(base_seed or 0) * 1000 + worker_index) & 0x7FFFFFFF
        ec.setdefault("seed", s)
        n = int(self.config.get("num_envs_per_worker", 1))
        self.env = make_vector_env(self.config.get("env"), n, ec)
        if self.env is None:
            raise ValueError("HybridRolloutWorker needs a native CPU vector env")
        torch.set_num_threads(1)
        self.device = torch.device("cuda:0")
        torch.cuda.set_device(0)
        torch.manual_seed(s)
        model = build_model(self.env.observation_space, self.env.action_space, self.config.get("model") or {})
        self.model = model.to(self.device).to(torch.bfloat16).to(memory_format=torch.channels_last)
        self.T = int(self.config.get("rollout_fragment_length", 200))
        self.n = n
        self.seed = s
        obs = np.asarray(self.env.vector_reset())
        T, dev = self.T, self.device
        self.h_obs = torch.empty(obs.shape, dtype=torch.uint8).pin_memory()
        self.h_obs.numpy()[:] = obs
        self.h_act = torch.empty(n, dtype=torch.int64).pin_memory()
        self.s_obs = torch.empty(obs.shape, dtype=torch.uint8, device=dev)
        self.s_obs.copy_(self.h_obs)
        with torch.no_grad():
            logits, _ = self.model(self.s_obs)
        self.A = int(logits.shape[-1])
        self.buf_act = torch.empty((T, n), dtype=torch.int64, device=dev)
        self.buf_logp = torch.empty((T, n), dtype=torch.float32, device=dev)
        self.buf_vf = torch.empty((T, n), dtype=torch.float32, device=dev)
        self.buf_logits = torch.empty((T, n, self.A), dtype=torch.float32, device=dev)
        self.act_now = torch.zeros(n, dtype=torch.int64, device=dev)
        self.ctr_t = torch.zeros(2, dtype=torch.int64, device=dev)  # {rng counter, rollout row}
        self.buf_obs = torch.empty((T,) + obs.shape, dtype=torch.uint8, device=dev)
        self.h_rew = torch.empty((T, n), dtype=torch.float32).pin_memory()
        self.h_done = torch.empty((T, n), dtype=torch.float32).pin_memory()
        self.stream = torch.cuda.Stream(dev)
        self.fused = hasattr(self.model, "forward_sample") and getattr(
            getattr(self.model, "heads", None), "out_features", -1) == self.A + 1
        self._graph = None
        self._ep_len = np.zeros(n, dtype=np.int64)
        self._ep_rew = np.zeros(n, dtype=np.float64)
        self._completed: List[tuple] = []
        self._sample_time = 0.0

    def _policy_step(self):
        """H2D obs → fused policy step (row t of the device buffers) → D2H actions; graph body."""
        import torch

        from ray_memory_management_amd._native import require_hip

        self.s_obs.copy_(self.h_obs, non_blocking=True)
        t, ctr = self.ctr_t[1:2], self.ctr_t[0:1]
        self.buf_obs.index_copy_(0, t, self.s_obs.unsqueeze(0))
        if not (self.fused and self.model.forward_sample(self.s_obs, t, ctr, self.seed, self.buf_act, self.buf_logp,
                                                          self.buf_vf, self.buf_logits, self.act_now)):
            hd = self.model.forward_heads(self.s_obs)
            lp, vp, ld = hd.data_ptr(), hd.data_ptr() + self.A * hd.element_size(), hd.stride(0)
            bf = hd.dtype == torch.bfloat16
            require_hip().sample_store(lp, bf, vp, bf, t.data_ptr(), ctr.data_ptr(), self.seed,
                                       self.buf_act.data_ptr(), self.buf_logp.data_ptr(), self.buf_vf.data_ptr(),
                                       self.buf_logits.data_ptr(), self.act_now.data_ptr(), self.n, self.A,
                                       torch.cuda.current_stream().cuda_stream, ldl=ld, ldv=ld)
        self.h_act.copy_(self.act_now, non_blocking=True)
        self.ctr_t.add_(1)

    def _capture(self):
        import torch

        with torch.cuda.stream(self.stream):
            for _ in range(2):
                self._policy_step()
            self.ctr_t[1].zero_()
        self.stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            self._policy_step()
        self._graph = g

    def sample(self):
        import time

        import torch

        from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment_device

        t0 = time.perf_counter()
        with torch.no_grad():
            if self._graph is None:
                try:
                    self._capture()
                except Exception as e:  # pragma: no cover
                    print(f"[HybridRolloutWorker] HIP graph capture failed ({e!r}); running eagerly")
                    self._graph = False
            # the previous fragment's frames (views of buf_obs) were copied into the HBM object store
            # on the default stream at task return: finish that before overwriting the buffers
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.ctr_t[1].zero_()
            obs_np = self.h_obs.numpy()
            act_np = self.h_act.numpy()
            rew_np, done_np = self.h_rew.numpy(), self.h_done.numpy()
            for t in range(self.T):
                if self._graph:
                    self._graph.replay()
                else:
                    with torch.cuda.stream(self.stream):
                        self._policy_step()
                self.stream.synchronize()
                obs, rew, done = self.env.vector_step(act_np.copy())
                obs_np[:] = obs
                rew_np[t] = rew
                done_np[t] = done
                self._ep_rew += rew
                self._ep_len += 1
                if done.any():
                    for i in np.nonzero(done)[0]:
                        self._completed.append((float(self._ep_rew[i]), int(self._ep_len[i])))
                        self._ep_rew[i] = 0.0
                        self._ep_len[i] = 0
            with torch.cuda.stream(self.stream):
                self.s_obs.copy_(self.h_obs, non_blocking=True)
                _, last_v = self.model(self.s_obs)
                rew_d = self.h_rew.to(self.device, non_blocking=True)
                done_d = self.h_done.to(self.device, non_blocking=True)
                frag = pack_fragment_device(self.buf_obs, self.buf_logits, self.buf_logp, self.buf_vf, rew_d, done_d,
                                            self.buf_act, last_v)
            self.stream.synchronize()
        self._sample_time += time.perf_counter() - t0
        return frag

    def set_weights(self, weights, global_vars=None):
        import torch

        self.stream.synchronize()
        super().set_weights(weights, global_vars)
        torch.cuda.synchronize(self.device)
