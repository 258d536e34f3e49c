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

import os
from typing import Dict, List, Optional

import numpy as np

from ray_memory_management_amd.rllib.ppo_learner import bootstrap_value


class _GateTimeout(RuntimeError):
    """A gated policy step gave up waiting for its frames (the fragment is re-sampled ungated)."""


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
        from ray_memory_management_amd._private.numa import pin_to_gpu

        self.cpu_affinity = pin_to_gpu(0)  # the launching thread on the GPU's socket
        n = int(self.config.get("num_envs_per_worker", 1))
        self.env = GPUSyntheticAtariVectorEnv(n, self.device, num_actions=int(ec.get("num_actions", 4)),
                                              episode_len=int(ec.get("episode_len", 1000)), seed=s)
        torch.manual_seed(s)
        model = build_model(self.env.observation_space, self.env.action_space, self.config.get("model") or {})
        # bf16 inference weights in the layout the fused kernels read
        cdt = torch.float32 if str(self.config.get("compute_dtype", "bf16")) in ("fp32", "float32") else torch.bfloat16
        self.model = model.to(self.device).to(cdt).to(memory_format=torch.channels_last)
        _init_x3(self.model)
        self.T = int(self.config.get("rollout_fragment_length", 200))
        self.sampler = GPURolloutSampler(self.env, self.model, fragment=self.T, seed=s)
        self._ep_len = np.zeros(n, dtype=np.int64)
        self._completed: List[tuple] = []
        self._sample_time = 0.0

    def get_custom_metrics(self):
        return {}

    def sample(self, *_after):  # _after: refs the runtime resolves first (prefetched samples)
        import time

        import torch

        from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment_device

        t0 = time.perf_counter()
        S = self.sampler
        with torch.no_grad():
            S.run_fragment()
            last_v = bootstrap_value(self.model, S.s_obs)
            frag = pack_fragment_device(S.buf_obs, S.buf_logits, S.buf_logp, S.buf_vf, S.buf_rew, S.buf_done,
                                        S.buf_act, last_v)
        self._sample_time += time.perf_counter() - t0
        return frag

    def set_weights(self, weights, global_vars=None):
        import torch

        if isinstance(weights, dict) and "__rmm_shared_x3__" in weights:  # fp32 learner's live split pair
            self._set_shared_x3(weights)
            return
        if isinstance(weights, dict) and "__rmm_shared_bf16__" in weights:  # learner's live HBM weights
            import ray_memory_management_amd as rt

            ref = weights["__rmm_shared_bf16__"][0]
            if getattr(self, "_shared_key", None) == ref.binary():
                return  # already aliased: the learner updated them in place
            flat = rt.get(ref)  # zero-copy (hipIPC) view of the learner's weights
            params = dict(self.model.named_parameters())
            with torch.no_grad():
                if flat.device == self.device:  # same GPU: point the parameters at the learner's HBM
                    for name, off, shape, stride in weights["__rmm_layout__"]:
                        if name in params:
                            params[name].data = flat.as_strided(shape, stride, off)
                    self._shared_key, self._shared_flat = ref.binary(), flat
                    if os.environ.get("RMM_SHARED_WEIGHTS_DEBUG"):
                        import sys

                        lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * flat.element_size()
                        print(f"[shared-weights] worker pid {os.getpid()}: params alias {lo:#x} .. {hi:#x}",
                              file=sys.stderr, flush=True)
                        for name, p in self.model.named_parameters():
                            end = p.data_ptr() + p.numel() * p.element_size()
                            print(f"[shared-weights]   {name} {tuple(p.shape)} {tuple(p.stride())} {p.dtype} "
                                  f"{p.data_ptr():#x}..{end:#x} {'in' if lo <= p.data_ptr() and end <= hi else 'OUTSIDE'}",
                                  file=sys.stderr, flush=True)
                        torch.cuda.synchronize(self.device)
                        chk = float(flat.float().abs().sum())  # reads every byte through the mapping
                        torch.cuda.synchronize(self.device)
                        print(f"[shared-weights] worker pid {os.getpid()}: read the whole alias ok (sum|w| {chk:.4g})",
                              file=sys.stderr, flush=True)
                    self._on_params_rebound()
                    return
                for name, off, shape, stride in weights["__rmm_layout__"]:  # another GPU: copy
                    if name in params:
                        params[name].copy_(flat.to(self.device).as_strided(shape, stride, off))
            return
        if isinstance(weights, dict) and "__rmm_flat_bf16__" in weights:  # learner's HBM weights object
            self._unalias_x3()
            flat = weights["__rmm_flat_bf16__"]
            if flat.device != self.device:
                flat = flat.to(self.device)
            with torch.no_grad():
                sd = self.model.state_dict()
                for name, off, shape, stride in weights["__rmm_layout__"]:
                    if name in sd:
                        sd[name].copy_(flat.as_strided(shape, stride, off))
            self._after_weight_copy()
            return
        self._unalias_x3()
        with torch.no_grad():
            sd = self.model.state_dict()
            for k, v in weights.items():
                if k in sd:
                    sd[k].copy_(torch.as_tensor(np.asarray(v)).to(sd[k].dtype), non_blocking=False)
        self._after_weight_copy()

    def _unalias_x3(self):
        """Before a weight COPY into an fp32 policy that aliases the learner (shared split pair): give the
        parameters their own storage again, so the copy never writes the learner's buffers."""
        if getattr(self.model, "x3_pairs", lambda: None)() is None or getattr(self, "_shared_key", None) is None:
            return
        import torch

        with torch.no_grad():
            for p in self.model.parameters():
                p.data = p.data.clone()
        self._shared_key = None
        self._x3_rebound = True

    def _after_weight_copy(self):
        """Copied fp32 weights: re-split them into the model's own pair (its fused fp32 path reads pairs);
        a worker that aliased the learner's pair before recaptures its graphs."""
        if getattr(self.model, "x3_pairs", lambda: None)() is None:
            return
        self.model.refresh_x3()
        if getattr(self, "_x3_rebound", False):
            self._x3_rebound = False
            self._on_params_rebound()

    def _set_shared_x3(self, weights):
        """Alias the fp32 learner's split pair (hipIPC views of its HBM objects): the model's fused path
        reads the learner's live hi / lo planes, no copy per iteration. Another GPU: copy + re-split."""
        import torch

        import ray_memory_management_amd as rt
        from ray_memory_management_amd.ops import x3

        m_ref, hi_ref, lo_ref = weights["__rmm_shared_x3__"]
        key = m_ref.binary() + hi_ref.binary() + lo_ref.binary()
        if getattr(self, "_shared_key", None) == key:
            return  # already aliased: the learner updates master and pair in place
        master, hi, lo = rt.get(m_ref), rt.get(hi_ref), rt.get(lo_ref)
        params = dict(self.model.named_parameters())
        layout = weights["__rmm_layout__"]
        with torch.no_grad():
            if master.device == self.device:  # same GPU: parameters alias the fp32 master, kernels the pair
                for name, off, shape, stride in layout:
                    if name in params:
                        params[name].data = master.as_strided(shape, stride, off)
                self.model.attach_x3({name: x3.Pair(hi.as_strided(shape, stride, off), lo.as_strided(shape, stride, off))
                                      for name, off, shape, stride in layout})
                self._shared_key, self._shared_flat = key, (master, hi, lo)
                self._on_params_rebound()
                return
            for name, off, shape, stride in layout:  # another GPU: copy + own pair
                if name in params:
                    params[name].copy_(master.to(self.device).as_strided(shape, stride, off))
        self.model.refresh_x3()

    def get_weights(self, policies=None):
        return {k: v.detach().float().cpu().numpy() for k, v in self.model.state_dict().items()}

    def _on_params_rebound(self):
        """Parameters now live elsewhere: captured graphs hold the old pointers."""
        self.sampler._graph = None

    def get_metrics(self) -> List[tuple]:
        out, self._completed = self._completed, []
        return out

    def sample_time(self):
        return self._sample_time

    def apply(self, fn, *args):
        return fn(self, *args)

    def stop(self):
        pass


def _init_x3(model) -> None:
    """fp32 Nature-CNN policy: give the model its own split-bf16 weight pair so its rollout step runs on
    the fused x3 kernels (K10x / K13x / K16x); bf16 models and other networks are left alone."""
    import torch

    if (getattr(model, "nature", False) and hasattr(model, "refresh_x3")
            and getattr(getattr(model, "heads", None), "weight", None) is not None
            and model.heads.weight.dtype == torch.float32 and model.heads.weight.is_cuda):
        from ray_memory_management_amd.rllib.ppo_learner import _x3_available

        if _x3_available():
            model.refresh_x3()


class _EnvGroup:
    """One double-buffered slice of a hybrid worker's envs: its own CPU vector env, pinned
    observation / action staging, device rollout buffers, RNG/row counters and HIP graph."""

    def __init__(self, env, model, T: int, A: int, dev, seed: int):
        import torch

        self.env, self.model, self.T, self.A, self.dev, self.seed = env, model, T, A, dev, seed
        obs = np.asarray(env.vector_reset())
        n = self.n = obs.shape[0]
        self.h_obs = torch.empty(obs.shape, dtype=torch.uint8).pin_memory()
        self.h_obs.numpy()[:] = obs
        self.h_act = torch.empty(n, dtype=torch.int64).pin_memory()
        self.h_rew = torch.empty((T, n), dtype=torch.float32).pin_memory()
        self.h_done = torch.empty((T, n), dtype=torch.float32).pin_memory()
        self.s_obs = torch.empty(obs.shape, dtype=torch.uint8, device=dev)
        self.buf_obs = torch.empty((T,) + obs.shape, dtype=torch.uint8, device=dev)
        self.buf_act = torch.empty((T, n), dtype=torch.int64, device=dev)
        self.buf_logp = torch.empty((T, n), dtype=torch.float32, device=dev)
        self.buf_vf = torch.empty((T, n), dtype=torch.float32, device=dev)
        self.buf_logits = torch.empty((T, n, A), dtype=torch.float32, device=dev)
        self.act_now = torch.zeros(n, dtype=torch.int64, device=dev)
        self.ctr_t = torch.zeros(2, dtype=torch.int64, device=dev)  # {rng counter, rollout row}
        # K16's completion counter (K16 advances the step counters itself); RMM_NO_K16_ADVANCE=1 → add kernel
        # (word 0; the fused K13x + K16x launch also uses one ticket word per 16-row tile after it)
        self.k16_done = (None if os.environ.get("RMM_NO_K16_ADVANCE")
                         else torch.zeros(64, dtype=torch.int32, device=dev))
        self.fused = hasattr(model, "forward_sample") and getattr(
            getattr(model, "heads", None), "out_features", -1) == A + 1
        # device frame stacks (K19): upload only each env's newest frame, shift the stack in HBM
        self.device_stack = (bool(getattr(env, "frame_stack_continuous", False)) and hasattr(env, "vector_step_frames")
                             and obs.ndim == 4 and obs.shape[1] == 4 and (obs.shape[2] * obs.shape[3]) % 16 == 0)
        # K10 band mode (rollout): each frame split over 4 workgroups; the frame stack of step t is
        # rollout row t-1 (mod T), so no separate stack buffer is kept. Opt-in (RMM_BAND_PUSH=1) until
        # measured on the GPU
        self.band = (self.device_stack and self.fused and os.environ.get("RMM_BAND_PUSH") == "1"
                     and os.environ.get("RMM_NO_FOLD_PUSH") is None
                     and bool(getattr(model, "fused_trunk_ok", lambda o: False)(self.s_obs)))
        if self.device_stack:
            self.hw = obs.shape[2] * obs.shape[3]
            self.h_new = torch.empty((n,) + obs.shape[2:], dtype=torch.uint8).pin_memory()
            self.s_new = torch.empty((n,) + obs.shape[2:], dtype=torch.uint8, device=dev)
            # stack state such that the first push yields the reset observation
            init = torch.from_numpy(np.ascontiguousarray(obs))
            (self.buf_obs[T - 1] if self.band else self.s_obs)[:, 1:].copy_(init[:, :3].to(dev))
            self.h_new.copy_(init[:, 3])
            # K19 reads the newest frames straight from pinned host memory (zero-copy over the host
            # link) when the pinned buffer is device-mapped: no separate H2D blit per step
            self.h_new_dev = 0
            try:
                from ray_memory_management_amd._native import require_hip

                self.h_new_dev = int(require_hip().host_device_pointer(self.h_new.data_ptr()))
            except Exception:
                self.h_new_dev = 0
        # K16 can store the sampled actions straight into the pinned action buffer (device-mapped):
        # the CPU env reads them after the step's event, no D2H blit
        self.h_act_dev = 0
        if self.fused:
            try:
                from ray_memory_management_amd._native import require_hip

                self.h_act_dev = int(require_hip().host_device_pointer(self.h_act.data_ptr()))
            except Exception:
                self.h_act_dev = 0
        # K19 folded into the K10 trunk launch (push mode); RMM_NO_FOLD_PUSH=1 keeps the separate kernel
        self.fold_push = os.environ.get("RMM_NO_FOLD_PUSH") is None
        # step gate (graphs only, opt-in RMM_ROLLOUT_GATE=1): step t+1 is enqueued before step t's CPU
        # env step and held by a device-side gate until the host releases it, so the graph launch
        # overlaps the env step. Measured SLOWER on MI355X (runtime PPO 17.4 -> 18.5 ms/iter,
        # profiles/rollout_push_r3.txt): the gate node + host-memory polling cost more than the
        # launch latency it hides.
        self.gate = False
        self.h_release = torch.zeros(1, dtype=torch.int64).pin_memory()
        self._rel = self.h_release.numpy()
        self.h_release_dev = 0
        try:
            from ray_memory_management_amd._native import require_hip

            self.h_release_dev = int(require_hip().host_device_pointer(self.h_release.data_ptr()))
        except Exception:
            self.h_release_dev = 0
        self.dev_seq = torch.zeros(1, dtype=torch.int64, device=dev)
        self.gate_err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = None
        self.ep_len = np.zeros(n, dtype=np.int64)
        self.ep_rew = np.zeros(n, dtype=np.float64)

    def policy_step(self):
        """H2D obs → frame row t → fused policy step (row t of the device buffers) → D2H actions."""
        import torch

        from ray_memory_management_amd._native import require_hip

        t, ctr = self.ctr_t[1:2], self.ctr_t[0:1]
        if self.gate:
            require_hip().step_gate(self.h_release_dev, self.dev_seq.data_ptr(), 200000, self.gate_err.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
        push = None
        if self.device_stack:
            src = self.h_new_dev
            if not src:
                self.s_new.copy_(self.h_new, non_blocking=True)
                src = self.s_new.data_ptr()
            if self.band:
                push = (src, self.buf_obs, "rows")  # K10 reads row t-1 + new frames, stores row t
            elif self.fused and self.fold_push and (self.model.fused_trunk_ok(self.s_obs)
                                                    or getattr(self.model, "fused_x3_ok", lambda o: False)(self.s_obs)):
                push = (src, self.buf_obs)  # K10 shifts the stack and stores row t itself
            else:
                require_hip().frame_push(self.s_obs.data_ptr(), src, self.buf_obs.data_ptr(),
                                         t.data_ptr(), self.n, self.hw, torch.cuda.current_stream().cuda_stream)
        else:
            self.s_obs.copy_(self.h_obs, non_blocking=True)
            self.buf_obs.index_copy_(0, t, self.s_obs.unsqueeze(0))
        direct = bool(self.fused and self.h_act_dev)
        advanced = bool(self.fused and self.model.forward_sample(self.s_obs, t, ctr, self.seed, self.buf_act,
                                                                 self.buf_logp, self.buf_vf, self.buf_logits,
                                                                 self.h_act_dev if direct else self.act_now,
                                                                 done=self.k16_done, push=push))
        if not advanced:
            direct = False
            hd = self.model.forward_heads(self.s_obs)
            lp, vp, ld = hd.data_ptr(), hd.data_ptr() + self.A * hd.element_size(), hd.stride(0)
            bf = hd.dtype == torch.bfloat16
            require_hip().sample_store(lp, bf, vp, bf, t.data_ptr(), ctr.data_ptr(), self.seed,
                                       self.buf_act.data_ptr(), self.buf_logp.data_ptr(), self.buf_vf.data_ptr(),
                                       self.buf_logits.data_ptr(), self.act_now.data_ptr(), self.n, self.A,
                                       torch.cuda.current_stream().cuda_stream, ldl=ld, ldv=ld)
        if not direct:
            self.h_act.copy_(self.act_now, non_blocking=True)
        if not (advanced and self.k16_done is not None):  # else K16 advanced the counters itself
            self.ctr_t.add_(1)

    def release(self):
        """Open the device-side gate of the next enqueued step (its frames are written)."""
        self._rel[0] += 1

    def resync(self, stream):
        """Align the host release counter with the device gate sequence (fragment start: a gated
        step abandoned by an exception has consumed a sequence number on its bounded timeout)."""
        if self.gate:
            stream.synchronize()
            self._rel[0] = int(self.dev_seq.item())
            if int(self.gate_err.item()):
                self.gate_err.zero_()
                raise RuntimeError("rollout step gate timed out (a policy step ran without its frames)")

    def capture(self, stream):
        import torch

        self.gate = bool(self.h_release_dev) and os.environ.get("RMM_ROLLOUT_GATE", "0") != "0"
        with torch.cuda.stream(stream):
            saved = self.s_obs.clone() if self.device_stack else None
            saved_ctr = self.ctr_t.clone()  # a capture has no effect on the sampling stream
            for _ in range(2):
                # the warm-up steps write rollout row *t: a recapture after a fragment (parameters
                # rebound, e.g. zero-copy shared weights) finds t == T there, and rows T, T+1 lie past
                # the end of the rollout buffers (the K10 push stores a whole frame row: the GPU
                # memory fault of the round-3/4 shared-weights runs, profiles/shared_weights_r4.txt)
                self.ctr_t[1].zero_()
                self.release()
                self.policy_step()
            self.ctr_t.copy_(saved_ctr)
            self.ctr_t[1].zero_()
            if saved is not None:  # warm-up pushes must not advance the frame stacks
                self.s_obs.copy_(saved)
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            self.policy_step()
        self.graph = g

    def launch(self, stream, current: bool = False):
        """Enqueue one policy step on `stream` (graph replay launches on the current stream) and
        return an event that completes with the action store. With ``current=True`` the caller has
        already made `stream` current (the rollout loop does, once per fragment). The group reuses
        ONE event: the previous step's event has been waited on before the next launch."""
        import torch

        ev = getattr(self, "_ev", None)
        if ev is None:
            ev = self._ev = torch.cuda.Event()
        if current:
            self.graph.replay() if self.graph else self.policy_step()
            ev.record(stream)
            return ev
        with torch.cuda.stream(stream):
            if self.graph:
                self.graph.replay()
            else:
                self.policy_step()
            ev.record(stream)
        return ev

    def env_step(self, t: int, completed: list):
        v = getattr(self, "_np", None)
        if v is None:  # numpy views of the pinned staging buffers, made once
            v = self._np = {"act": self.h_act.numpy(), "rew": self.h_rew.numpy(), "done": self.h_done.numpy(),
                            "obs": self.h_obs.numpy(),
                            "new": self.h_new.numpy() if self.device_stack else None}
        if self.device_stack:
            rew, done = self.env.vector_step_frames(v["act"].copy(), v["new"])
        else:
            obs, rew, done = self.env.vector_step(v["act"].copy())
            v["obs"][:] = obs
        v["rew"][t] = rew
        v["done"][t] = done
        self.ep_rew += rew
        self.ep_len += 1
        if done.any():
            for i in np.nonzero(done)[0]:
                completed.append((float(self.ep_rew[i]), int(self.ep_len[i])))
                self.ep_rew[i] = 0.0
                self.ep_len[i] = 0


class HybridRolloutWorker(GPURolloutWorker):
    """CPU rollout worker whose env steps on the CPU and whose policy runs on its (fractional) GPU.

    Role parity: reference rllib/evaluation/rollout_worker.py with ``num_gpus_per_worker > 0`` and
    a CPU env (the policy is placed on the worker's GPU). MI355X design: each env step is ONE
    HIP-graph replay — pinned-host → HBM observation copy, frame row store, K10 trunk → K13 dense →
    K16 heads + Gumbel sampling + rollout-row stores, action copy back to pinned host. The envs
    are split into two groups that are double-buffered: while the GPU runs group A's policy step
    the CPU steps group B's envs and vice versa, so env time and inference latency overlap. The
    frames each step uploads stay in HBM as the fragment's observation rows, so the fragment is
    returned as CUDA tensors (``pack_fragment_device``): it lands in this process's HBM object store
    and the learner on the same GPU reads it zero-copy via hipIPC.
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
        n = int(self.config.get("num_envs_per_worker", 1))
        # double-buffered env groups hide a SLOW env step behind the other group's policy step. With
        # the native env core the env step is a few µs and the native loop runs, so one group (one
        # policy step of all n envs per env step) is faster: runtime PPO 15.4-15.9 vs 17.5-19.7
        # ms/iter on MI355X (profiles/native_rollout_r3.txt). "auto" (default) = split only envs
        # without a native core.
        dbl = self.config.get("rollout_double_buffer", "auto")
        if os.environ.get("RMM_ROLLOUT_DOUBLE_BUFFER") is not None:  # A/B override
            dbl = os.environ["RMM_ROLLOUT_DOUBLE_BUFFER"] != "0"
        from ray_memory_management_amd._private.numa import pin_to_gpu

        # the env loop thread, the native envs' memory and the pinned frame / completion buffers (all
        # allocated below) on the GPU's socket
        self.cpu_affinity = pin_to_gpu(0)
        first = make_vector_env(self.config.get("env"), n, {**ec, "seed": s * 7})
        if dbl == "auto":
            dbl = getattr(first, "_native", None) is None or os.environ.get("RMM_NO_NATIVE_ROLLOUT") is not None
        groups = 2 if n >= 2 and dbl else 1
        sizes = [n // groups + (1 if g < n % groups else 0) for g in range(groups)]
        envs = [first if groups == 1 else make_vector_env(self.config.get("env"), k, {**ec, "seed": s * 7 + g})
                for g, k in enumerate(sizes)]
        if any(e is None for e in envs):
            raise ValueError("HybridRolloutWorker needs a native CPU vector env")
        self.env = envs[0]
        torch.set_num_threads(1)
        self.device = torch.device("cuda:0")
        torch.cuda.set_device(0)
        torch.manual_seed(s)
        model = build_model(self.env.observation_space, self.env.action_space, self.config.get("model") or {})
        cdt = torch.float32 if str(self.config.get("compute_dtype", "bf16")) in ("fp32", "float32") else torch.bfloat16
        self.model = model.to(self.device).to(cdt).to(memory_format=torch.channels_last)
        _init_x3(self.model)
        self.T = int(self.config.get("rollout_fragment_length", 200))
        self.n = n
        probe = torch.zeros((1,) + tuple(np.asarray(self.env.vector_reset()).shape[1:]), dtype=torch.uint8,
                            device=self.device)
        with torch.no_grad():
            self.A = int(self.model(probe)[0].shape[-1])
        self.groups = [_EnvGroup(e, self.model, self.T, self.A, self.device, (s * 131 + g) & 0x7FFFFFFF)
                       for g, e in enumerate(envs)]
        self.stream = torch.cuda.Stream(self.device)
        # optional stream per env group (group A's policy step may run concurrently with group B's).
        # Off by default: measured no gain in the worker probe (profiles/hybrid_group_streams.txt)
        gs = self.config.get("rollout_group_streams", os.environ.get("RMM_GROUP_STREAMS", "0") != "0")
        self.group_streams = ([torch.cuda.Stream(self.device) for _ in self.groups] if gs and len(self.groups) > 1
                              else [self.stream] * len(self.groups))
        # HIP-graph replay per policy step (default) or eager launches (rollout_graphs=False)
        self._captured = not self.config.get("rollout_graphs", os.environ.get("RMM_NO_ROLLOUT_GRAPH") is None)
        if self._captured:
            for g in self.groups:
                g.graph = False
        self._completed: List[tuple] = []
        self._sample_time = 0.0

    def sample(self, *_after):  # _after: refs the runtime resolves first (prefetched samples)
        """One fragment. A step-gate timeout (the host stalled longer than `rollout_gate_timeout_ms`
        between a launch and its release, so a gated policy step read stale frames) never fails the
        iteration: that fragment is discarded and re-sampled once on the ungated path."""
        try:
            return self._sample_once()
        except _GateTimeout:
            self.gate_timeouts = getattr(self, "gate_timeouts", 0) + 1
            self._gate_bypass = True
            try:
                return self._sample_once()
            finally:
                self._gate_bypass = False

    def _sample_once(self):
        import time

        import torch

        from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment_device

        t0 = time.perf_counter()
        stamps = getattr(self, "_stamps", None)
        if stamps is not None:
            stamps.append(("sample_start", time.time()))
        G, T, st = self.groups, self.T, self.stream
        with torch.no_grad():
            S = self.group_streams
            dbg = os.environ.get("RMM_CAPTURE_DEBUG")
            if not self._captured:
                self._captured = True
                for g, gs in zip(G, S):
                    try:
                        g.capture(gs)
                    except Exception as e:  # pragma: no cover
                        print(f"[HybridRolloutWorker] HIP graph capture failed ({e!r}); running eagerly")
                        g.graph = False
                if dbg:
                    import sys

                    torch.cuda.synchronize(self.device)
                    print(f"[hybrid-worker pid {os.getpid()}] policy-step graphs captured ok", file=sys.stderr,
                          flush=True)
            # the previous fragment's frames (views of the group buffers) were copied into the HBM
            # object store on the default stream at task return: finish that before overwriting
            cur = torch.cuda.current_stream(self.device)
            for gs in dict.fromkeys(S):
                gs.wait_stream(cur)
            for g, gs in zip(G, S):
                with torch.cuda.stream(gs):
                    g.ctr_t[1].zero_()
                g.resync(gs)
            shared = all(gs is st for gs in S)
            server = self._server_args(G, S)
            direct = None if server is not None else self._direct_args(G, S)
            native = None if (server is not None or direct is not None) else self._native_loop(G, S)
            if direct is not None:  # the native loop, launching the step's kernels directly
                from ray_memory_management_amd._native import require_hip

                th = int(os.environ.get("RMM_ENV_THREADS") or self.config.get("rollout_env_threads", 1) or 1)
                spin = os.environ.get("RMM_NATIVE_SPIN", "0") == "1"
                self._completed.extend(require_hip().hybrid_rollout_direct(**direct, T=T, threads=max(1, th),
                                                                          spin=spin))
                if "gate_err" in direct and int(self._gate_err.item()):
                    self._gate_err.zero_()  # a gated step gave up waiting: it ran on stale frames
                    raise _GateTimeout("rollout step gate timed out during this fragment; fragment discarded")
            elif server is not None:  # K21: the whole fragment in ONE persistent kernel launch
                from ray_memory_management_amd._native import require_hip

                th = int(os.environ.get("RMM_ENV_THREADS") or self.config.get("rollout_env_threads", 1) or 1)
                try:
                    self._completed.extend(require_hip().hybrid_rollout_server(**server, T=T, threads=max(1, th)))
                except RuntimeError:
                    # a server timeout (e.g. another process held the CUs) aborts this fragment; the
                    # worker falls back to the per-step graph loop for good
                    self._server_off = True
                    raise
            elif native is not None:  # the whole T-step loop in C++ (csrc/hip/rollout_loop.cc)
                from ray_memory_management_amd._native import require_hip

                # rollout_env_threads (default 1) splits each env step over that many CPU threads; measured
                # neutral for the synthetic env (profiles/native_rollout_r3.txt); RMM_ENV_THREADS overrides
                th = int(os.environ.get("RMM_ENV_THREADS") or self.config.get("rollout_env_threads", 1) or 1)
                # blocking event waits by default: a bounded poll was faster on an idle host but gave
                # outliers when the host's CPUs were shared (profiles/native_rollout_r3.txt)
                spin = os.environ.get("RMM_NATIVE_SPIN", "0") == "1"
                self._completed.extend(require_hip().hybrid_rollout(native, T, threads=max(1, th), spin=spin))
            else:
                self._python_loop(G, S, T, st, shared)
            if dbg:
                import sys

                torch.cuda.synchronize(self.device)
                print(f"[hybrid-worker pid {os.getpid()}] fragment loop ok", file=sys.stderr, flush=True)
            t_loop = time.perf_counter()
            self._loop_time = getattr(self, "_loop_time", 0.0) + (t_loop - t0)
            with torch.cuda.stream(st):
                for gs in dict.fromkeys(S):
                    if gs is not st:
                        st.wait_stream(gs)
                parts = []
                for g in G:
                    if g.device_stack:  # observation after the last env step (pushed next fragment)
                        g.s_new.copy_(g.h_new, non_blocking=True)
                        stack = g.buf_obs[T - 1] if g.band else g.s_obs  # the last step's frame stack
                        last_v = bootstrap_value(self.model, torch.cat([stack[:, 1:], g.s_new.unsqueeze(1)], dim=1))
                    else:
                        g.s_obs.copy_(g.h_obs, non_blocking=True)
                        last_v = bootstrap_value(self.model, g.s_obs)
                    parts.append((g.buf_obs, g.buf_logits, g.buf_logp, g.buf_vf,
                                  g.h_rew.to(self.device, non_blocking=True),
                                  g.h_done.to(self.device, non_blocking=True), g.buf_act, last_v.reshape(-1)))
                if len(parts) == 1:
                    frag = pack_fragment_device(*parts[0])
                else:  # time-major [T, n]: the groups' env columns side by side
                    cat = [torch.cat(xs, dim=0 if k == 7 else 1) for k, xs in enumerate(zip(*parts))]
                    frag = pack_fragment_device(*cat)
            st.synchronize()
            for g in G:  # a gated step that timed out ran on stale frames: never hand that fragment out
                if g.gate and int(g.gate_err.item()):
                    g.gate_err.zero_()
                    raise RuntimeError("rollout step gate timed out during this fragment (a policy step ran "
                                       "without its frames); fragment discarded")
        self._sample_time += time.perf_counter() - t0
        if stamps is not None:
            stamps.append(("sample_end", time.time()))
        return frag

    def phase_stamps(self, on: bool = True):
        """Wall-clock (start, end) stamps of every sample() from now on (hand-off latency probes); returns
        and clears the stamps recorded so far."""
        from ray_memory_management_amd._private import worker as _w

        cw = _w.global_worker
        out = (getattr(self, "_stamps", None) or []) + [("task",) + t for t in (getattr(cw, "task_stamps", None) or [])]
        self._stamps = [] if on else None
        if cw is not None:
            cw.task_stamps = [] if on else None
        return out

    def _server_args(self, G, S):
        """Arguments of the K21 persistent rollout server (csrc/hip/rollout_server.hip) for this
        worker, or None when it does not apply: opt-in (RMM_ROLLOUT_SERVER=1 or config
        rollout_server=True), one env group of <= 64 native synthetic envs with device frame stacks
        (not band mode), the fused bf16 Nature-CNN policy, device-mapped pinned frame / action
        buffers. One launch per fragment; bit-identical to the per-step graph loop."""
        if getattr(self, "_server_off", False) or os.environ.get("RMM_NO_NATIVE_ROLLOUT"):
            return None
        on = os.environ.get("RMM_ROLLOUT_SERVER")
        if not (on == "1" if on is not None else bool(self.config.get("rollout_server", False))):
            return None
        k = self._kernel_args(G, S)
        if k is None or k.get("x3"):
            return None
        return {key: v for key, v in k.items() if key != "x3"}

    def _direct_args(self, G, S):
        """Arguments of the native loop with DIRECT kernel launches per policy step (K10 push → K13s →
        K16, rollout_loop.cc:rollout_step_direct) instead of a HIP-graph launch; same conditions as
        the server. Default on (RMM_ROLLOUT_DIRECT=0 or config rollout_direct=False: graph launches):
        a 3-kernel graph launch cost more host time than the three launches, 48-49 -> 43-44 µs per
        50-env step, runtime bench 351k -> 370k samples/s (profiles/rollout_direct_r4.txt)."""
        if os.environ.get("RMM_NO_NATIVE_ROLLOUT") or os.environ.get("RMM_ROLLOUT_SPIN", "0") != "0":
            return None
        on = os.environ.get("RMM_ROLLOUT_DIRECT")
        if not (on == "1" if on is not None else bool(self.config.get("rollout_direct", True))):
            return None
        if any(g.gate for g in G):  # the step gate lives in the captured graph
            return None
        k = self._kernel_args(G, S)
        if k is None or G[0].k16_done is None:
            return None
        out = dict(group=k["group"], weights=k["weights"], w1s=k["w1s"], w2s=k["w2s"],
                   bufs=k["bufs"][:12] if k.get("x3") else k["bufs"][:11],
                   B=k["B"], S=k["S"], A1=k["A1"], seed=k["seed"], k16_done=G[0].k16_done.data_ptr())
        if k.get("x3") and int(k["B"]) <= 64 and G[0].k16_done.numel() >= 1 + (int(k["B"]) + 15) // 16 and \
                os.environ.get("RMM_ROLLOUT_FUSED_HEADS", "0") == "1":
            out["fused_heads"] = True  # K13x + K16x in one launch (x3_dense_heads_sample)
        if os.environ.get("RMM_ROLLOUT_SEQ", "1") != "0":
            # completion word: K16 stores row + 1 into mapped pinned memory, the loop polls it (no event
            # record / interrupt wake-up): 44-47 -> 41-42 µs per 50-env step, runtime bench +2%
            # (profiles/rollout_direct_r4.txt); RMM_ROLLOUT_SEQ=0 waits on events
            if getattr(self, "_h_seq", None) is None:
                import torch

                from ray_memory_management_amd._native import require_hip

                self._h_seq = torch.zeros(1, dtype=torch.int64).pin_memory()
                self._h_seq_dev = int(require_hip().host_device_pointer(self._h_seq.data_ptr()))
            if self._h_seq_dev:
                out.update(host_seq=self._h_seq.data_ptr(), host_seq_dev=self._h_seq_dev)
        if k.get("x3") and os.environ.get("RMM_ROLLOUT_DIRECT_GATE", "1") != "0" and not getattr(self, "_gate_bypass", False):
            # in-kernel step gate (fp32 policy): step t+1 is launched before step t's env step and K10x
            # waits for the host's release counter before reading the new frames, so the three launches
            # leave the step's critical path
            if getattr(self, "_h_rel", None) is None:
                import torch

                from ray_memory_management_amd._native import require_hip

                self._h_rel = torch.zeros(1, dtype=torch.int64).pin_memory()
                self._h_rel_dev = int(require_hip().host_device_pointer(self._h_rel.data_ptr()))
                self._gate_err = torch.zeros(1, dtype=torch.int32, device=self.device)
            if self._h_rel_dev:
                # the envs are stepped in `parts` ranges, each released as soon as its frames are written
                # (K10x workgroup b waits for its own range): the first frames cross PCIe while the rest
                # are stepped. RMM_ROLLOUT_GATE_PARTS=1: one release after the whole env step
                parts = int(os.environ.get("RMM_ROLLOUT_GATE_PARTS", "10"))
                tmo = int(os.environ.get("RMM_ROLLOUT_GATE_TIMEOUT_MS") or self.config.get("rollout_gate_timeout_ms", 2000))
                out.update(release=self._h_rel.data_ptr(), release_dev=self._h_rel_dev,
                           gate_err=self._gate_err.data_ptr(), gate_parts=max(1, min(parts, int(k["B"]))),
                           gate_timeout_ms=max(1, tmo))
        return out

    def _kernel_args(self, G, S):
        """Weights / buffers / strides of the fused rollout step for one native env group (shared by
        the K21 server and the direct-launch loop), or None when the group does not qualify."""
        cached = getattr(self, "_server_cache", None)
        if cached is not None:
            return cached
        import torch

        from ray_memory_management_amd._native import require_hip

        if len(G) != 1:
            return None
        g, gs = G[0], S[0]
        m = self.model
        x3 = bool(getattr(m, "fused_x3_ok", lambda o: False)(g.s_obs))  # fp32 policy: split-bf16 kernels
        ok = (g.device_stack and not g.band and g.fused and g.h_new_dev and g.h_act_dev and g.n <= 64
              and getattr(g.env, "_native", None) is not None and hasattr(g.env, "native_state")
              and getattr(m, "nature", False) and (m.fused_trunk_ok(g.s_obs) or x3) and m.dense_tail is not None
              and m.dense_tail.out_features == 256 and m.dense_tail.in_features == 3872
              and m.dense_tail.weight.is_contiguous() and m.heads.weight.is_contiguous()
              and 3 <= m.heads.out_features <= 16)
        if not ok:
            return None
        hip = require_hip()
        B, A1 = g.n, m.heads.out_features
        c1, c2, dl, hd = m.convs[0], m.convs[1], m.dense_tail, m.heads
        group = [0, int(gs.cuda_stream), *map(int, g.env.native_state()), g.h_act.data_ptr(), g.h_new.data_ptr(),
                 g.h_rew.data_ptr(), g.h_done.data_ptr(), g.ep_rew.ctypes.data, g.ep_len.ctypes.data]
        if x3:
            from ray_memory_management_amd.ops import x3 as X3

            P = m.x3_pairs()
            S_ = hip.x3_dense_fwd_part_slices(B, 3872, 256)
            self._server_h2 = X3.Pair.empty((B, 3872), self.device)
            h2_hi, h2_lo = self._server_h2.hi.data_ptr(), self._server_h2.lo.data_ptr()
            weights = ([P[n].hi.data_ptr() for n in m._X3_NAMES] + [P[n].lo.data_ptr() for n in m._X3_NAMES])
        else:
            S_ = hip.dense_fwd_part_slices(B, 3872, 256)
            self._server_h2 = torch.empty((B, 3872), dtype=torch.bfloat16, device=self.device)
            h2_hi, h2_lo = self._server_h2.data_ptr(), 0
            weights = [c1.weight.data_ptr(), c1.bias.data_ptr(), c2.weight.data_ptr(), c2.bias.data_ptr(),
                       dl.weight.data_ptr(), dl.bias.data_ptr(), hd.weight.data_ptr(), hd.bias.data_ptr()]
        self._server_hpart = torch.empty(S_ * B * 256, dtype=torch.float32, device=self.device)
        bufs = [g.s_obs.data_ptr(), int(g.h_new_dev), g.buf_obs.data_ptr(), h2_hi,
                self._server_hpart.data_ptr(), g.buf_act.data_ptr(), g.buf_logp.data_ptr(), g.buf_vf.data_ptr(),
                g.buf_logits.data_ptr(), int(g.h_act_dev), g.ctr_t.data_ptr()]
        if x3:
            bufs.append(h2_lo)
        if os.environ.get("RMM_ROLLOUT_SERVER_PROF"):  # per-step phase stamps of workgroup 0 (probe)
            self._server_prof = torch.zeros((self.T, 5), dtype=torch.int64, device=self.device)
            bufs.append(self._server_prof.data_ptr())
        # grid: 128 workgroups by default (phase B's 512 K13s units in two passes; fewer workgroups
        # than CUs keeps barrier arrivals cheap and leaves CUs to other processes); RMM_ROLLOUT_SERVER_WGS
        wgs = int(os.environ.get("RMM_ROLLOUT_SERVER_WGS", "128"))
        self._server_cache = dict(group=group, weights=weights, w1s=list(c1.weight.stride()),
                                  w2s=list(c2.weight.stride()), bufs=bufs, B=B, S=S_, A1=A1, seed=int(g.seed),
                                  workgroups=max(wgs, B), x3=x3)
        return self._server_cache

    def _native_loop(self, G, S):
        """Per-group descriptors for the native rollout loop (csrc/hip/rollout_loop.cc), or None when
        a group needs the Python loop: the env must be the native synthetic vector env, the policy
        step a captured HIP graph reading the newest frames from mapped pinned memory and storing the
        actions into it (K10 push mode + K16 direct store); with the step gate (RMM_ROLLOUT_GATE=1)
        step t+1 is launched before step t's env step and released after it. RMM_NO_NATIVE_ROLLOUT=1
        forces the Python loop."""
        if os.environ.get("RMM_NO_NATIVE_ROLLOUT") or os.environ.get("RMM_ROLLOUT_SPIN", "0") != "0":
            return None
        cached = getattr(self, "_native_desc", None)
        if cached is not None:
            return cached
        desc = []
        for g, gs in zip(G, S):
            ok = (g.graph not in (None, False) and g.device_stack and g.h_new_dev and g.fused
                  and g.h_act_dev and getattr(g.env, "_native", None) is not None
                  and hasattr(g.env, "native_state") and hasattr(g.graph, "raw_cuda_graph_exec"))
            if not ok:
                return None
            desc.append([int(g.graph.raw_cuda_graph_exec()), int(gs.cuda_stream), *map(int, g.env.native_state()),
                         g.h_act.data_ptr(), g.h_new.data_ptr(), g.h_rew.data_ptr(), g.h_done.data_ptr(),
                         g.ep_rew.ctypes.data, g.ep_len.ctypes.data, g.h_release.data_ptr() if g.gate else 0])
        self._native_desc = desc
        return desc

    def _python_loop(self, G, S, T, st, shared):
        """The rollout loop in Python (any vector env; also the step-gate / event-polling variants)."""
        import torch

        with torch.cuda.stream(st):  # one stream switch per fragment (per launch with group streams)
            try:
                evs = []
                for g, gs in zip(G, S):
                    torch.cuda.set_stream(gs)
                    evs.append(g.launch(gs, current=True))
                    if g.gate:
                        g.release()  # step 0's frames are already staged
                # RMM_ROLLOUT_SPIN=1: poll each step's event instead of a blocking wait (measured no gain)
                spin = os.environ.get("RMM_ROLLOUT_SPIN", "0") != "0"
                for t in range(T):
                    for i, g in enumerate(G):  # group i's env step overlaps the other group's inference
                        if spin:  # poll the event: no blocking-wait wake-up latency on the step's critical path
                            ev = evs[i]
                            while not ev.query():
                                pass
                        else:
                            evs[i].synchronize()
                        if g.gate:  # enqueue step t+1 first; it waits on the device for release()
                            if t + 1 < T:
                                if not shared:
                                    torch.cuda.set_stream(S[i])
                                evs[i] = g.launch(S[i], current=True)
                            g.env_step(t, self._completed)
                            if t + 1 < T:
                                g.release()
                            continue
                        g.env_step(t, self._completed)
                        if t + 1 < T:
                            if not shared:
                                torch.cuda.set_stream(S[i])
                            evs[i] = g.launch(S[i], current=True)
            finally:
                torch.cuda.set_stream(st)

    def set_weights(self, weights, global_vars=None):
        import time

        import torch

        t0 = time.perf_counter()
        self.stream.synchronize()
        super().set_weights(weights, global_vars)
        torch.cuda.synchronize(self.device)
        self._set_weights_time = getattr(self, "_set_weights_time", 0.0) + time.perf_counter() - t0

    def _on_params_rebound(self):
        """Parameters now alias the learner's HBM weights: recapture the policy-step graphs (and the
        native loop's graph handles) at the next sample."""
        self._captured = False
        self._native_desc = None
        self._server_cache = None

    def timing(self):
        """Accumulated seconds in sample() and set_weights() (phase breakdown probes)."""
        return {"sample_s": self._sample_time, "set_weights_s": getattr(self, "_set_weights_time", 0.0),
                "loop_s": getattr(self, "_loop_time", 0.0)}
