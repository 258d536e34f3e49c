"""RolloutWorker. Parity: reference rllib/evaluation/rollout_worker.py + sampler.py
(SyncSampler; batch_mode truncate_episodes / complete_episodes) + metrics.py (episode reward /
length stats) + postprocessing.py (GAE with bootstrapped value on truncation).

A worker steps `num_envs_per_worker` copies of the env in lock-step (one batched policy forward
per step), writes time-major buffers, then postprocesses the whole fragment with ONE GAE call.
"""
from __future__ import annotations

import time
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ray_memory_management_amd.rllib.env import VectorEnv, make_env, make_vector_env
from ray_memory_management_amd.rllib.policy import TorchPolicy, compute_gae_for_trajectories
from ray_memory_management_amd.rllib.sample_batch import SampleBatch, concat_samples


def unpack_flat_weights(weights: Dict) -> Dict:
    """A learner actor's flat bf16 weight publication ({'__rmm_flat_bf16__': flat, '__rmm_layout__':
    [(name, offset, shape, stride)]}, LearnerActor.get_weights_device) → per-parameter fp32 CPU
    tensors, for rollout workers that run the policy on the CPU."""
    import torch

    flat = weights["__rmm_flat_bf16__"]
    flat = flat.detach().to("cpu", torch.float32) if isinstance(flat, torch.Tensor) else \
        torch.as_tensor(np.asarray(flat)).float()
    return {name: flat.as_strided(tuple(shape), tuple(stride), int(off)).contiguous()
            for name, off, shape, stride in weights["__rmm_layout__"]}


class _FlattenObsVectorEnv:
    """Dict / Tuple observations → flat float32 vectors at the env boundary (the reference's
    preprocessor step in the sampler), so every sampling path handles plain [n, N] arrays; the
    observation space stays the composite one for the model (ComplexInputNetwork restores it)."""

    def __init__(self, env):
        from ray_memory_management_amd.rllib.modelv2 import flatten_observation

        self._env, self._flat = env, flatten_observation
        self.num_envs = env.num_envs
        self.observation_space, self.action_space = env.observation_space, env.action_space

    def _f(self, o):
        return self._flat(self.observation_space, o)

    def vector_reset(self):
        return [self._f(o) for o in self._env.vector_reset()]

    def reset_at(self, i):
        return self._f(self._env.reset_at(i))

    def vector_step(self, actions):
        obs, rew, done, info = self._env.vector_step(actions)
        return [self._f(o) for o in obs], rew, done, info

    def __getattr__(self, k):
        return getattr(self._env, k)


class RolloutWorker:
    def __init__(self, env_creator=None, config: Optional[Dict] = None, worker_index: int = 0,
                 num_workers: int = 0, policy_config: Optional[Dict] = None, seed: Optional[int] = None):
        self.config = dict(config or {})
        # policies see their worker's slot (per-worker exploration, e.g. Ape-X epsilons)
        self.config["worker_index"], self.config["num_workers"] = worker_index, num_workers
        self.worker_index = worker_index
        self.num_workers = num_workers
        env = self.config.get("env")
        env_config = dict(self.config.get("env_config") or {})
        n_envs = int(self.config.get("num_envs_per_worker", 1))
        base_seed = seed if seed is not None else self.config.get("seed")

        def mk(i):
            e = env_creator(env_config) if env_creator is not None else make_env(env, env_config)
            if base_seed is not None and hasattr(e, "reset"):
                try:
                    e.reset(seed=int(base_seed) * 1000 + worker_index * 100 + i)
                except TypeError:
                    pass
            return e

        import torch

        # rollout workers are single-threaded CPU processes by default (num_cpus_per_worker)
        torch.set_num_threads(max(1, int(self.config.get("num_cpus_per_worker", 1) or 1)))
        vcfg = dict(env_config)
        if base_seed is not None:
            vcfg.setdefault("seed", int(base_seed) * 1000 + worker_index)
        self.vec_env = None if env_creator is not None else make_vector_env(env, n_envs, vcfg)
        self.env = self.vec_env if self.vec_env is not None else VectorEnv(mk, n_envs)
        if hasattr(self.env.observation_space, "spaces"):
            self.env = _FlattenObsVectorEnv(self.env)
        pcls = self.config.get("policy_class") or TorchPolicy
        if isinstance(pcls, str):
            import importlib

            mod, _, name = pcls.rpartition(".")
            pcls = getattr(importlib.import_module(mod), name)
        self.policy = pcls(self.env.observation_space, self.env.action_space, self.config, device="cpu")
        if base_seed is not None:
            torch.manual_seed(int(base_seed) + worker_index)
        self._obs = self.env.vector_reset()
        self._ep_reward = np.zeros(n_envs)
        self._ep_len = np.zeros(n_envs, dtype=np.int64)
        self._completed: List[tuple] = []
        self._sample_time = 0.0
        cb = self.config.get("callbacks")
        self.callbacks = cb() if cb is not None else None
        self._episodes: Dict[int, Any] = {}
        self._custom_metrics: Dict[str, List[float]] = {}
        # offline IO (reference rllib/offline + rollout_worker input_creator / output_creator)
        self.output_writer = None
        out = self.config.get("output")
        if out:
            from ray_memory_management_amd.rllib.offline import JsonWriter

            self.output_writer = JsonWriter(out, self.config.get("output_max_file_size", 64 << 20),
                                            self.config.get("output_compress_columns", ("obs", "new_obs")),
                                            worker_index)
        self.input_reader = None
        inp = self.config.get("input", "sampler")
        if callable(inp):  # input creator(ioctx) -> InputReader (e.g. PolicyServerInput)
            from ray_memory_management_amd.rllib.offline import IOContext

            self.input_reader = inp(IOContext(config=self.config, worker_index=worker_index, worker=self))
        elif inp and inp != "sampler":
            from ray_memory_management_amd.rllib.offline import JsonReader, ShuffledInput

            self.input_reader = ShuffledInput(JsonReader(inp, seed=base_seed),
                                              int(self.config.get("shuffle_buffer_size", 0) or 0), seed=base_seed)

    # ------------------------------------------------------------------ sampling
    def sample(self, *_after) -> SampleBatch:  # _after: refs resolved before it runs (prefetch)
        if self.input_reader is not None:  # offline data replaces the env sampler
            return self.input_reader.next()
        if getattr(self.policy.model, "is_recurrent", False):
            batch = self._sample_recurrent()
        else:
            batch = self._sample_vector() if self.vec_env is not None else self._sample_env()
        if self.output_writer is not None and "_raw" not in batch:
            self.output_writer.write(batch)
        return batch

    def _episode(self, i: int):
        """The callbacks' Episode object of env slot i (created on first use = episode start)."""
        ep = self._episodes.get(i)
        if ep is None:
            from ray_memory_management_amd.rllib.algorithms.callbacks import Episode

            ep = self._episodes[i] = Episode(int(self._eps[i]) if getattr(self, "_eps", None) is not None else i, i)
            self.callbacks.on_episode_start(worker=self, base_env=self.env, policies={"default_policy": self.policy},
                                            episode=ep, env_index=i)
        return ep

    def _end_episode(self, i: int):
        ep = self._episodes.pop(i, None)
        if ep is None:
            return
        self.callbacks.on_episode_end(worker=self, base_env=self.env, policies={"default_policy": self.policy},
                                      episode=ep, env_index=i)
        for k, v in ep.custom_metrics.items():
            self._custom_metrics.setdefault(k, []).append(float(v))

    def get_custom_metrics(self) -> Dict[str, List[float]]:
        out, self._custom_metrics = self._custom_metrics, {}
        return out

    def _sample_env(self) -> SampleBatch:
        t0 = time.perf_counter()
        T = int(self.config.get("rollout_fragment_length", 200))
        n = self.env.num_envs
        obs_buf, act_buf, logp_buf, vf_buf, logits_buf, rew_buf, done_buf = [], [], [], [], [], [], []
        nobs_buf = []
        eps_buf = []
        if getattr(self, "_eps", None) is None:  # per-env episode ids, unique across workers
            self._eps = np.arange(n, dtype=np.int64) + self.worker_index * (1 << 40)
            self._next_eps = int(self._eps[-1]) + 1
        for _ in range(T):
            obs = np.stack([np.asarray(o) for o in self._obs])
            eps_buf.append(self._eps.copy())
            a, _, extra = self.policy.compute_actions(obs, explore=self.config.get("explore", True))
            nobs, rew, done, _info = self.env.vector_step(list(a))
            nobs_buf.append(np.stack([np.asarray(o) for o in nobs]))  # before resets: terminal obs kept
            obs_buf.append(obs)
            act_buf.append(a)
            logp_buf.append(extra[SampleBatch.ACTION_LOGP])
            vf_buf.append(extra[SampleBatch.VF_PREDS])
            logits_buf.append(extra[SampleBatch.ACTION_DIST_INPUTS])
            rew_buf.append(np.asarray(rew, dtype=np.float32))
            done_buf.append(np.asarray(done, dtype=np.float32))
            self._ep_reward += np.asarray(rew, dtype=np.float64)
            self._ep_len += 1
            if self.callbacks is not None:
                for i in range(n):
                    ep = self._episode(i)
                    ep.length += 1
                    ep.total_reward += float(rew[i])
                    ep._last_obs, ep._last_action, ep._last_reward = nobs[i], a[i], float(rew[i])
                    self.callbacks.on_episode_step(worker=self, base_env=self.env,
                                                   policies={"default_policy": self.policy}, episode=ep, env_index=i)
                    if done[i]:
                        self._end_episode(i)
            for i in range(n):
                if done[i]:
                    self._completed.append((float(self._ep_reward[i]), int(self._ep_len[i])))
                    self._ep_reward[i] = 0.0
                    self._ep_len[i] = 0
                    nobs[i] = self.env.reset_at(i)
                    self._eps[i] = self._next_eps
                    self._next_eps += 1
            self._obs = nobs
        last_v = self.policy.value(np.stack([np.asarray(o) for o in self._obs]))
        rew = np.stack(rew_buf)
        vf = np.stack(vf_buf)
        dn = np.stack(done_buf)
        if not self.config.get("use_critic", True):  # PG: advantages = discounted returns, no baseline
            vf = np.zeros_like(vf)
            last_v = np.zeros_like(np.asarray(last_v))
        adv, ret = compute_gae_for_trajectories(rew, vf, dn, last_v, self.config.get("gamma", 0.99),
                                                self.config.get("lambda", self.config.get("lambda_", 1.0)))

        def flat(x):  # time-major [T, n, ...] -> env-major rows (each env's trajectory contiguous)
            x = np.asarray(x)
            return np.swapaxes(x, 0, 1).reshape((T * n,) + x.shape[2:])

        batch = SampleBatch({
            SampleBatch.OBS: flat(obs_buf), SampleBatch.ACTIONS: flat(act_buf),
            SampleBatch.ACTION_LOGP: flat(logp_buf).astype(np.float32), SampleBatch.VF_PREDS: flat(vf),
            SampleBatch.ACTION_DIST_INPUTS: flat(logits_buf).astype(np.float32), SampleBatch.REWARDS: flat(rew),
            SampleBatch.DONES: flat(dn), SampleBatch.NEXT_OBS: flat(nobs_buf), SampleBatch.EPS_ID: flat(eps_buf),
            SampleBatch.ADVANTAGES: flat(adv).astype(np.float32),
            SampleBatch.VALUE_TARGETS: flat(ret).astype(np.float32),
        })
        if self.callbacks is not None:
            self.callbacks.on_sample_end(worker=self, samples=batch)
        self._sample_time += time.perf_counter() - t0
        return batch

    def _sample_vector(self) -> SampleBatch:
        """Native vector env: whole-batch env steps, one batched policy forward per step, into
        preallocated time-major buffers. With ``postprocess_on_learner`` the fragment is returned
        packed for the learner's GPU ingest (K17: GAE + standardisation on the learner GPU);
        otherwise GAE runs here as in the reference's postprocess_trajectory."""
        import torch

        t0 = time.perf_counter()
        T = int(self.config.get("rollout_fragment_length", 200))
        n = self.env.num_envs
        obs0 = np.asarray(self._obs)
        bufs = getattr(self, "_vbufs", None)
        if bufs is None or bufs["obs"].shape[:2] != (T, n):
            A = getattr(self.env.action_space, "n", 1)
            bufs = self._vbufs = {
                "obs": np.empty((T, n) + obs0.shape[1:], dtype=obs0.dtype),
                "logits": np.empty((T, n, A), dtype=np.float32), "logp": np.empty((T, n), dtype=np.float32),
                "vf": np.empty((T, n), dtype=np.float32), "rew": np.empty((T, n), dtype=np.float32),
                "done": np.empty((T, n), dtype=np.float32), "act": np.empty((T, n), dtype=np.int64)}
        model = self.policy.model
        explore = self.config.get("explore", True)
        obs = obs0
        with torch.inference_mode():
            for t in range(T):
                bufs["obs"][t] = obs
                logits, v = model(torch.from_numpy(bufs["obs"][t]))
                logits = logits.float()
                lsm = torch.log_softmax(logits, dim=-1)
                if explore:  # Gumbel-max sampling of the categorical policy
                    g = -torch.log(-torch.log(torch.rand_like(logits).clamp_(1e-10, 1.0)))
                    a = torch.argmax(logits + g, dim=-1)
                else:
                    a = torch.argmax(logits, dim=-1)
                bufs["logits"][t] = logits.numpy()
                bufs["logp"][t] = lsm.gather(1, a.unsqueeze(1)).squeeze(1).numpy()
                bufs["vf"][t] = v.float().numpy()
                an = a.numpy()
                bufs["act"][t] = an
                obs, rew, done = self.env.vector_step(an)
                bufs["rew"][t] = rew
                bufs["done"][t] = done
                self._ep_reward += rew
                self._ep_len += 1
                if done.any():
                    for i in np.nonzero(done)[0]:
                        self._completed.append((float(self._ep_reward[i]), int(self._ep_len[i])))
                        self._ep_reward[i] = 0.0
                        self._ep_len[i] = 0
            _, last_v = model(torch.from_numpy(np.ascontiguousarray(obs)))
            last_v = last_v.float().numpy()
        self._obs = obs
        self.policy.global_timestep += T * n
        if self.config.get("postprocess_on_learner"):
            from ray_memory_management_amd.rllib.execution.sample_ingest import pack_fragment

            out = pack_fragment(bufs["obs"], bufs["logits"], bufs["logp"], bufs["vf"], bufs["rew"], bufs["done"],
                                bufs["act"], last_v)
        else:
            vfb = bufs["vf"] if self.config.get("use_critic", True) else np.zeros_like(bufs["vf"])
            if not self.config.get("use_critic", True):
                last_v = np.zeros_like(last_v)
            adv, ret = compute_gae_for_trajectories(bufs["rew"], vfb, bufs["done"], last_v,
                                                    self.config.get("gamma", 0.99),
                                                    self.config.get("lambda", self.config.get("lambda_", 1.0)))
            rows = T * n  # time-major rows (row = t*n + env)
            out = SampleBatch({
                SampleBatch.OBS: bufs["obs"].reshape((rows,) + obs0.shape[1:]).copy(),
                SampleBatch.ACTIONS: bufs["act"].reshape(rows).copy(),
                SampleBatch.ACTION_LOGP: bufs["logp"].reshape(rows).copy(),
                SampleBatch.VF_PREDS: bufs["vf"].reshape(rows).copy(),
                SampleBatch.ACTION_DIST_INPUTS: bufs["logits"].reshape(rows, -1).copy(),
                SampleBatch.REWARDS: bufs["rew"].reshape(rows).copy(),
                SampleBatch.DONES: bufs["done"].reshape(rows).copy(),
                SampleBatch.ADVANTAGES: adv.reshape(rows).astype(np.float32),
                SampleBatch.VALUE_TARGETS: ret.reshape(rows).astype(np.float32)})
        self._sample_time += time.perf_counter() - t0
        return out

    # ------------------------------------------------------------------ recurrent / attention policies
    def _env_reset_all(self):
        return np.asarray(self._obs) if self.vec_env is not None else np.stack([np.asarray(o) for o in self._obs])

    def _recurrent_rollout(self, T: int, snapshot_every: int):
        """T env steps of a sequence model with per-env state carried across fragments. Returns the
        time-major buffers, the state snapshots taken every `snapshot_every` steps (t = 0, L, ..),
        the state / previous action / reward after the last step and the last observation."""
        import torch

        n = self.env.num_envs
        model = self.policy.model
        dist_cls = self.policy.dist_class
        discrete = hasattr(self.env.action_space, "n")
        if getattr(self, "_rstate", None) is None:
            self._rstate = model.initial_state(n, torch.device("cpu"))
            self._prev_a = np.zeros(n, np.int64) if discrete else np.zeros((n,) + tuple(self.env.action_space.shape),
                                                                           np.float32)
            self._prev_r = np.zeros(n, np.float32)
        explore = self.config.get("explore", True)
        obs = self._env_reset_all()
        buf = {"obs": [], "actions": [], "action_logp": [], "vf_preds": [], "action_dist_inputs": [], "rewards": [],
               "dones": [], "prev_actions": [], "prev_rewards": []}
        snaps = [[] for _ in self._rstate]
        state = self._rstate
        with torch.no_grad():
            for t in range(T):
                if t % snapshot_every == 0:
                    for k, s_ in enumerate(state):
                        snaps[k].append(s_.numpy().copy())
                logits, v, new = model.step(torch.as_tensor(obs), state, torch.as_tensor(self._prev_a),
                                            torch.as_tensor(self._prev_r))
                d = dist_cls(logits.float())
                a = d.sample() if explore else d.deterministic_sample()
                an = a.numpy()
                buf["obs"].append(obs)
                buf["actions"].append(an)
                buf["action_logp"].append(d.logp(a).numpy())
                buf["vf_preds"].append(v.float().numpy())
                buf["action_dist_inputs"].append(logits.float().numpy())
                buf["prev_actions"].append(self._prev_a.copy())
                buf["prev_rewards"].append(self._prev_r.copy())
                if self.vec_env is not None:
                    nobs, rew, done = self.env.vector_step(an)
                    rew, done = np.asarray(rew, np.float32), np.asarray(done, bool)
                else:
                    nl, rew, done, _ = self.env.vector_step(list(an))
                    rew, done = np.asarray(rew, np.float32), np.asarray(done, bool)
                    for i in np.nonzero(done)[0]:
                        nl[i] = self.env.reset_at(i)
                    nobs = np.stack([np.asarray(o) for o in nl])
                buf["rewards"].append(rew)
                buf["dones"].append(done.astype(np.float32))
                self._ep_reward += rew
                self._ep_len += 1
                for i in np.nonzero(done)[0]:
                    self._completed.append((float(self._ep_reward[i]), int(self._ep_len[i])))
                    self._ep_reward[i] = 0.0
                    self._ep_len[i] = 0
                state = new
                self._prev_a = an.copy()
                self._prev_r = rew.copy()
                if done.any():  # a new episode starts from the initial state, no previous action / reward
                    state = model.reset_state(state, done)
                    self._prev_a[done] = 0
                    self._prev_r[done] = 0.0
                obs = np.asarray(nobs)
            _, last_v, _ = model.step(torch.as_tensor(obs), state, torch.as_tensor(self._prev_a),
                                      torch.as_tensor(self._prev_r))
        self._rstate = state
        self._obs = obs if self.vec_env is not None else list(obs)
        self.policy.global_timestep += T * n
        return {k: np.stack(v) for k, v in buf.items()}, [np.stack(s_) for s_ in snaps], last_v.float().numpy(), obs

    def _sample_recurrent(self) -> SampleBatch:
        """On-policy sample for a sequence model (LSTM / attention): GAE time-major, then the
        fixed-length sequence layout of rllib/policy/rnn_sequencing.fragment_to_sequences (state at
        every sequence start, `resets` where an episode begins inside a sequence)."""
        from ray_memory_management_amd.rllib.policy.rnn_sequencing import SEQ_LENS, RESETS, fragment_to_sequences, \
            state_key

        t0 = time.perf_counter()
        T = int(self.config.get("rollout_fragment_length", 200))
        L = int(self.policy.model.max_seq_len)
        buf, snaps, last_v, _ = self._recurrent_rollout(T, L)
        vf = buf["vf_preds"] if self.config.get("use_critic", True) else np.zeros_like(buf["vf_preds"])
        if not self.config.get("use_critic", True):
            last_v = np.zeros_like(last_v)
        adv, ret = compute_gae_for_trajectories(buf["rewards"], vf, buf["dones"], last_v, self.config.get("gamma", 0.99),
                                                self.config.get("lambda", self.config.get("lambda_", 1.0)))
        cols = dict(buf)
        cols[SampleBatch.ADVANTAGES] = adv.astype(np.float32)
        cols[SampleBatch.VALUE_TARGETS] = ret.astype(np.float32)
        seq_cols, state_in, seq_lens, resets = fragment_to_sequences(cols, buf["dones"], snaps, L)
        out = SampleBatch({SampleBatch.OBS: seq_cols.pop("obs"), **seq_cols})
        for k, st in enumerate(state_in):
            dict.__setitem__(out, state_key(k), st)
        dict.__setitem__(out, SEQ_LENS, seq_lens)
        dict.__setitem__(out, RESETS, resets)
        out.count = len(resets)
        if self.callbacks is not None:
            self.callbacks.on_sample_end(worker=self, samples=out)
        self._sample_time += time.perf_counter() - t0
        return out

    def sample_time_major(self) -> Dict[str, Any]:
        """One unroll for an off-policy (V-trace) learner: time-major [T, n] columns + each env's
        observation after the last step (the learner bootstraps from its own value of it).
        Parity: reference rllib/algorithms/impala (rollout_fragment_length unrolls, make_time_major).
        Returns {"T", "n", "obs", "actions", "action_logp", "action_dist_inputs", "rewards",
        "dones", "last_obs"}; no GAE, no value head on the worker."""
        import torch

        t0 = time.perf_counter()
        T = int(self.config.get("rollout_fragment_length", 50))
        n = self.env.num_envs
        if getattr(self.policy.model, "is_recurrent", False):
            # recurrent V-trace unroll: the state at the unroll start, previous actions / rewards, and
            # `resets` where an episode begins inside the unroll; the learner re-runs the sequence
            buf, snaps, _, last_obs = self._recurrent_rollout(T, T)
            resets = np.zeros((T, n), np.float32)
            resets[1:] = buf["dones"][:-1]
            out = {"obs": buf["obs"], "actions": buf["actions"], "action_logp": buf["action_logp"],
                   "action_dist_inputs": buf["action_dist_inputs"], "rewards": buf["rewards"], "dones": buf["dones"],
                   "prev_actions": buf["prev_actions"], "prev_rewards": buf["prev_rewards"], "resets": resets,
                   "state_in": [s_[0] for s_ in snaps], "last_prev_actions": self._prev_a.copy(),
                   "last_prev_rewards": self._prev_r.copy(), "T": T, "n": n, "last_obs": np.array(last_obs, copy=True)}
            self._sample_time += time.perf_counter() - t0
            return out
        explore = self.config.get("explore", True)
        obs0 = np.asarray(self._obs) if self.vec_env is not None else np.stack([np.asarray(o) for o in self._obs])
        A = getattr(self.env.action_space, "n", 1)
        out = {"obs": np.empty((T, n) + obs0.shape[1:], dtype=obs0.dtype), "actions": np.empty((T, n), np.int64),
               "action_logp": np.empty((T, n), np.float32), "action_dist_inputs": np.empty((T, n, A), np.float32),
               "rewards": np.empty((T, n), np.float32), "dones": np.empty((T, n), np.float32)}
        model = self.policy.model
        obs = obs0
        with torch.inference_mode():
            for t in range(T):
                out["obs"][t] = obs
                logits, _ = model(torch.from_numpy(np.ascontiguousarray(obs)))
                logits = logits.float()
                if explore:  # Gumbel-max sampling of the categorical policy
                    g = -torch.log(-torch.log(torch.rand_like(logits).clamp_(1e-10, 1.0)))
                    a = torch.argmax(logits + g, dim=-1)
                else:
                    a = torch.argmax(logits, dim=-1)
                out["action_dist_inputs"][t] = logits.numpy()
                out["action_logp"][t] = torch.log_softmax(logits, -1).gather(1, a.unsqueeze(1)).squeeze(1).numpy()
                an = a.numpy()
                out["actions"][t] = an
                if self.vec_env is not None:
                    obs, rew, done = self.env.vector_step(an)
                    rew, done = np.asarray(rew, np.float32), np.asarray(done, bool)
                else:
                    nobs, rew, done, _ = self.env.vector_step(list(an))
                    rew, done = np.asarray(rew, np.float32), np.asarray(done, bool)
                    for i in np.nonzero(done)[0]:
                        nobs[i] = self.env.reset_at(i)
                    obs = np.stack([np.asarray(o) for o in nobs])
                out["rewards"][t] = rew
                out["dones"][t] = done
                self._ep_reward += rew
                self._ep_len += 1
                for i in np.nonzero(done)[0]:
                    self._completed.append((float(self._ep_reward[i]), int(self._ep_len[i])))
                    self._ep_reward[i] = 0.0
                    self._ep_len[i] = 0
        self._obs = obs if self.vec_env is not None else list(obs)
        self.policy.global_timestep += T * n
        out.update(T=T, n=n, last_obs=np.array(obs, copy=True))
        self._sample_time += time.perf_counter() - t0
        return out

    def sample_with_count(self):
        b = self.sample()
        return b, b.count

    # ------------------------------------------------------------------ weights / metrics
    def get_weights(self, policies=None):
        return self.policy.get_weights()

    def set_weights(self, weights, global_vars=None):
        import warnings

        import torch

        if "__rmm_flat_bf16__" in weights:  # a learner's flat bf16 HBM publication (LearnerActor)
            weights = {**{k: v.detach().cpu() for k, v in self.policy.model.state_dict().items()},
                       **unpack_flat_weights(weights)}  # buffers keep their current values
        with warnings.catch_warnings():  # store-backed arrays are read-only; load_state_dict copies them
            warnings.simplefilter("ignore", UserWarning)
            self.policy.set_weights({k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v)))
                                     for k, v in weights.items()})

    # ------------------------------------------------------------------ learning (policy templates)
    def learn_on_batch(self, samples) -> Dict:
        return {"default_policy": self.policy.learn_on_batch(samples)}

    def compute_gradients(self, samples):
        return self.policy.compute_gradients(samples)

    def apply_gradients(self, grads) -> None:
        self.policy.apply_gradients(grads)

    def get_global_vars(self) -> Dict:
        return {"timestep": getattr(self.policy, "global_timestep", 0)}

    def set_global_vars(self, global_vars: Dict) -> None:
        if "timestep" in (global_vars or {}):
            self.policy.global_timestep = global_vars["timestep"]

    def get_metrics(self) -> List[tuple]:
        out, self._completed = self._completed, []
        return out

    def get_policy(self, policy_id: str = "default_policy"):
        return self.policy

    def foreach_policy(self, fn):
        return [fn(self.policy, "default_policy")]

    def apply(self, fn, *args):
        return fn(self, *args)

    def sample_time(self):
        return self._sample_time

    def stop(self):
        if self.output_writer is not None:
            self.output_writer.close()

    @staticmethod
    def evaluate_episodes(policy, env_creator, env, env_config, num_episodes: int, max_steps: int = 100000,
                          seed: Optional[int] = None):
        """Greedy evaluation episodes; with `seed` the episode starts are reproducible."""
        e = env_creator(env_config) if env_creator is not None else make_env(env, env_config)
        rewards, lens = [], []
        for k in range(num_episodes):
            if seed is not None:
                try:
                    o = e.reset(seed=int(seed) * 7919 + 100003 + k)
                except TypeError:
                    o = e.reset()
            else:
                o = e.reset()
            total, steps, done = 0.0, 0, False
            while not done and steps < max_steps:
                a = policy.compute_single_action(np.asarray(o), explore=False)
                o, r, done, _ = e.step(int(a) if np.ndim(a) == 0 else a)
                total += r
                steps += 1
            rewards.append(total)
            lens.append(steps)
        return rewards, lens
