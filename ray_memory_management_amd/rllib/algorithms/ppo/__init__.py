"""PPO. Parity: reference rllib/algorithms/ppo/ppo.py (PPOConfig defaults + training(...),
PPO.training_step: synchronous_parallel_sample -> standardize advantages ->
multi_gpu_train_one_step (num_sgd_iter x minibatches) -> sync weights -> UpdateKL).

With ``num_learner_workers=N`` the learner is N GPU learner actors (rllib/execution/learner_group.py)
averaging gradients over RCCL; with ``postprocess_on_learner=True`` rollout workers ship raw
fragments and GAE + advantage standardisation run on the learner GPUs (K17).

On MI355X the learner is the fused PPOLearner (bf16 weights / fp32 master, HIP-graph SGD steps,
K5 loss, K6 Adam); with `gpu_rollouts=True` and a GPU-vectorisable env the sampler is the
on-device GPURolloutSampler too (the bench.py configuration).
"""
from __future__ import annotations

import os

from typing import Dict

import torch

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class PPOConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or PPO)
        self.lr_schedule = None
        self.use_critic = True
        self.use_gae = True
        self.lambda_ = 1.0
        self.kl_coeff = 0.2
        self.sgd_minibatch_size = 128
        self.num_sgd_iter = 30
        self.shuffle_sequences = True
        self.vf_loss_coeff = 1.0
        self.entropy_coeff = 0.0
        self.entropy_coeff_schedule = None
        self.clip_param = 0.3
        self.vf_clip_param = 10.0
        self.grad_clip = None
        self.kl_target = 0.01
        self.rollout_fragment_length = 200
        self.train_batch_size = 4000
        self.lr = 5e-5
        self.model["vf_share_layers"] = False

    def training(self, *, lr_schedule=None, use_critic=None, use_gae=None, lambda_=None, kl_coeff=None,
                 sgd_minibatch_size=None, num_sgd_iter=None, shuffle_sequences=None, vf_loss_coeff=None,
                 entropy_coeff=None, entropy_coeff_schedule=None, clip_param=None, vf_clip_param=None,
                 grad_clip=None, kl_target=None, **kwargs) -> "PPOConfig":
        super().training(**kwargs)
        for k, v in dict(lr_schedule=lr_schedule, use_critic=use_critic, use_gae=use_gae, lambda_=lambda_,
                         kl_coeff=kl_coeff, sgd_minibatch_size=sgd_minibatch_size, num_sgd_iter=num_sgd_iter,
                         shuffle_sequences=shuffle_sequences, vf_loss_coeff=vf_loss_coeff,
                         entropy_coeff=entropy_coeff, entropy_coeff_schedule=entropy_coeff_schedule,
                         clip_param=clip_param, vf_clip_param=vf_clip_param, grad_clip=grad_clip,
                         kl_target=kl_target).items():
            if v is not None:
                setattr(self, k, v)
        return self


class PPO(Algorithm):
    _config_class = PPOConfig
    _supports_sequence_models = True
    learner = None
    learner_group = None
    _weights_ref = None

    def validate_config(self, c):
        super().validate_config(c)
        if c.sgd_minibatch_size > c.train_batch_size:
            raise ValueError(f"`sgd_minibatch_size` ({c.sgd_minibatch_size}) must be <= `train_batch_size` "
                             f"({c.train_batch_size}).")
        if c.entropy_coeff < 0:
            raise ValueError("`entropy_coeff` must be >= 0.0")
        from ray_memory_management_amd.rllib.recurrent_net import wants_sequence_model

        if wants_sequence_model(c.model):
            if type(self).__name__ != "PPO":
                raise ValueError(f"{type(self).__name__} does not train recurrent / attention models")
            if getattr(c, "gpu_rollouts", False):
                raise ValueError("gpu_rollouts (device env + fused sampler) runs feed-forward policies only; "
                                 "use CPU rollout workers with use_lstm / use_attention")
            # sequences need the state recorded by the rollout: GAE + sequence layout on the workers
            c.postprocess_on_learner = False
        if c.num_learner_workers and c.num_learner_workers > 1:
            if c.train_batch_size % c.num_learner_workers or c.sgd_minibatch_size % c.num_learner_workers:
                raise ValueError("train_batch_size and sgd_minibatch_size are totals across learner workers: "
                                 "they must be divisible by num_learner_workers")
            if c.num_workers % c.num_learner_workers:
                raise ValueError("num_workers (rollout workers) must be a multiple of num_learner_workers so "
                                 "every learner trains on the same number of fragments")

    def _learner_cfg(self, n_learners: int = 1) -> dict:
        c = self.algo_config
        return dict(gamma=c.gamma, lambda_=c.lambda_, kl_coeff=c.kl_coeff, kl_target=c.kl_target,
                    clip_param=c.clip_param, vf_clip_param=c.vf_clip_param, vf_loss_coeff=c.vf_loss_coeff,
                    entropy_coeff=c.entropy_coeff, lr=c.lr, train_batch_size=c.train_batch_size // n_learners,
                    sgd_minibatch_size=c.sgd_minibatch_size // n_learners, num_sgd_iter=c.num_sgd_iter,
                    grad_clip=c.grad_clip, lr_schedule=c.lr_schedule,
                    entropy_coeff_schedule=c.entropy_coeff_schedule,
                    compute_dtype=getattr(c, "compute_dtype", "bf16"))

    def _setup_learner(self):
        from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

        c = self.algo_config
        local = self.workers.local_worker()
        self.learner = None
        self.learner_group = None
        self._weights_ref = None
        if c.num_learner_workers and c.num_learner_workers > 0:
            from ray_memory_management_amd.rllib.execution.learner_group import LearnerGroup

            n = int(c.num_learner_workers)
            self.learner_group = LearnerGroup(
                n, local.env.observation_space, local.env.action_space, c.model, self._learner_cfg(n),
                num_gpus_per_learner=c.num_gpus_per_learner_worker,
                num_cpus_per_learner=c.num_cpus_per_learner_worker, backend=c.learner_collective_backend,
                seed=int(c.seed or 0), strategy=self.learner_strategy())
            self._device = "learner_actors"
            self._weights_ref = self.learner_group.weights_ref()
            local.set_weights(ray.get(self._weights_ref))
            self.workers.sync_weights(ref=self._weights_ref)
            return
        import copy

        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        model = copy.deepcopy(local.policy.model)
        self.learner = PPOLearner(model, self._learner_cfg(), device=dev, action_space=local.env.action_space)
        self._device = dev
        self._sync_from_learner()

    def _sync_from_learner(self):
        w = self.learner.get_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def _ma_learner(self, pid, policy):
        import copy

        from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

        dev = "cuda" if self.algo_config.num_gpus and torch.cuda.is_available() else "cpu"
        return PPOLearner(copy.deepcopy(policy.model), self._learner_cfg(), device=dev,
                          action_space=policy.action_space)

    def _ma_update(self, learner, batch):
        b = SampleBatch({k: torch.as_tensor(v) for k, v in batch.items()})
        if learner.device.type != "cpu":
            b = b.to_device(learner.device)
        return dict(learner.update(b))

    def training_step(self) -> Dict:
        if self._multi_agent:
            return self._ma_training_step()
        if self.learner_group is not None:
            return self._training_step_learner_actors()
        c = self.algo_config
        batch = self.workers.synchronous_parallel_sample(c.train_batch_size, concat=not c.postprocess_on_learner)
        n = sum(b.count for b in batch) if isinstance(batch, list) else batch.count
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        if c.postprocess_on_learner:
            st = self.learner.update_fragments(batch)
        else:
            batch = SampleBatch({k: torch.as_tensor(v) for k, v in batch.items()})
            if self._device != "cpu":
                batch = batch.to_device(self._device)
            st = self.learner.update(batch)
        self._counters["num_env_steps_trained"] += n
        self._counters["num_agent_steps_trained"] += n
        self._sync_from_learner()
        return dict(st)

    def _training_step_learner_actors(self) -> Dict:
        """synchronous_parallel_sample over the rollout actors (each first loads the weights the
        learners published last iteration — same actor queue, so no extra round trip) → every
        learner actor trains on its shard of fragments straight from the object store → learner 0
        publishes the new weights as an object ref for the next round. The driver only sees refs
        and the small stats dicts."""
        from ray_memory_management_amd.rllib.execution.sample_ingest import split_for_learners

        c = self.algo_config
        remote = self.workers.remote_workers()
        if not remote:
            raise ValueError("learner actors need remote rollout workers (num_workers > 0)")
        n_l = self.learner_group.n
        refs, steps = [], 0
        per_round = c.num_workers * c.rollout_fragment_length * c.num_envs_per_worker
        rounds = max(1, -(-c.train_batch_size // max(per_round, 1)))
        dev = self._device_weights_ok()
        shared = dev and self._shared_weights_ok()
        pre, self._prefetched = self._prefetched, None
        for r in range(rounds):
            if r == 0 and pre is not None:  # queued behind last iteration's update (see below)
                refs.extend(pre)
                steps += per_round
                continue
            for i, w in enumerate(remote):
                if r == 0 and self._weights_ref is not None:
                    w.set_weights.remote(self._dev_refs[i % n_l] if dev and self._dev_refs else self._weights_ref)
                    if shared and self._dev_refs:
                        self._aliased = True
                refs.append(w.sample.remote())
            steps += per_round
        if c.postprocess_on_learner:
            pending = self.learner_group.update_async(split_for_learners(refs, n_l))
        else:
            from ray_memory_management_amd.rllib.sample_batch import concat_samples

            shards = split_for_learners(refs, n_l)
            pending = [l.update_batch.remote(concat_samples(ray.get(s)))
                       for l, s in zip(self.learner_group.learners, shards)]
        # the weight publication is queued right behind the update on each learner (actor calls run
        # in order), so it runs while the driver is still collecting the update's stats: no extra
        # driver round trip before the next iteration's set_weights + sample
        if shared:  # once: the learners move their live weights into HBM objects the workers alias
            if self._dev_refs is None:
                self._dev_refs = self.learner_group.shared_weights_refs()
                self._dev_shared = True
        elif dev:  # GPU rollout workers read the learners' bf16 weights from HBM (hipIPC)
            self._dev_refs = self.learner_group.device_weights_refs()
        else:
            self._weights_ref = self.learner_group.weights_ref()
        if (shared and self._aliased and rounds == 1 and c.postprocess_on_learner
                and os.environ.get("RMM_PREFETCH_SAMPLE", "1") != "0"):
            # the workers alias the learners' live weights, so the next iteration's samples need only
            # wait for this update: queue them now with the update's result refs as arguments (the
            # runtime starts each sample the moment its learner's update finished) — the driver's
            # get + submit round trip leaves the critical path; same samples, same weights
            self._prefetched = [w.sample.remote(pending[i % n_l]) for i, w in enumerate(remote)]
        stats = ray.get(pending)
        self._counters["num_env_steps_sampled"] += steps
        self._counters["num_env_steps_trained"] += steps
        self._counters["num_agent_steps_trained"] += steps
        self._timesteps_total += steps
        st = dict(stats[0])
        st["num_learners"] = n_l
        st["learner_update_s_max"] = max(s.get("learner_update_s", 0.0) for s in stats)
        return st

    _dev_refs = None
    _prefetched = None  # next iteration's sample refs, queued behind this iteration's update
    _aliased = False    # the rollout workers were sent the learners' shared weights
    _dev_shared = False  # _dev_refs are live shared-weight descriptors (not per-iteration copies)

    def _shared_weights_ok(self) -> bool:
        """Rollout workers alias the learners' live HBM weights (zero-copy, set once) instead of
        receiving a copy per iteration. Default on (RMM_SHARED_WEIGHTS=0 or config
        share_device_weights=False turns it off): runtime bench 338-348k -> 350-354k samples/s on
        MI355X. The GPU memory fault this path hit in rounds 3-4 was the hybrid worker's graph
        recapture after the rebind: its warm-up steps ran at rollout row T and wrote past the
        rollout buffers (fixed in HybridGroup.capture; profiles/shared_weights_r4.txt)."""
        import os

        env = os.environ.get("RMM_SHARED_WEIGHTS")
        want = env == "1" if env is not None else bool(getattr(self.algo_config, "share_device_weights", True))
        # only learners with live device weights (the bf16 compute weights or the fp32 learner's split
        # pair) can be aliased; others publish a fresh copy every iteration
        return want and self.learner_group is not None and self.learner_group.shared_kind() is not None

    def _device_weights_ok(self) -> bool:
        """Weights go learner → rollout workers through HBM when both sides are GPU processes:
        learners with GPUs and rollout workers with a GPU slice (hybrid / GPU rollouts)."""
        c = self.algo_config
        if getattr(self, "_dev_w", None) is None:
            import os

            # only the GPU rollout-worker classes load the flat bf16 HBM layout; WorkerSet falls back
            # to a plain RolloutWorker for envs outside the vector registry or with an env_creator
            cls = getattr(self.workers, "remote_worker_class", None)
            gpu_cls = getattr(cls, "__name__", "") in ("GPURolloutWorker", "HybridRolloutWorker")
            self._dev_w = bool(c.num_gpus_per_learner_worker and (c.num_gpus_per_worker or c.gpu_rollouts)
                               and gpu_cls and not os.environ.get("RMM_HOST_WEIGHTS"))
        return self._dev_w

    def _extra_state(self):
        if self._multi_agent:
            return {}
        if self.learner_group is not None:
            s = self.learner_group.get_state()
            return {"kl_coeff": s["kl_coeff"], "learner_timesteps": s["timesteps"]}
        return {"kl_coeff": self.learner.kl_coeff, "learner_timesteps": self.learner.timesteps}

    def _load_extra_state(self, s):
        if self.learner_group is not None:
            st = self.learner_group.get_state()
            st.update({"kl_coeff": s.get("kl_coeff", st["kl_coeff"]),
                       "timesteps": s.get("learner_timesteps", st["timesteps"])})
            self.learner_group.set_state(st)
            return
        if "kl_coeff" in s:
            self.learner.kl_coeff = s["kl_coeff"]
        if "learner_timesteps" in s:
            self.learner.timesteps = s["learner_timesteps"]

    def get_weights(self):
        if self._multi_agent:
            return {pid: ln.get_weights() for pid, ln in self.ma_learners.items()}
        if self.learner_group is not None:
            return self.learner_group.get_weights()
        return self.learner.get_weights()

    def set_weights(self, weights):
        self._prefetched = None  # samples queued with the previous weights must not be trained on
        if self.learner_group is not None:
            self.learner_group.set_weights(weights)
            self._weights_ref = self.learner_group.weights_ref()
            if self._dev_refs is not None and not self._dev_shared:
                # copies: the next iteration must not push pre-restore HBM weights. Shared mode keeps its
                # descriptors: the learners wrote the restored weights into the aliased buffers in place,
                # and a flat snapshot must never be copied into parameters that alias the learner
                self._dev_refs = self.learner_group.device_weights_refs()
            self.workers.local_worker().set_weights(weights)
            self.workers.sync_weights(ref=self._weights_ref)
            return
        self.learner.set_weights(weights)
        self._sync_from_learner()

    def get_policy(self, policy_id: str = "default_policy"):
        if self.learner_group is not None and self._weights_ref is not None:
            if self._dev_refs is not None:  # the host ref is only refreshed on demand on this path
                self._weights_ref = self.learner_group.weights_ref()
            self.workers.local_worker().set_weights(ray.get(self._weights_ref))
        return super().get_policy(policy_id)

    def cleanup(self):
        pre, self._prefetched = self._prefetched, None
        if pre:  # let queued samples finish before the learners whose weights they alias go away
            try:
                ray.wait(pre, num_returns=len(pre), timeout=30.0)
            except Exception:
                pass
        if getattr(self, "learner_group", None) is not None and not getattr(self, "_multi_agent", False):
            self.learner_group.stop()
        super().cleanup()


DEFAULT_CONFIG = PPOConfig().to_dict()
