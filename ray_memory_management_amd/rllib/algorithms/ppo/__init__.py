"""PPO. Parity: reference rllib/algorithms/ppo/ppo.py (PPOConfig defaults + training(...),
PPO.training_step: synchronous_parallel_sample -> standardize advantages ->
multi_gpu_train_one_step (num_sgd_iter x minibatches) -> sync weights -> UpdateKL).

On MI355X the learner is the fused PPOLearner (bf16 weights / fp32 master, HIP-graph SGD steps,
K5 loss, K6 Adam); with `gpu_rollouts=True` and a GPU-vectorisable env the sampler is the
on-device GPURolloutSampler too (the bench.py configuration).
"""
from __future__ import annotations

from typing import Dict

import torch

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

    def validate_config(self, c):
        super().validate_config(c)
        if c.sgd_minibatch_size > c.train_batch_size:
            raise ValueError(f"`sgd_minibatch_size` ({c.sgd_minibatch_size}) must be <= `train_batch_size` "
                             f"({c.train_batch_size}).")
        if c.entropy_coeff < 0:
            raise ValueError("`entropy_coeff` must be >= 0.0")

    def _setup_learner(self):
        from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        local = self.workers.local_worker()
        import copy

        model = copy.deepcopy(local.policy.model)
        lcfg = dict(gamma=c.gamma, lambda_=c.lambda_, kl_coeff=c.kl_coeff, kl_target=c.kl_target,
                    clip_param=c.clip_param, vf_clip_param=c.vf_clip_param, vf_loss_coeff=c.vf_loss_coeff,
                    entropy_coeff=c.entropy_coeff, lr=c.lr, train_batch_size=c.train_batch_size,
                    sgd_minibatch_size=c.sgd_minibatch_size, num_sgd_iter=c.num_sgd_iter, grad_clip=c.grad_clip)
        self.learner = PPOLearner(model, lcfg, device=dev, action_space=local.env.action_space)
        self._device = dev
        self._sync_from_learner()

    def _sync_from_learner(self):
        w = self.learner.get_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def training_step(self) -> Dict:
        c = self.algo_config
        batch = self.workers.synchronous_parallel_sample(c.train_batch_size)
        n = batch.count
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        batch = SampleBatch({k: torch.as_tensor(v) for k, v in batch.items()})
        if self._device != "cpu":
            batch = batch.to_device(self._device)
        stats = self.learner.update(batch)
        self._counters["num_env_steps_trained"] += n
        self._counters["num_agent_steps_trained"] += n
        self._sync_from_learner()
        return dict(stats)

    def _extra_state(self):
        return {"kl_coeff": self.learner.kl_coeff}

    def _load_extra_state(self, s):
        if "kl_coeff" in s:
            self.learner.kl_coeff = s["kl_coeff"]

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, weights):
        self.learner.set_weights(weights)
        self._sync_from_learner()


DEFAULT_CONFIG = PPOConfig().to_dict()
