"""AlgorithmConfig builder. Parity: reference rllib/algorithms/algorithm_config.py (environment /
framework / rollouts / training / resources / evaluation / debugging / reporting / callbacks /
exploration builder methods, to_dict, build, copy)."""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional, Type


class AlgorithmConfig:
    def __init__(self, algo_class=None):
        self.algo_class = algo_class
        # environment
        self.env = None
        self.env_config: Dict[str, Any] = {}
        self.observation_space = None
        self.action_space = None
        # framework
        self.framework_str = "torch"
        # rollouts
        self.num_workers = 2
        self.num_envs_per_worker = 1
        self.rollout_fragment_length = 200
        self.batch_mode = "truncate_episodes"
        self.explore = True
        # training
        self.gamma = 0.99
        self.lr = 0.001
        self.train_batch_size = 4000
        self.model: Dict[str, Any] = {"fcnet_hiddens": [256, 256], "fcnet_activation": "tanh",
                                      "vf_share_layers": False, "conv_filters": None}
        self.optimizer: Dict[str, Any] = {}
        # resources
        self.num_gpus = 0
        self.num_cpus_per_worker = 1
        self.num_gpus_per_worker = 0
        self.num_cpus_for_local_worker = 1
        # evaluation
        self.evaluation_interval = None
        self.evaluation_duration = 10
        self.evaluation_duration_unit = "episodes"
        self.evaluation_config: Dict[str, Any] = {}
        self.evaluation_num_workers = 0
        # reporting / debugging
        self.metrics_num_episodes_for_smoothing = 100
        self.min_time_s_per_iteration = None
        self.min_sample_timesteps_per_iteration = 0
        self.seed = None
        self.log_level = "WARN"
        self.callbacks_class = None
        self.exploration_config: Dict[str, Any] = {}
        self.recreate_failed_workers = False
        # MI355X fast path: on-device vectorised env + fused learner
        self.gpu_rollouts = False
        # GPU compute precision of the fused learner and the GPU rollout policy: "bf16" (fp32 master
        # weights + moments, bf16 MFMA kernels) or "fp32" (precision-matched with the reference's
        # fp32 torch PPO: fp32 weights, gradients and convolutions end to end)
        self.compute_dtype = "bf16"
        # learner actors: one data-parallel learner per GPU, gradients all-reduced over RCCL
        # (0 = one learner in the driver process, the reference's default)
        self.num_learner_workers = 0
        self.num_gpus_per_learner_worker = 1
        self.num_cpus_per_learner_worker = 1
        self.learner_collective_backend = "auto"  # nccl (=RCCL) for GPU learners, gloo on CPU
        # rollout workers ship raw fragments; GAE + advantage standardisation run on the learner GPU
        self.postprocess_on_learner = False
        # rollout-side policy class (class or dotted import path); None = the PG TorchPolicy
        self.policy_class = None
        # offline data (reference AlgorithmConfig.offline_data)
        self.input_ = "sampler"
        self.shuffle_buffer_size = 0
        self.output = None
        self.output_compress_columns = ["obs", "new_obs"]
        self.output_max_file_size = 64 * 1024 * 1024
        self.off_policy_estimation_methods = {}
        # multi-agent (reference AlgorithmConfig.multi_agent): policies {id: PolicySpec | tuple | None}
        self.multiagent: Dict[str, Any] = {"policies": {}, "policy_mapping_fn": None, "policies_to_train": None}

    # ---- builder methods (each returns self)
    def environment(self, env=None, *, env_config=None, observation_space=None, action_space=None,
                    **kw) -> "AlgorithmConfig":
        if env is not None:
            self.env = env
        if env_config is not None:
            self.env_config = dict(env_config)
        if observation_space is not None:
            self.observation_space = observation_space
        if action_space is not None:
            self.action_space = action_space
        return self

    def framework(self, framework: Optional[str] = None, **kw) -> "AlgorithmConfig":
        if framework is not None:
            if framework not in ("torch",):
                raise ValueError(f"framework={framework!r}: only 'torch' (PyTorch-ROCm) is supported")
            self.framework_str = framework
        return self

    def rollouts(self, *, num_rollout_workers=None, num_envs_per_worker=None, rollout_fragment_length=None,
                 batch_mode=None, gpu_rollouts=None, postprocess_on_learner=None, **kw) -> "AlgorithmConfig":
        if postprocess_on_learner is not None:
            self.postprocess_on_learner = bool(postprocess_on_learner)
        if num_rollout_workers is not None:
            self.num_workers = num_rollout_workers
        if num_envs_per_worker is not None:
            self.num_envs_per_worker = num_envs_per_worker
        if rollout_fragment_length is not None:
            self.rollout_fragment_length = rollout_fragment_length
        if batch_mode is not None:
            self.batch_mode = batch_mode
        if gpu_rollouts is not None:
            self.gpu_rollouts = gpu_rollouts
        for k, v in kw.items():  # e.g. rollout_env_threads, rollout_double_buffer (hybrid rollout workers)
            if v is not None:
                setattr(self, k, v)
        return self

    def training(self, *, gamma=None, lr=None, train_batch_size=None, model=None, optimizer=None,
                 **kw) -> "AlgorithmConfig":
        if gamma is not None:
            self.gamma = gamma
        if lr is not None:
            self.lr = lr
        if train_batch_size is not None:
            self.train_batch_size = train_batch_size
        if model is not None:
            self.model = {**self.model, **model}
        if optimizer is not None:
            self.optimizer = dict(optimizer)
        for k, v in kw.items():
            if v is not None:
                setattr(self, k, v)
        return self

    def resources(self, *, num_gpus=None, num_cpus_per_worker=None, num_gpus_per_worker=None,
                  num_cpus_for_local_worker=None, num_learner_workers=None, num_gpus_per_learner_worker=None,
                  num_cpus_per_learner_worker=None, learner_collective_backend=None, **kw) -> "AlgorithmConfig":
        if learner_collective_backend is not None:
            self.learner_collective_backend = learner_collective_backend
        if num_learner_workers is not None:
            self.num_learner_workers = int(num_learner_workers)
        if num_gpus_per_learner_worker is not None:
            self.num_gpus_per_learner_worker = num_gpus_per_learner_worker
        if num_cpus_per_learner_worker is not None:
            self.num_cpus_per_learner_worker = num_cpus_per_learner_worker
        if num_gpus is not None:
            self.num_gpus = num_gpus
        if num_cpus_per_worker is not None:
            self.num_cpus_per_worker = num_cpus_per_worker
        if num_gpus_per_worker is not None:
            self.num_gpus_per_worker = num_gpus_per_worker
        if num_cpus_for_local_worker is not None:
            self.num_cpus_for_local_worker = num_cpus_for_local_worker
        return self

    def evaluation(self, *, evaluation_interval=None, evaluation_duration=None, evaluation_duration_unit=None,
                   evaluation_config=None, evaluation_num_workers=None, **kw) -> "AlgorithmConfig":
        if evaluation_interval is not None:
            self.evaluation_interval = evaluation_interval
        if evaluation_duration is not None:
            self.evaluation_duration = evaluation_duration
        if evaluation_duration_unit is not None:
            self.evaluation_duration_unit = evaluation_duration_unit
        if evaluation_config is not None:
            self.evaluation_config = dict(evaluation_config)
        if evaluation_num_workers is not None:
            self.evaluation_num_workers = evaluation_num_workers
        return self

    def debugging(self, *, seed=None, log_level=None, **kw) -> "AlgorithmConfig":
        if seed is not None:
            self.seed = seed
        if log_level is not None:
            self.log_level = log_level
        return self

    def reporting(self, *, metrics_num_episodes_for_smoothing=None, min_time_s_per_iteration=None,
                  min_sample_timesteps_per_iteration=None, **kw) -> "AlgorithmConfig":
        if metrics_num_episodes_for_smoothing is not None:
            self.metrics_num_episodes_for_smoothing = metrics_num_episodes_for_smoothing
        if min_time_s_per_iteration is not None:
            self.min_time_s_per_iteration = min_time_s_per_iteration
        if min_sample_timesteps_per_iteration is not None:
            self.min_sample_timesteps_per_iteration = min_sample_timesteps_per_iteration
        return self

    def callbacks(self, callbacks_class) -> "AlgorithmConfig":
        self.callbacks_class = callbacks_class
        return self

    def exploration(self, *, explore=None, exploration_config=None, **kw) -> "AlgorithmConfig":
        if explore is not None:
            self.explore = explore
        if exploration_config is not None:
            self.exploration_config = dict(exploration_config)
        return self

    def offline_data(self, *, input_=None, shuffle_buffer_size=None, output=None, output_compress_columns=None,
                     output_max_file_size=None, off_policy_estimation_methods=None, **kw) -> "AlgorithmConfig":
        if input_ is not None:
            self.input_ = input_
        if shuffle_buffer_size is not None:
            self.shuffle_buffer_size = shuffle_buffer_size
        if output is not None:
            self.output = output
        if output_compress_columns is not None:
            self.output_compress_columns = list(output_compress_columns)
        if output_max_file_size is not None:
            self.output_max_file_size = output_max_file_size
        if off_policy_estimation_methods is not None:
            self.off_policy_estimation_methods = dict(off_policy_estimation_methods)
        return self

    def multi_agent(self, *, policies=None, policy_mapping_fn=None, policies_to_train=None,
                    **kw) -> "AlgorithmConfig":
        if policies is not None:
            self.multiagent["policies"] = policies
        if policy_mapping_fn is not None:
            self.multiagent["policy_mapping_fn"] = policy_mapping_fn
        if policies_to_train is not None:
            self.multiagent["policies_to_train"] = list(policies_to_train)
        return self

    def is_multi_agent(self) -> bool:
        return bool(self.multiagent.get("policies"))

    def fault_tolerance(self, *, recreate_failed_workers=None, **kw) -> "AlgorithmConfig":
        if recreate_failed_workers is not None:
            self.recreate_failed_workers = recreate_failed_workers
        return self

    # ---- conversion
    def to_dict(self) -> Dict[str, Any]:
        d = {k: copy.deepcopy(v) for k, v in self.__dict__.items() if k != "algo_class"}
        d["framework"] = d.pop("framework_str")
        d["callbacks"] = d.pop("callbacks_class")
        d["input"] = d.pop("input_", "sampler")
        if d.get("lambda_", d.get("lambda")) is not None:
            d["lambda"] = d.get("lambda_", d.get("lambda"))
        return d

    def update_from_dict(self, d: Dict[str, Any]) -> "AlgorithmConfig":
        for k, v in d.items():
            if k == "framework":
                self.framework_str = v
            elif k == "callbacks":
                self.callbacks_class = v
            elif k == "lambda":
                self.lambda_ = v
            elif k == "input":
                self.input_ = v
            elif k == "model":
                self.model = {**self.model, **v}
            else:
                setattr(self, k, v)
        return self

    def copy(self) -> "AlgorithmConfig":
        return copy.deepcopy(self)

    def build(self, env=None, logger_creator=None):
        if env is not None:
            self.env = env
        if self.algo_class is None:
            raise ValueError("AlgorithmConfig has no algorithm class to build")
        return self.algo_class(config=self)

    def __getitem__(self, k):
        return self.to_dict()[k]

    def get(self, k, default=None):
        return self.to_dict().get(k, default)
