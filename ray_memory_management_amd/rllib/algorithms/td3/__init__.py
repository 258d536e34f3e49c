"""TD3: DDPG with twin critics (clipped double-Q), delayed actor/target updates and target-policy
smoothing. Parity: reference rllib/algorithms/td3/td3.py (TD3Config = DDPGConfig with twin_q,
policy_delay=2, smooth_target_policy, Gaussian exploration after 10k random steps, tau 5e-3,
l2_reg 0, train_batch_size 100). Runs on the DDPG learner (`ddpg.DDPGLearner`)."""
from __future__ import annotations

from ray_memory_management_amd.rllib.algorithms.ddpg import DDPG, DDPGConfig


class TD3Config(DDPGConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or TD3)
        self.twin_q = True
        self.policy_delay = 2
        self.smooth_target_policy = True
        self.target_noise = 0.2
        self.target_noise_clip = 0.5
        self.l2_reg = 0.0
        self.tau = 5e-3
        self.train_batch_size = 100
        self.replay_buffer_config = {**self.replay_buffer_config, "capacity": 1000000}
        self.num_steps_sampled_before_learning_starts = 10000
        self.exploration_config = {"type": "GaussianNoise", "random_timesteps": 10000, "stddev": 0.1,
                                   "initial_scale": 1.0, "final_scale": 1.0, "scale_timesteps": 1}


class TD3(DDPG):
    _config_class = TD3Config


DEFAULT_CONFIG = TD3Config().to_dict()
