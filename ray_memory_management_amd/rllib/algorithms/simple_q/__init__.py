"""SimpleQ: plain Q-learning with a target network and a uniform replay buffer (no double-Q, no
dueling, no prioritisation). Parity: reference rllib/algorithms/simple_q/simple_q.py
(SimpleQConfig defaults) and simple_q_torch_policy.py; runs on the DQN learner."""
from __future__ import annotations

from ray_memory_management_amd.rllib.algorithms.dqn import DQN, DQNConfig


class SimpleQConfig(DQNConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or SimpleQ)
        self.double_q = False
        self.dueling = False
        self.replay_buffer_config = {"type": "MultiAgentReplayBuffer", "capacity": 50000}
        self.grad_clip = None


class SimpleQ(DQN):
    _config_class = SimpleQConfig


DEFAULT_CONFIG = SimpleQConfig().to_dict()
