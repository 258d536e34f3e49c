"""AlphaZero: MCTS finds the rewarding action sequence with an untrained network, ranked rewards
map returns to +/-1, and the algorithm trains through rollout-worker self-play. Mirrors reference
rllib/algorithms/alpha_zero/tests/test_alpha_zero.py (compilation) plus search invariants."""
import numpy as np
import pytest

from ray_memory_management_amd.rllib.env import Discrete, Box


class ChainEnv:
    """Pick action 1 three times in a row to earn 1 at the end; anything else ends with 0."""

    def __init__(self, config=None):
        self.observation_space = Box(0.0, 3.0, shape=(2,), dtype=np.float32)
        self.action_space = Discrete(2)
        self.t, self.ok = 0, True

    def _obs(self):
        return np.array([self.t, float(self.ok)], np.float32)

    def reset(self, *, seed=None):
        self.t, self.ok = 0, True
        return self._obs()

    def step(self, a):
        self.ok = self.ok and int(a) == 1
        self.t += 1
        done = self.t >= 3
        return self._obs(), (1.0 if done and self.ok else 0.0), done, {}

    def get_state(self):
        return (self.t, self.ok)

    def set_state(self, s):
        self.t, self.ok = s
        return self._obs()


def test_mcts_finds_rewarding_path_with_untrained_net():
    from ray_memory_management_amd.rllib.algorithms.alpha_zero import MCTS, Node, PolicyValueNet

    env = ChainEnv()
    net = PolicyValueNet(2, 2, (8,))
    for p in net.parameters():  # uniform priors, zero values
        p.data.zero_()
    rng = np.random.default_rng(0)
    tree = MCTS(net, env, {"num_simulations": 60, "add_dirichlet_noise": False, "argmax_tree_policy": True,
                           "puct_coefficient": 1.0}, rng)
    o = env.reset()
    root = Node(env.get_state(), o, 0.0, False, None, None, 2)
    path = []
    for _ in range(3):
        pi, a = tree.search(root)
        path.append(a)
        root = tree._child(root, a)
        root.parent = None
    assert path == [1, 1, 1] and root.reward == 1.0


def test_ranked_rewards():
    from ray_memory_management_amd.rllib.algorithms.alpha_zero import RankedRewards

    rr = RankedRewards(75, rng=np.random.default_rng(0))
    for r in range(100):
        rr.add(float(r))
    assert rr.normalize(90.0) == 1.0 and rr.normalize(10.0) == -1.0 and rr.normalize(74.25) in (-1.0, 1.0)


def test_alpha_zero_trains_with_worker_self_play(ray_shared):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    cls = get_algorithm_class("AlphaZero")
    cfg = (cls.get_default_config().environment("CartPoleSparseRewards-v1")
           .rollouts(num_rollout_workers=2)
           .training(lr=1e-3, num_sgd_iter=5, sgd_minibatch_size=64, model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    cfg.mcts_config = {**cfg.mcts_config, "num_simulations": 8}
    cfg.ranked_rewards = {**cfg.ranked_rewards, "initialize_buffer": 2}
    a = cfg.build()
    for _ in range(3):
        r = a.train()
    st = r["info"]["learner"]["default_policy"]["learner_stats"]
    assert np.isfinite(st["policy_loss"]) and np.isfinite(st["value_loss"])
    assert r["episodes_total"] >= 6 and r["num_env_steps_sampled"] > 0
    assert a.compute_single_action(np.zeros(4, np.float32)) in (0, 1)
    a.stop()
