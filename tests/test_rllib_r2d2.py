"""R2D2 on CPU. Mirrors reference rllib/algorithms/r2d2/tests/test_r2d2.py (compilation + learning)
plus invariants: value rescaling is invertible, the unroll resets state after done, sequence rows
carry their start state."""
import numpy as np
import pytest
import torch


def test_h_function_inverse():
    from ray_memory_management_amd.rllib.algorithms.r2d2 import h_function, h_inverse

    x = torch.linspace(-500, 500, 1001, dtype=torch.float64)
    torch.testing.assert_close(h_inverse(h_function(x)), x, rtol=1e-6, atol=1e-6)


def test_unroll_resets_state_after_done():
    from ray_memory_management_amd.rllib.algorithms.r2d2 import RecurrentQModel

    torch.manual_seed(0)
    m = RecurrentQModel(3, 2, (8,), 8)
    obs = torch.randn(1, 6, 3)
    resets = torch.tensor([[0, 0, 0, 1, 0, 0]], dtype=torch.float32)
    q = m.unroll(obs, m.initial_state(1), resets)
    q_fresh = m.unroll(obs[:, 3:], m.initial_state(1), torch.zeros(1, 3))
    torch.testing.assert_close(q[:, 3:], q_fresh)  # a reset makes step 3 independent of the past
    q_noreset = m.unroll(obs, m.initial_state(1), torch.zeros(1, 6))
    assert not torch.allclose(q_noreset[:, 3:], q_fresh)


def test_r2d2_learns_cartpole(ray_shared):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class
    from ray_memory_management_amd.rllib.algorithms.r2d2 import R2D2Config

    assert get_algorithm_class("R2D2").__name__ == "R2D2"
    cfg = (R2D2Config().environment("CartPole-v1")
           .rollouts(num_rollout_workers=0, num_envs_per_worker=8)
           .training(lr=1e-3, train_batch_size=32, replay_sequence_length=10, burn_in=2,
                     target_network_update_freq=1000, num_steps_sampled_before_learning_starts=500,
                     training_intensity=4, model={"fcnet_hiddens": [64], "lstm_cell_size": 32},
                     replay_buffer_config={"capacity": 40000})
           .exploration(exploration_config={"initial_epsilon": 1.0, "final_epsilon": 0.02, "epsilon_timesteps": 4000})
           .reporting(min_sample_timesteps_per_iteration=800)
           .debugging(seed=0))
    algo = cfg.build()
    b = algo._sample()
    assert b["obs_seq"].shape == (8, 11, 4) and b["act_seq"].shape == (8, 10) and b["state_h"].shape == (8, 32)
    best = 0.0
    for _ in range(40):
        r = algo.train()
        best = max(best, r["episode_reward_mean"])
        if best > 100:
            break
    assert best > 100, best
    assert r["info"]["num_target_updates"] >= 1
    algo.stop()
