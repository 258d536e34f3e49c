"""MB-MPO on a point mass with a known reward function: the dynamics ensemble fits the real
transitions and meta-policy optimisation in the learned models improves the REAL return.
Mirrors reference rllib/algorithms/mbmpo/tests/test_mbmpo.py (compilation) plus learning."""
import numpy as np
import torch


def test_ensemble_members_train_on_bootstraps():
    from ray_memory_management_amd.rllib.algorithms.mbmpo import DynamicsEnsemble

    e = DynamicsEnsemble(2, 1, k=3, hidden=8)
    out = e(torch.zeros(3, 4, 2), torch.zeros(3, 4, 1))
    assert out.shape == (3, 4, 2)
    assert not torch.allclose(e.W[0][0], e.W[0][1])  # independent members


def test_mbmpo_improves_real_return(ray_shared):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    torch.set_num_threads(2)
    a = get_algorithm_class("MBMPO").get_default_config().environment("PointMass-v0").debugging(seed=0).build()
    random_ret = float(np.mean([r for r, _ in a._episode_history]))
    rets = []
    for _ in range(8):
        st = a.train()["info"]["learner"]["default_policy"]["learner_stats"]
        rets.append(st["real_return"])
    assert st["dynamics_loss"] < 0.01
    assert np.mean(rets[-3:]) > random_ret + 3.0, (random_ret, rets)
    a.stop()
