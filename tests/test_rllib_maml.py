"""MAML on a task-settable goal bandit: meta-training makes one inner policy-gradient step adapt
better (reference rllib/algorithms/maml/tests/test_maml.py checks compilation; this also checks
the meta-learning effect and the differentiable inner step)."""
import numpy as np
import torch


def test_inner_step_is_differentiable():
    from ray_memory_management_amd.rllib.algorithms.maml import GaussianPolicyNet, _pg_loss

    net = GaussianPolicyNet(1, 1, (4,))
    params = dict(net.named_parameters())
    b = {"obs": torch.ones(6, 1), "actions": torch.randn(6, 1), "returns": torch.randn(6)}
    loss = _pg_loss(net, params, b)
    g = torch.autograd.grad(loss, list(params.values()), create_graph=True)
    adapted = {k: v - 0.1 * gi for (k, v), gi in zip(params.items(), g)}
    outer = _pg_loss(net, adapted, b)
    outer.backward()  # second-order path through the inner update
    assert all(p.grad is not None for p in net.parameters())


def test_maml_meta_training_improves_adaptation(ray_shared):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    torch.set_num_threads(2)
    a = (get_algorithm_class("MAML").get_default_config().environment("GoalBandit-v0")
         .rollouts(num_rollout_workers=2).training(lr=1e-2, inner_lr=0.2, episodes_per_task=20)
         .debugging(seed=0)).build()
    _, post0 = a.adaptation_gain(n_tasks=8)
    for _ in range(40):
        r = a.train()
    pre1, post1 = a.adaptation_gain(n_tasks=8)
    st = r["info"]["learner"]["default_policy"]["learner_stats"]
    assert np.isfinite(st["meta_loss"])
    assert post1 > pre1 and post1 > post0, (post0, pre1, post1)
    a.stop()
