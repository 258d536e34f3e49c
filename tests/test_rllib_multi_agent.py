"""Multi-agent RLlib on CPU: MultiAgentEnv API, make_multi_agent, policy_mapping_fn, per-policy
batches and learners, policies_to_train. Mirrors reference rllib/tests/test_multi_agent_env.py and
rllib/examples/multi_agent_cartpole.py."""
import numpy as np
import pytest
import torch


def test_make_multi_agent_env_api():
    from ray_memory_management_amd.rllib.env import MultiAgentCartPole, MultiAgentEnv

    env = MultiAgentCartPole({"num_agents": 3})
    assert isinstance(env, MultiAgentEnv) and env.get_agent_ids() == {0, 1, 2}
    obs = env.reset(seed=0)
    assert set(obs) == {0, 1, 2} and obs[0].shape == (4,)
    o, r, d, i = env.step({0: 1, 1: 0, 2: 1})
    assert set(r) == {0, 1, 2} and d["__all__"] is False


def test_multi_agent_worker_batches_per_policy(ray_shared):
    from ray_memory_management_amd.rllib.evaluation.multi_agent_worker import MultiAgentRolloutWorker

    cfg = {"env": "MultiAgentCartPole-v0", "env_config": {"num_agents": 4}, "rollout_fragment_length": 50,
           "model": {"fcnet_hiddens": [16]}, "gamma": 0.99, "lambda": 1.0,
           "multiagent": {"policies": {"even", "odd"},
                          "policy_mapping_fn": lambda aid, episode=None, worker=None, **kw: "even" if aid % 2 == 0
                          else "odd"}}
    w = MultiAgentRolloutWorker(None, cfg, 0, 0, seed=0)
    mb = w.sample()
    assert mb.env_steps() == 50 and set(mb.policy_batches) == {"even", "odd"}
    # every env step of every live agent lands in its policy's batch
    assert mb.agent_steps() <= 4 * 50 and mb.policy_batches["even"].count > 0
    b = mb.policy_batches["odd"]
    assert set(np.unique(b["agent_index"])) <= {hash(1) & 0x7FFFFFFF, hash(3) & 0x7FFFFFFF}
    assert np.isfinite(b["advantages"]).all() and b["obs"].shape[1] == 4
    wts = w.get_weights()
    assert set(wts) == {"even", "odd"}


@pytest.mark.parametrize("algo", ["PPO", "PG"])
def test_multi_agent_cartpole_learns_two_policies(ray_shared, algo):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    cls = get_algorithm_class(algo)
    cfg = (cls.get_default_config().environment("MultiAgentCartPole-v0", env_config={"num_agents": 2})
           .rollouts(num_rollout_workers=1, rollout_fragment_length=200)
           .training(lr=1e-3 if algo == "PPO" else 4e-3, train_batch_size=800, model={"fcnet_hiddens": [32]})
           .multi_agent(policies={"p0": None, "p1": None, "frozen": None},
                        policy_mapping_fn=lambda aid, episode=None, worker=None, **kw: ["p0", "p1"][aid],
                        policies_to_train=["p0", "p1"])
           .debugging(seed=0))
    if algo == "PPO":
        cfg.training(sgd_minibatch_size=128, num_sgd_iter=6, vf_loss_coeff=0.01)
    algo_ = cfg.build()
    frozen0 = {k: v.clone() for k, v in algo_.get_policy("frozen").get_weights().items()}
    best, want = 0.0, (120 if algo == "PPO" else 80)  # a random policy pair scores about 44
    for _ in range(30):
        r = algo_.train()
        best = max(best, r["episode_reward_mean"])  # summed over both agents
        if best > want:
            break
    assert best > want, best
    assert set(r["info"]["learner"]) == {"p0", "p1"}
    assert r["info"]["num_agent_steps_trained"] > r["num_env_steps_trained"]
    for k, v in algo_.get_policy("frozen").get_weights().items():
        assert torch.equal(v, frozen0[k])  # not in policies_to_train
    a = algo_.compute_single_action(np.zeros(4, np.float32), policy_id="p1")
    assert int(a) in (0, 1)
    algo_.stop()


def test_multi_agent_rejected_by_single_agent_algos(ray_shared):
    from ray_memory_management_amd.rllib.algorithms.dqn import DQNConfig

    with pytest.raises(ValueError, match="multi-agent"):
        DQNConfig().environment("MultiAgentCartPole-v0").multi_agent(policies={"a"}).build()
