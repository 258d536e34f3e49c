"""Connectors. Mirrors reference rllib/connectors/tests/{test_connector.py, test_agent.py,
test_action.py}: pipelines (insert / remove / lookup), serialisation round trip through
to_state / get_connector, reward clipping, obs preprocessing, view requirements fed by policy
outputs, action normalisation / clipping / immutability, connectors built from a policy config."""
import numpy as np
import pytest

from ray_memory_management_amd.rllib import connectors as C
from ray_memory_management_amd.rllib.env import Box, Discrete


def _ctx():
    return C.ConnectorContext(observation_space=Box(-1, 1, shape=(2, 2), dtype=np.float32),
                              action_space=Box(-2.0, 2.0, shape=(2,), dtype=np.float32))


def test_agent_pipeline_and_state_round_trip():
    ctx = _ctx()
    p = C.AgentConnectorPipeline(ctx, [C.ClipRewardAgentConnector(ctx, limit=1.0), C.ObsPreprocessorConnector(ctx)])
    p.append(C.ViewRequirementAgentConnector(ctx))
    p.insert_before("ObsPreprocessorConnector", C.MeanStdObservationFilterAgentConnector(ctx))
    assert [type(c).__name__ for c in p.connectors] == ["ClipRewardAgentConnector",
                                                        "MeanStdObservationFilterAgentConnector",
                                                        "ObsPreprocessorConnector", "ViewRequirementAgentConnector"]
    out = p([C.AgentConnectorDataType(0, "a", {"obs": np.ones((2, 2)), "rewards": 5.0})])
    d = out[0].data
    assert d["rewards"] == 1.0 and d["obs"].shape == (4,) and d["view"]["t"] == 0
    p.on_policy_output(C.ActionConnectorDataType(0, "a", {}, (np.array([0.3, 0.1]), [], {})))
    d2 = p([C.AgentConnectorDataType(0, "a", {"obs": np.zeros((2, 2)), "rewards": -3.0})])[0].data
    assert d2["view"]["prev_rewards"] == 1.0 and np.allclose(d2["view"]["prev_actions"], [0.3, 0.1])
    p.reset(0)
    name, params = p.to_state()
    q = C.get_connector(ctx, name, params)
    assert [type(c).__name__ for c in q.connectors] == [type(c).__name__ for c in p.connectors]
    assert q[C.MeanStdObservationFilterAgentConnector][0].n == 2
    p.remove("ViewRequirementAgentConnector")
    assert len(p.connectors) == 3 and p[0].limit == 1.0


def test_action_connectors_and_config_factory():
    import torch

    ctx = _ctx()
    acts = C.get_action_connectors_from_config(ctx, {"normalize_actions": True, "clip_actions": True})
    out = acts(C.ActionConnectorDataType(0, "a", {}, (torch.tensor([1.0, -3.0]), [], {"vf": torch.tensor(0.5)})))
    a = out.output[0]
    assert isinstance(a, np.ndarray) and np.allclose(a, [2.0, -2.0]) and not a.flags.writeable
    agents = C.get_agent_connectors_from_config(ctx, {"clip_rewards": True, "observation_filter": "MeanStdFilter"})
    d = agents([C.AgentConnectorDataType(1, 0, {"obs": np.ones((2, 2)), "rewards": -0.2})])[0].data
    assert d["rewards"] == -1.0
    disc = C.ObsPreprocessorConnector(C.ConnectorContext(observation_space=Discrete(3)))
    assert disc([C.AgentConnectorDataType(0, 0, {"obs": 2})])[0].data["obs"].tolist() == [0, 0, 1]


def test_lambda_connector_registry():
    cls = C.register_lambda_agent_connector("DoubleObs", lambda d: {**d, "obs": d["obs"] * 2})
    ctx = _ctx()
    c = C.get_connector(ctx, "DoubleObs", None)
    assert isinstance(c, cls) and c([C.AgentConnectorDataType(0, 0, {"obs": 3})])[0].data["obs"] == 6
    with pytest.raises(NameError):
        C.get_connector(ctx, "Nope", None)


def test_connectors_attach_to_policy():
    from ray_memory_management_amd.rllib.env import CartPoleEnv
    from ray_memory_management_amd.rllib.policy import TorchPolicy

    env = CartPoleEnv()
    pol = TorchPolicy(env.observation_space, env.action_space, {})
    C.create_connectors_for_policy(pol, {"clip_rewards": 1.0})
    obs = pol.agent_connectors([C.AgentConnectorDataType(0, 0, {"obs": env.reset(), "rewards": 3.0})])[0]
    a, s, e = pol.compute_actions([obs.data["obs"]])
    out = pol.action_connectors(C.ActionConnectorDataType(0, 0, obs.data, (a, s, e)))
    assert out.output[0][0] in (0, 1) and obs.data["rewards"] == 1.0
    restored = C.restore_connectors_for_policy(pol, pol.agent_connectors.to_state())
    assert len(restored.connectors) == len(pol.agent_connectors.connectors)
