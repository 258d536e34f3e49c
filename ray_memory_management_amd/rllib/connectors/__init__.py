"""Connectors: composable transforms between env and policy.

Parity: reference rllib/connectors/{connector.py (ConnectorContext, Connector to_state /
from_state, AgentConnector / ActionConnector, ConnectorPipeline remove / insert_before /
insert_after / prepend / append / __getitem__, register_connector / get_connector),
agent/{clip_reward,obs_preproc,lambdas,pipeline,state_buffer,view_requirement}.py,
action/{clip,normalize,immutable,lambdas,pipeline}.py, util.py (build connectors from a policy
config and restore them from saved state)}.

Agent connectors map env outputs (per env / agent dicts) to policy inputs; action connectors map
policy outputs back to env actions. Each is serialisable as (name, params) so a policy's
pipeline is restored identically in another process (e.g. a Serve replica)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple, Type, Union

import numpy as np


@dataclass
class ConnectorContext:
    config: Dict = field(default_factory=dict)
    initial_states: List = field(default_factory=list)
    observation_space: Any = None
    action_space: Any = None
    view_requirements: Dict = field(default_factory=dict)
    is_policy_recurrent: bool = False

    @staticmethod
    def from_policy(policy) -> "ConnectorContext":
        return ConnectorContext(config=dict(getattr(policy, "config", {}) or {}),
                                observation_space=policy.observation_space, action_space=policy.action_space)


@dataclass
class AgentConnectorDataType:
    env_id: Any
    agent_id: Any
    data: Any


@dataclass
class ActionConnectorDataType:
    env_id: Any
    agent_id: Any
    input_dict: Dict
    output: Tuple  # (actions, state_outs, extra_fetches)


_REGISTRY: Dict[str, Type["Connector"]] = {}


def register_connector(name: str, cls: Type["Connector"]) -> None:
    if not issubclass(cls, Connector):
        raise TypeError(f"{cls} is not a Connector")
    _REGISTRY[name] = cls


def get_connector(ctx: ConnectorContext, name: str, params) -> "Connector":
    if name not in _REGISTRY:
        raise NameError(f"connector {name!r} is not registered")
    return _REGISTRY[name].from_state(ctx, params)


class Connector:
    def __init__(self, ctx: ConnectorContext):
        self.ctx = ctx
        self._is_training = True

    def in_training(self) -> None:
        self._is_training = True

    def in_eval(self) -> None:
        self._is_training = False

    def is_training(self, is_training: bool) -> None:
        self._is_training = is_training

    def __str__(self, indentation: int = 0) -> str:
        return " " * indentation + type(self).__name__

    def to_state(self) -> Tuple[str, Any]:
        return type(self).__name__, None

    @classmethod
    def from_state(cls, ctx: ConnectorContext, params) -> "Connector":
        return cls(ctx)


class AgentConnector(Connector):
    def reset(self, env_id) -> None:
        pass

    def on_policy_output(self, output: ActionConnectorDataType) -> None:
        pass

    def __call__(self, acd_list: List[AgentConnectorDataType]) -> List[AgentConnectorDataType]:
        return [self.transform(d) for d in acd_list]

    def transform(self, ac_data: AgentConnectorDataType) -> AgentConnectorDataType:
        raise NotImplementedError


class ActionConnector(Connector):
    def __call__(self, ac_data: ActionConnectorDataType) -> ActionConnectorDataType:
        return self.transform(ac_data)

    def transform(self, ac_data: ActionConnectorDataType) -> ActionConnectorDataType:
        raise NotImplementedError


class ConnectorPipeline:
    connectors: List[Connector]

    def _index(self, key) -> int:
        for i, c in enumerate(self.connectors):
            if (isinstance(key, str) and type(c).__name__ == key) or (isinstance(key, type) and isinstance(c, key)):
                return i
        raise KeyError(key)

    def remove(self, name: str) -> None:
        try:
            del self.connectors[self._index(name)]
        except KeyError:
            pass

    def insert_before(self, name: str, connector: Connector) -> None:
        self.connectors.insert(self._index(name), connector)

    def insert_after(self, name: str, connector: Connector) -> None:
        self.connectors.insert(self._index(name) + 1, connector)

    def prepend(self, connector: Connector) -> None:
        self.connectors.insert(0, connector)

    def append(self, connector: Connector) -> None:
        self.connectors.append(connector)

    def __getitem__(self, key: Union[str, int, type]):
        if isinstance(key, int):
            return self.connectors[key]
        return [c for c in self.connectors
                if (isinstance(key, str) and type(c).__name__ == key) or (isinstance(key, type) and isinstance(c, key))]

    def __str__(self, indentation: int = 0) -> str:
        return "\n".join([" " * indentation + type(self).__name__] +
                         [c.__str__(indentation + 4) for c in self.connectors])

    def in_training(self):
        for c in self.connectors:
            c.in_training()

    def in_eval(self):
        for c in self.connectors:
            c.in_eval()

    def to_state(self):
        return type(self).__name__, [c.to_state() for c in self.connectors]

    @classmethod
    def from_state(cls, ctx, params):
        return cls(ctx, [get_connector(ctx, n, p) for n, p in params])


class AgentConnectorPipeline(ConnectorPipeline, AgentConnector):
    def __init__(self, ctx: ConnectorContext, connectors: List[Connector]):
        AgentConnector.__init__(self, ctx)
        self.connectors = list(connectors)

    def reset(self, env_id):
        for c in self.connectors:
            c.reset(env_id)

    def on_policy_output(self, output):
        for c in self.connectors:
            c.on_policy_output(output)

    def __call__(self, acd_list):
        for c in self.connectors:
            acd_list = c(acd_list)
        return acd_list


class ActionConnectorPipeline(ConnectorPipeline, ActionConnector):
    def __init__(self, ctx: ConnectorContext, connectors: List[Connector]):
        ActionConnector.__init__(self, ctx)
        self.connectors = list(connectors)

    def __call__(self, ac_data):
        for c in self.connectors:
            ac_data = c(ac_data)
        return ac_data


# --- agent connectors --------------------------------------------------------------------------
class ClipRewardAgentConnector(AgentConnector):
    """Clip (or sign) the reward in each env-output dict."""

    def __init__(self, ctx, sign: bool = False, limit: Optional[float] = None):
        super().__init__(ctx)
        if sign and limit:
            raise ValueError("ClipRewardAgentConnector: sign and limit are exclusive")
        self.sign, self.limit = sign, limit

    def transform(self, ac_data):
        d = dict(ac_data.data)
        if "rewards" in d:
            r = d["rewards"]
            d["rewards"] = float(np.sign(r)) if self.sign else float(np.clip(r, -self.limit, self.limit)) \
                if self.limit else r
        return AgentConnectorDataType(ac_data.env_id, ac_data.agent_id, d)

    def to_state(self):
        return type(self).__name__, {"sign": self.sign, "limit": self.limit}

    @classmethod
    def from_state(cls, ctx, params):
        return cls(ctx, **(params or {}))


class ObsPreprocessorConnector(AgentConnector):
    """Apply the policy's observation preprocessing (here: flatten Box observations to float32,
    one-hot Discrete observations) to `obs` / `new_obs`."""

    def _prep(self, o):
        space = self.ctx.observation_space
        n = getattr(space, "n", None)
        if n is not None and np.ndim(o) == 0:
            v = np.zeros(n, dtype=np.float32)
            v[int(o)] = 1.0
            return v
        return np.asarray(o, dtype=np.float32).reshape(-1)

    def transform(self, ac_data):
        d = dict(ac_data.data)
        for k in ("obs", "new_obs"):
            if k in d:
                d[k] = self._prep(d[k])
        return AgentConnectorDataType(ac_data.env_id, ac_data.agent_id, d)


class MeanStdObservationFilterAgentConnector(AgentConnector):
    """Running mean/std normalisation of observations (Welford; frozen in eval mode)."""

    def __init__(self, ctx, clip: float = 10.0):
        super().__init__(ctx)
        self.clip, self.n, self.mean, self.m2 = clip, 0, None, None

    def transform(self, ac_data):
        d = dict(ac_data.data)
        if "obs" in d:
            x = np.asarray(d["obs"], dtype=np.float64)
            if self.mean is None:
                self.mean, self.m2 = np.zeros_like(x), np.zeros_like(x)
            if self._is_training:
                self.n += 1
                delta = x - self.mean
                self.mean += delta / self.n
                self.m2 += delta * (x - self.mean)
            std = np.sqrt(self.m2 / max(self.n - 1, 1)) + 1e-8 if self.n > 1 else np.ones_like(x)
            d["obs"] = np.clip((x - self.mean) / std, -self.clip, self.clip).astype(np.float32)
        return AgentConnectorDataType(ac_data.env_id, ac_data.agent_id, d)

    def to_state(self):
        return type(self).__name__, {"clip": self.clip, "n": self.n,
                                     "mean": None if self.mean is None else self.mean.tolist(),
                                     "m2": None if self.m2 is None else self.m2.tolist()}

    @classmethod
    def from_state(cls, ctx, params):
        c = cls(ctx, params["clip"])
        c.n = params["n"]
        c.mean = None if params["mean"] is None else np.asarray(params["mean"])
        c.m2 = None if params["m2"] is None else np.asarray(params["m2"])
        return c


class ViewRequirementAgentConnector(AgentConnector):
    """Keep per-(env, agent) history and emit the policy's input view: the current obs plus the
    previous action / reward (reference view_requirement.py, the common subset)."""

    def __init__(self, ctx):
        super().__init__(ctx)
        self._hist: Dict[Tuple, Dict] = {}

    def reset(self, env_id):
        for k in [k for k in self._hist if k[0] == env_id]:
            del self._hist[k]

    def transform(self, ac_data):
        key = (ac_data.env_id, ac_data.agent_id)
        h = self._hist.setdefault(key, {"prev_actions": 0, "prev_rewards": 0.0, "t": -1})
        d = dict(ac_data.data)
        h["t"] += 1
        view = {"obs": d.get("obs"), "prev_actions": h["prev_actions"], "prev_rewards": h["prev_rewards"],
                "t": h["t"], "agent_index": ac_data.agent_id, "env_id": ac_data.env_id}
        if "rewards" in d:
            h["prev_rewards"] = d["rewards"]
        d["view"] = view
        return AgentConnectorDataType(ac_data.env_id, ac_data.agent_id, d)

    def on_policy_output(self, output: ActionConnectorDataType):
        h = self._hist.get((output.env_id, output.agent_id))
        if h is not None:
            h["prev_actions"] = output.output[0]


class LambdaAgentConnector(AgentConnector):
    fn: Callable = staticmethod(lambda data: data)

    def transform(self, ac_data):
        return AgentConnectorDataType(ac_data.env_id, ac_data.agent_id, type(self).fn(ac_data.data))


def register_lambda_agent_connector(name: str, fn: Callable[[Any], Any]) -> Type[AgentConnector]:
    cls = type(name, (LambdaAgentConnector,), {"fn": staticmethod(fn)})
    register_connector(name, cls)
    return cls


FlattenDataAgentConnector = register_lambda_agent_connector(
    "FlattenDataAgentConnector",
    lambda data: {k: (np.asarray(v).reshape(-1) if isinstance(v, (np.ndarray, list)) else v) for k, v in data.items()})


# --- action connectors -------------------------------------------------------------------------
class ConvertToNumpyConnector(ActionConnector):
    def transform(self, ac_data):
        a, s, e = ac_data.output
        conv = (lambda x: x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x))
        return ActionConnectorDataType(ac_data.env_id, ac_data.agent_id, ac_data.input_dict,
                                       (conv(a), [conv(x) for x in s], {k: conv(v) for k, v in e.items()}))


class ClipActionsConnector(ActionConnector):
    def transform(self, ac_data):
        a, s, e = ac_data.output
        sp = self.ctx.action_space
        if hasattr(sp, "low"):
            a = np.clip(a, sp.low, sp.high)
        return ActionConnectorDataType(ac_data.env_id, ac_data.agent_id, ac_data.input_dict, (a, s, e))


class NormalizeActionsConnector(ActionConnector):
    """Map policy actions in [-1, 1] to the Box action space's [low, high]."""

    def transform(self, ac_data):
        a, s, e = ac_data.output
        sp = self.ctx.action_space
        if hasattr(sp, "low"):
            a = sp.low + (np.clip(a, -1.0, 1.0) + 1.0) * 0.5 * (sp.high - sp.low)
        return ActionConnectorDataType(ac_data.env_id, ac_data.agent_id, ac_data.input_dict, (a, s, e))


class ImmutableActionsConnector(ActionConnector):
    def transform(self, ac_data):
        a, s, e = ac_data.output
        if isinstance(a, np.ndarray):
            a = a.copy()
            a.setflags(write=False)
        return ActionConnectorDataType(ac_data.env_id, ac_data.agent_id, ac_data.input_dict, (a, s, e))


for _c in (AgentConnectorPipeline, ActionConnectorPipeline, ClipRewardAgentConnector, ObsPreprocessorConnector,
           MeanStdObservationFilterAgentConnector, ViewRequirementAgentConnector, ConvertToNumpyConnector,
           ClipActionsConnector, NormalizeActionsConnector, ImmutableActionsConnector):
    register_connector(_c.__name__, _c)


# --- util (reference connectors/util.py) -------------------------------------------------------
def get_agent_connectors_from_config(ctx: ConnectorContext, config: Dict) -> AgentConnectorPipeline:
    cs: List[Connector] = []
    if config.get("clip_rewards") is True:
        cs.append(ClipRewardAgentConnector(ctx, sign=True))
    elif isinstance(config.get("clip_rewards"), (int, float)) and config.get("clip_rewards"):
        cs.append(ClipRewardAgentConnector(ctx, limit=abs(float(config["clip_rewards"]))))
    if config.get("observation_filter") == "MeanStdFilter":
        cs.append(MeanStdObservationFilterAgentConnector(ctx))
    if config.get("preprocessor_pref", "deepmind") is not None:
        cs.append(ObsPreprocessorConnector(ctx))
    cs.append(ViewRequirementAgentConnector(ctx))
    return AgentConnectorPipeline(ctx, cs)


def get_action_connectors_from_config(ctx: ConnectorContext, config: Dict) -> ActionConnectorPipeline:
    cs: List[Connector] = [ConvertToNumpyConnector(ctx)]
    if config.get("normalize_actions", False):
        cs.append(NormalizeActionsConnector(ctx))
    if config.get("clip_actions", False):
        cs.append(ClipActionsConnector(ctx))
    cs.append(ImmutableActionsConnector(ctx))
    return ActionConnectorPipeline(ctx, cs)


def create_connectors_for_policy(policy, config: Dict) -> None:
    ctx = ConnectorContext.from_policy(policy)
    policy.agent_connectors = get_agent_connectors_from_config(ctx, config)
    policy.action_connectors = get_action_connectors_from_config(ctx, config)


def restore_connectors_for_policy(policy, connector_config: Tuple[str, Any]) -> ConnectorPipeline:
    name, params = connector_config
    return get_connector(ConnectorContext.from_policy(policy), name, params)
