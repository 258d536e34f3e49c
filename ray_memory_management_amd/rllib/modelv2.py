"""ModelV2 interface, the model catalog, preprocessors and torch action distributions.

Parity: reference rllib/models/{modelv2.py, torch/torch_modelv2.py, catalog.py (ModelCatalog,
MODEL_DEFAULTS), preprocessors.py, action_dist.py, torch/torch_action_dist.py}.

The built-in networks of this framework (``models.FullyConnectedNetwork`` / ``VisionNetwork``)
are plain ``nn.Module``s called as ``net(obs) -> (logits, value)`` — that is what the fused GPU
learners drive. ModelV2 is the user-facing extension point: a custom model registered with
``ModelCatalog.register_custom_model`` and named by ``config["model"]["custom_model"]`` is built
through ``build_model`` and wrapped (:class:`ModelV2Adapter`) so every algorithm's CPU/torch path
runs it; ``ModelCatalog.get_model_v2`` conversely wraps the built-in networks as ModelV2s
(``forward(input_dict, state, seq_lens)`` / ``value_function()``) for ModelV2-style code.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

# reference rllib/models/catalog.py MODEL_DEFAULTS (the keys users set in config["model"])
MODEL_DEFAULTS: Dict[str, Any] = {
    "_use_default_native_models": False,
    "_disable_preprocessor_api": False,
    "_disable_action_flattening": False,
    "fcnet_hiddens": [256, 256],
    "fcnet_activation": "tanh",
    "conv_filters": None,
    "conv_activation": "relu",
    "post_fcnet_hiddens": [],
    "post_fcnet_activation": "relu",
    "free_log_std": False,
    "no_final_linear": False,
    "vf_share_layers": True,
    "use_lstm": False,
    "max_seq_len": 20,
    "lstm_cell_size": 256,
    "lstm_use_prev_action": False,
    "lstm_use_prev_reward": False,
    "_time_major": False,
    "use_attention": False,
    "attention_num_transformer_units": 1,
    "attention_dim": 64,
    "attention_num_heads": 1,
    "attention_head_dim": 32,
    "attention_memory_inference": 50,
    "attention_memory_training": 50,
    "attention_position_wise_mlp_dim": 32,
    "attention_init_gru_gate_bias": 2.0,
    "attention_use_n_prev_actions": 0,
    "attention_use_n_prev_rewards": 0,
    "framestack": True,
    "dim": 84,
    "grayscale": False,
    "zero_mean": True,
    "custom_model": None,
    "custom_model_config": {},
    "custom_action_dist": None,
    "custom_preprocessor": None,
    "lstm_use_prev_action_reward": -1,
}


# ============================================================================ ModelV2
class ModelV2:
    """Model interface (reference rllib/models/modelv2.py): ``forward(input_dict, state,
    seq_lens) -> (outputs, state)`` plus ``value_function()`` for the last forward pass."""

    def __init__(self, obs_space, action_space, num_outputs: int, model_config: Dict, name: str,
                 framework: str = "torch"):
        self.obs_space, self.action_space = obs_space, action_space
        self.num_outputs = num_outputs
        self.model_config = model_config
        self.name = name or "default_model"
        self.framework = framework
        self.view_requirements = {"obs": None}
        self.time_major = bool(model_config.get("_time_major", False)) if model_config else False

    def get_initial_state(self) -> List[np.ndarray]:
        return []

    def forward(self, input_dict: Dict, state: List, seq_lens) -> Tuple[Any, List]:
        raise NotImplementedError

    def value_function(self):
        raise NotImplementedError

    def custom_loss(self, policy_loss, loss_inputs):
        return policy_loss

    def metrics(self) -> Dict:
        return {}

    def __call__(self, input_dict, state=None, seq_lens=None):
        if not isinstance(input_dict, dict):
            input_dict = {"obs": input_dict}
        if "obs_flat" not in input_dict and "obs" in input_dict:
            o = input_dict["obs"]
            if isinstance(o, torch.Tensor):
                input_dict = dict(input_dict, obs_flat=o.reshape(o.shape[0], -1).float())
        out, state_out = self.forward(input_dict, state or [], seq_lens)
        if not isinstance(state_out, (list, tuple)):
            raise ValueError(f"forward() must return (outputs, [state...]), got state {type(state_out)}")
        return out, list(state_out)

    def is_time_major(self) -> bool:
        return self.time_major

    def last_output(self):
        return getattr(self, "_last_output", None)

    def context(self):
        import contextlib

        return contextlib.nullcontext()

    def variables(self, as_dict: bool = False):
        return {}

    def trainable_variables(self, as_dict: bool = False):
        return self.variables(as_dict)


class TorchModelV2(ModelV2):
    """Torch ModelV2 (reference rllib/models/torch/torch_modelv2.py). Subclass as
    ``class MyModel(TorchModelV2, nn.Module)`` and call both constructors."""

    def __init__(self, obs_space, action_space, num_outputs, model_config, name):
        if not isinstance(self, nn.Module):
            raise ValueError("subclasses of TorchModelV2 must also subclass nn.Module, e.g. "
                             "`class MyModel(TorchModelV2, nn.Module)`")
        ModelV2.__init__(self, obs_space, action_space, num_outputs, model_config, name, framework="torch")

    def variables(self, as_dict: bool = False):
        p = dict(self.state_dict())
        return p if as_dict else list(p.values())

    def trainable_variables(self, as_dict: bool = False):
        p = {k: v for k, v in self.named_parameters() if v.requires_grad}
        return p if as_dict else list(p.values())


class ModelV2Adapter(nn.Module):
    """Presents a ModelV2 as this framework's ``net(obs) -> (logits, value)`` module."""

    def __init__(self, model: ModelV2):
        super().__init__()
        self.model_v2 = model  # an nn.Module ModelV2 registers as a submodule (its parameters train)

    def forward(self, obs):
        out, _ = self.model_v2({"obs": obs})
        v = self.model_v2.value_function()
        return out, v.reshape(-1)


class NativeModelV2(TorchModelV2, nn.Module):
    """One of the built-in networks exposed through the ModelV2 interface."""

    def __init__(self, net: nn.Module, obs_space, action_space, num_outputs, model_config, name):
        nn.Module.__init__(self)
        TorchModelV2.__init__(self, obs_space, action_space, num_outputs, model_config, name)
        self.net = net
        self._value = None

    def forward(self, input_dict, state, seq_lens):
        logits, v = self.net(input_dict["obs"])
        self._value = v
        self._last_output = logits
        return logits, state

    def value_function(self):
        if self._value is None:
            raise ValueError("value_function() called before forward()")
        return self._value.reshape(-1)


# ============================================================================ action distributions
class ActionDistribution:
    """reference rllib/models/action_dist.py."""

    def __init__(self, inputs, model=None):
        self.inputs, self.model = inputs, model

    def sample(self):
        raise NotImplementedError

    def deterministic_sample(self):
        raise NotImplementedError

    def sampled_action_logp(self):
        return self.logp(self.last_sample)

    def logp(self, x):
        raise NotImplementedError

    def kl(self, other):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    def multi_kl(self, other):
        return self.kl(other)

    def multi_entropy(self):
        return self.entropy()

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        raise NotImplementedError


class TorchDistributionWrapper(ActionDistribution):
    def __init__(self, inputs, model=None):
        if not isinstance(inputs, torch.Tensor):
            inputs = torch.as_tensor(np.asarray(inputs))
        super().__init__(inputs.float(), model)
        self.last_sample = None


class TorchCategorical(TorchDistributionWrapper):
    def __init__(self, inputs, model=None, temperature: float = 1.0):
        super().__init__(inputs, model)
        self.dist = torch.distributions.Categorical(logits=self.inputs / temperature)

    def sample(self):
        self.last_sample = self.dist.sample()
        return self.last_sample

    def deterministic_sample(self):
        self.last_sample = self.inputs.argmax(-1)
        return self.last_sample

    def logp(self, x):
        return self.dist.log_prob(torch.as_tensor(x).long())

    def entropy(self):
        return self.dist.entropy()

    def kl(self, other):
        return torch.distributions.kl.kl_divergence(self.dist, other.dist)

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        return int(action_space.n)


class TorchDiagGaussian(TorchDistributionWrapper):
    def __init__(self, inputs, model=None):
        super().__init__(inputs, model)
        mean, log_std = torch.chunk(self.inputs, 2, dim=-1)
        self.log_std = log_std
        self.dist = torch.distributions.Normal(mean, torch.exp(log_std))

    def sample(self):
        self.last_sample = self.dist.sample()
        return self.last_sample

    def deterministic_sample(self):
        self.last_sample = self.dist.mean
        return self.last_sample

    def logp(self, x):
        return self.dist.log_prob(torch.as_tensor(x).float()).sum(-1)

    def entropy(self):
        return self.dist.entropy().sum(-1)

    def kl(self, other):
        return torch.distributions.kl.kl_divergence(self.dist, other.dist).sum(-1)

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        return int(np.prod(action_space.shape)) * 2


class TorchDeterministic(TorchDistributionWrapper):
    def deterministic_sample(self):
        self.last_sample = self.inputs
        return self.inputs

    sample = deterministic_sample

    def logp(self, x):
        return torch.zeros(self.inputs.shape[0])

    def entropy(self):
        return torch.zeros(self.inputs.shape[0])

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        return int(np.prod(action_space.shape))


# ============================================================================ preprocessors
class Preprocessor:
    """reference rllib/models/preprocessors.py: fixed transform of raw observations."""

    def __init__(self, obs_space, options: Optional[Dict] = None):
        self._obs_space = obs_space
        self._options = options or {}
        self.shape = self._init_shape(obs_space, self._options)
        self._size = int(np.prod(self.shape))

    def _init_shape(self, obs_space, options):
        return tuple(obs_space.shape)

    def transform(self, observation):
        raise NotImplementedError

    def write(self, observation, array, offset: int):
        array[offset:offset + self._size] = np.asarray(self.transform(observation)).reshape(-1)

    def check_shape(self, observation):
        if hasattr(self._obs_space, "contains") and not self._obs_space.contains(observation):
            raise ValueError(f"Observation {observation!r} outside {self._obs_space}")

    @property
    def size(self) -> int:
        return self._size

    @property
    def observation_space(self):
        from ray_memory_management_amd.rllib.env import Box

        return Box(-1.0, 1.0, self.shape, dtype=np.float32)


class NoPreprocessor(Preprocessor):
    def transform(self, observation):
        return observation

    @property
    def observation_space(self):
        return self._obs_space


class OneHotPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        return (int(obs_space.n),)

    def transform(self, observation):
        a = np.zeros(self.shape, dtype=np.float32)
        a[int(observation)] = 1.0
        return a


class GenericPixelPreprocessor(Preprocessor):
    """Resize to dim x dim (nearest), optional grayscale and zero-mean scaling."""

    def _init_shape(self, obs_space, options):
        dim = int(options.get("dim", 84))
        return (dim, dim, 1) if options.get("grayscale") else (dim, dim, int(obs_space.shape[-1]))

    def transform(self, observation):
        obs = np.asarray(observation, dtype=np.float32)
        dim = self.shape[0]
        ys = (np.arange(dim) * obs.shape[0] / dim).astype(np.int64)
        xs = (np.arange(dim) * obs.shape[1] / dim).astype(np.int64)
        out = obs[ys][:, xs]
        if self._options.get("grayscale"):
            out = out.mean(axis=-1, keepdims=True)
        if self._options.get("zero_mean", True):
            out = (out - 128.0) / 128.0
        else:
            out = out / 255.0
        return out


class AtariRamPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        return (128,)

    def transform(self, observation):
        return (np.asarray(observation, dtype=np.float32) - 128.0) / 128.0


def _component_size(space) -> int:
    if hasattr(space, "n"):
        return int(space.n)
    if hasattr(space, "spaces"):
        subs = space.spaces.values() if isinstance(space.spaces, dict) else space.spaces
        return sum(_component_size(s) for s in subs)
    return int(np.prod(space.shape)) if space.shape else 1


def _write_component(space, value, array, offset: int) -> int:
    """Flatten one (possibly nested) observation component into array[offset:], return the new offset."""
    if hasattr(space, "n"):
        array[offset:offset + space.n] = 0.0
        array[offset + int(value)] = 1.0
        return offset + int(space.n)
    if hasattr(space, "spaces"):
        items = space.spaces.items() if isinstance(space.spaces, dict) else enumerate(space.spaces)
        for k, s in items:
            offset = _write_component(s, value[k], array, offset)
        return offset
    n = _component_size(space)
    array[offset:offset + n] = np.asarray(value, dtype=np.float32).reshape(-1)
    return offset + n


class DictFlatteningPreprocessor(Preprocessor):
    """Dict observation → one flat float32 vector: components in sorted-key order, Discrete as
    one-hot, Box flattened (reference preprocessors.DictFlatteningPreprocessor). The model gets the
    structure back with :func:`restore_original_dimensions`."""

    def _init_shape(self, obs_space, options):
        return (_component_size(obs_space),)

    def transform(self, observation):
        out = np.empty(self.shape, np.float32)
        _write_component(self._obs_space, observation, out, 0)
        return out

    def write(self, observation, array, offset: int):
        _write_component(self._obs_space, observation, array, offset)


class TupleFlatteningPreprocessor(DictFlatteningPreprocessor):
    """Tuple observation → one flat float32 vector (reference preprocessors.TupleFlatteningPreprocessor)."""


def restore_original_dimensions(obs, obs_space, tensorlib="torch"):
    """Unflatten a [B, N] flat observation batch into the Dict / Tuple structure of `obs_space`:
    Box components get their shape back, Discrete components stay one-hot [B, n]
    (reference rllib/models/modelv2.py restore_original_dimensions)."""
    if not hasattr(obs_space, "spaces"):
        return obs

    def rec(space, flat, off):
        if hasattr(space, "n"):
            return flat[:, off:off + space.n], off + int(space.n)
        if hasattr(space, "spaces"):
            if isinstance(space.spaces, dict):
                out = {}
                for k, s in space.spaces.items():
                    out[k], off = rec(s, flat, off)
                return out, off
            out = []
            for s in space.spaces:
                v, off = rec(s, flat, off)
                out.append(v)
            return tuple(out), off
        n = _component_size(space)
        return flat[:, off:off + n].reshape((flat.shape[0],) + tuple(space.shape)), off + n

    return rec(obs_space, obs, 0)[0]


def flatten_observation(space, obs) -> np.ndarray:
    """One Dict / Tuple observation → its flat float32 vector (identity for other spaces)."""
    if not hasattr(space, "spaces"):
        return obs
    out = np.empty(_component_size(space), np.float32)
    _write_component(space, obs, out, 0)
    return out


def get_preprocessor(space):
    """Preprocessor class for an observation space (reference preprocessors.get_preprocessor)."""
    if hasattr(space, "spaces"):
        return DictFlatteningPreprocessor if isinstance(space.spaces, dict) else TupleFlatteningPreprocessor
    if hasattr(space, "n"):
        return OneHotPreprocessor
    shape = tuple(getattr(space, "shape", ()) or ())
    if shape == (128,) and getattr(space, "dtype", None) == np.uint8:
        return AtariRamPreprocessor
    return NoPreprocessor


# ============================================================================ catalog
class ModelCatalog:
    """reference rllib/models/catalog.py: registry of custom models / action distributions /
    preprocessors and the factory methods the policies use."""

    _custom_models: Dict[str, Any] = {}
    _custom_action_dists: Dict[str, Any] = {}
    _custom_preprocessors: Dict[str, Any] = {}

    @staticmethod
    def _publish(kind: str, name: str, cls) -> None:
        """Registrations also go to the cluster's internal KV (like the reference's tune
        registry in the GCS), so rollout workers / learner actors in other processes resolve the
        same names."""
        try:
            import cloudpickle

            from ray_memory_management_amd import internal

            if internal._internal_kv_initialized():
                internal._internal_kv_put(f"rllib:{kind}:{name}".encode(), cloudpickle.dumps(cls), True,
                                          namespace="rllib")
        except Exception:
            pass

    @staticmethod
    def register_custom_model(model_name: str, model_class) -> None:
        ModelCatalog._custom_models[model_name] = model_class
        ModelCatalog._publish("model", model_name, model_class)

    @staticmethod
    def register_custom_action_dist(action_dist_name: str, action_dist_class) -> None:
        ModelCatalog._custom_action_dists[action_dist_name] = action_dist_class
        ModelCatalog._publish("action_dist", action_dist_name, action_dist_class)

    @staticmethod
    def register_custom_preprocessor(preprocessor_name: str, preprocessor_class) -> None:
        ModelCatalog._custom_preprocessors[preprocessor_name] = preprocessor_class
        ModelCatalog._publish("preprocessor", preprocessor_name, preprocessor_class)

    @staticmethod
    def _resolve(name_or_cls, table: Dict, what: str):
        if name_or_cls is None or not isinstance(name_or_cls, str):
            return name_or_cls
        if name_or_cls in table:
            return table[name_or_cls]
        kind = {"model": "model", "action distribution": "action_dist", "preprocessor": "preprocessor"}[what]
        try:  # registered by another process of this cluster
            import pickle

            from ray_memory_management_amd import internal

            if internal._internal_kv_initialized():
                blob = internal._internal_kv_get(f"rllib:{kind}:{name_or_cls}".encode(), namespace="rllib")
                if blob:
                    table[name_or_cls] = pickle.loads(blob)  # written by register_custom_* above
                    return table[name_or_cls]
        except Exception:
            pass
        if "." in name_or_cls:
            import importlib

            mod, _, attr = name_or_cls.rpartition(".")
            return getattr(importlib.import_module(mod), attr)
        raise ValueError(f"Unknown {what} '{name_or_cls}': register it with ModelCatalog first")

    @staticmethod
    def get_action_dist(action_space, config: Optional[Dict] = None, dist_type=None, framework: str = "torch",
                        **kwargs):
        """Returns (dist_class, num_outputs) for `action_space`."""
        config = config or {}
        custom = config.get("custom_action_dist")
        if custom is not None:
            cls = ModelCatalog._resolve(custom, ModelCatalog._custom_action_dists, "action distribution")
            return cls, cls.required_model_output_shape(action_space, config)
        if dist_type is not None:
            return dist_type, dist_type.required_model_output_shape(action_space, config)
        if hasattr(action_space, "n"):
            return TorchCategorical, int(action_space.n)
        if hasattr(action_space, "shape"):
            return TorchDiagGaussian, int(np.prod(action_space.shape)) * 2
        raise NotImplementedError(f"No action distribution for {action_space}")

    @staticmethod
    def get_action_shape(action_space, framework: str = "torch"):
        if hasattr(action_space, "n"):
            return (np.int64, (None,))
        return (np.float32, (None,) + tuple(action_space.shape))

    @staticmethod
    def get_action_placeholder(action_space, name: str = "action"):
        dtype, shape = ModelCatalog.get_action_shape(action_space)
        return np.zeros([1 if s is None else s for s in shape], dtype=dtype)

    @staticmethod
    def get_model_v2(obs_space, action_space, num_outputs: int, model_config: Dict, framework: str = "torch",
                     name: str = "default_model", model_interface=None, default_model=None, **model_kwargs):
        if framework not in ("torch", None):
            raise ValueError(f"framework={framework!r}: this framework is PyTorch-ROCm only")
        cfg = {**MODEL_DEFAULTS, **(model_config or {})}
        custom = cfg.get("custom_model")
        if custom is not None:
            cls = ModelCatalog._resolve(custom, ModelCatalog._custom_models, "model")
            kwargs = {**(cfg.get("custom_model_config") or {}), **model_kwargs}
            try:
                m = cls(obs_space, action_space, num_outputs, cfg, name, **kwargs)
            except TypeError:
                m = cls(obs_space, action_space, num_outputs, cfg, name)
            return m
        if default_model is not None:
            return default_model(obs_space, action_space, num_outputs, cfg, name)
        from ray_memory_management_amd.rllib.models import build_model

        net = build_model(obs_space, action_space, {k: v for k, v in cfg.items() if k != "custom_model"})
        return NativeModelV2(net, obs_space, action_space, num_outputs, cfg, name)

    @staticmethod
    def get_preprocessor(env, options: Optional[Dict] = None):
        return ModelCatalog.get_preprocessor_for_space(env.observation_space, options)

    @staticmethod
    def get_preprocessor_for_space(observation_space, options: Optional[Dict] = None) -> Preprocessor:
        options = options or MODEL_DEFAULTS
        custom = options.get("custom_preprocessor")
        if custom is not None:
            cls = ModelCatalog._resolve(custom, ModelCatalog._custom_preprocessors, "preprocessor")
        else:
            cls = get_preprocessor(observation_space)
        return cls(observation_space, options)


def build_custom_model(obs_space, action_space, model_config: Dict):
    """The `custom_model` hook of models.build_model: a ModelV2 behind the (logits, value) API."""
    dist_cls, num_outputs = ModelCatalog.get_action_dist(action_space, model_config)
    m = ModelCatalog.get_model_v2(obs_space, action_space, num_outputs, model_config)
    return ModelV2Adapter(m)
