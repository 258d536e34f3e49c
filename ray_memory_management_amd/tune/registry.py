"""Named trainables / envs. Parity: reference python/ray/tune/registry.py (register_trainable,
register_env, get_trainable_cls)."""
from __future__ import annotations

_trainables = {}
_envs = {}


def register_trainable(name: str, trainable, warn: bool = True):
    from ray_memory_management_amd.tune.trainable import wrap_function

    _trainables[name] = wrap_function(trainable)


def get_trainable_cls(name: str):
    if name in _trainables:
        return _trainables[name]
    try:  # RLlib algorithms by name ("PPO")
        from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

        return get_algorithm_class(name)
    except (ImportError, KeyError, ValueError):
        raise ValueError(f"Unknown trainable {name!r}")


def register_env(name: str, env_creator):
    _envs[name] = env_creator
    try:
        from ray_memory_management_amd.rllib.env import register_env as _rl

        _rl(name, env_creator)
    except ImportError:
        pass


def get_env(name: str):
    return _envs.get(name)
