"""RuntimeEnv / RuntimeEnvConfig. Parity: reference python/ray/runtime_env/runtime_env.py (a dict
subclass validated on construction; fields env_vars, working_dir, py_modules, pip, conda,
container, excludes, config) — accepted wherever a runtime_env dict is (`ray.init`,
`.options(runtime_env=...)`). pip / conda / container need package installation, which this
offline image cannot do: they are rejected with a clear error when a worker would need them."""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

_KNOWN = {"env_vars", "working_dir", "py_modules", "pip", "conda", "container", "excludes", "config",
          "_ray_release", "_ray_commit", "eager_install"}
_NEEDS_INSTALL = ("pip", "conda", "container")


class RuntimeEnvConfig(dict):
    def __init__(self, setup_timeout_seconds: int = 600, eager_install: bool = True):
        if setup_timeout_seconds <= 0 and setup_timeout_seconds != -1:
            raise ValueError("setup_timeout_seconds must be > 0 or -1")
        super().__init__(setup_timeout_seconds=setup_timeout_seconds, eager_install=eager_install)


class RuntimeEnv(dict):
    def __init__(self, *, py_modules: Optional[List[str]] = None, working_dir: Optional[str] = None,
                 pip=None, conda=None, container: Optional[Dict] = None, env_vars: Optional[Dict[str, str]] = None,
                 config: Optional[RuntimeEnvConfig] = None, _validate: bool = True, **kwargs):
        super().__init__()
        fields = dict(py_modules=py_modules, working_dir=working_dir, pip=pip, conda=conda, container=container,
                      env_vars=env_vars, config=config, **kwargs)
        for k, v in fields.items():
            if v is not None:
                self[k] = v
        if _validate:
            self.validate()

    def validate(self) -> None:
        unknown = set(self) - _KNOWN
        if unknown:
            raise ValueError(f"unknown runtime_env fields: {sorted(unknown)}")
        ev = self.get("env_vars")
        if ev is not None and not (isinstance(ev, dict) and all(isinstance(k, str) and isinstance(v, str)
                                                                 for k, v in ev.items())):
            raise TypeError("runtime_env['env_vars'] must be a Dict[str, str]")
        if "pip" in self and "conda" in self:
            raise ValueError("runtime_env cannot set both 'pip' and 'conda'")
        if "py_modules" in self and not isinstance(self["py_modules"], (list, tuple)):
            raise TypeError("runtime_env['py_modules'] must be a list")

    def needs_install(self) -> List[str]:
        return [k for k in _NEEDS_INSTALL if self.get(k)]

    def to_dict(self) -> Dict[str, Any]:
        return dict(self)

    def serialize(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def deserialize(cls, s: str) -> "RuntimeEnv":
        return cls(**json.loads(s))

    def env_vars(self) -> Dict[str, str]:
        return dict(self.get("env_vars") or {})

    def working_dir(self) -> Optional[str]:
        return self.get("working_dir")

    def py_modules(self) -> List[str]:
        return list(self.get("py_modules") or [])

    def has_pip(self) -> bool:
        return bool(self.get("pip"))


__all__ = ["RuntimeEnvConfig", "RuntimeEnv"]
