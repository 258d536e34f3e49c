"""Search-space primitives. Parity: reference python/ray/tune/search/sample.py (Domain, Float,
Integer, Categorical, Function with uniform / loguniform / normal / quantized samplers) and the
tune.* constructors (uniform, quniform, loguniform, qloguniform, randn, qrandn, randint,
qrandint, lograndint, qlograndint, choice, sample_from, grid_search)."""
from __future__ import annotations

import math
import random
from typing import Any, Callable, Dict, List, Optional, Sequence


class Domain:
    sampler = None

    def sample(self, spec=None, size: int = 1, random_state: Optional[random.Random] = None):
        rng = random_state or random
        out = [self._sample_one(spec, rng) for _ in range(size)]
        return out[0] if size == 1 else out

    def is_grid(self) -> bool:
        return False

    def is_function(self) -> bool:
        return False

    def _sample_one(self, spec, rng):
        raise NotImplementedError


class Float(Domain):
    def __init__(self, lower: Optional[float], upper: Optional[float]):
        self.lower, self.upper = lower, upper
        self._kind = "uniform"
        self._q = None
        self._mean = self._sd = None
        self._base = 10

    def uniform(self):
        if self.lower is None or self.upper is None:
            raise ValueError("Uniform requires a lower and upper bound")
        self._kind = "uniform"
        return self

    def loguniform(self, base: float = 10):
        if not self.lower > 0:
            raise ValueError("LogUniform requires a lower bound greater than 0.")
        self._kind, self._base = "loguniform", base
        return self

    def normal(self, mean=0.0, sd=1.0):
        self._kind, self._mean, self._sd = "normal", mean, sd
        return self

    def quantized(self, q: float):
        self._q = q
        return self

    def _sample_one(self, spec, rng):
        if self._kind == "uniform":
            v = rng.uniform(self.lower, self.upper)
        elif self._kind == "loguniform":
            lo, hi = math.log(self.lower, self._base), math.log(self.upper, self._base)
            v = self._base ** rng.uniform(lo, hi)
        else:
            v = rng.gauss(self._mean, self._sd)
        if self._q is not None:
            v = round(v / self._q) * self._q
            if self.lower is not None:
                v = max(v, self.lower)
            if self.upper is not None:
                v = min(v, self.upper)
        return float(v)

    def __repr__(self):
        return f"Float({self.lower}, {self.upper}, {self._kind})"


class Integer(Domain):
    def __init__(self, lower: int, upper: int):
        self.lower, self.upper = lower, upper
        self._kind = "uniform"
        self._q = None
        self._base = 10

    def uniform(self):
        self._kind = "uniform"
        return self

    def loguniform(self, base: float = 10):
        if not self.lower > 0:
            raise ValueError("LogUniform requires a lower bound greater than 0.")
        self._kind, self._base = "loguniform", base
        return self

    def quantized(self, q: int):
        self._q = q
        return self

    def _sample_one(self, spec, rng):
        if self._kind == "uniform":
            v = rng.randrange(self.lower, self.upper)  # upper exclusive (reference randint)
        else:
            lo, hi = math.log(self.lower, self._base), math.log(self.upper, self._base)
            v = int(self._base ** rng.uniform(lo, hi))
            v = min(max(v, self.lower), self.upper - 1)
        if self._q is not None:
            v = int(round(v / self._q) * self._q)
            v = min(max(v, self.lower), self.upper)
        return int(v)

    def __repr__(self):
        return f"Integer({self.lower}, {self.upper})"


class Categorical(Domain):
    def __init__(self, categories: Sequence):
        self.categories = list(categories)

    def uniform(self):
        return self

    def grid(self):
        return GridSearch(self.categories)

    def _sample_one(self, spec, rng):
        return rng.choice(self.categories)

    def __len__(self):
        return len(self.categories)

    def __repr__(self):
        return f"Categorical({self.categories})"


class Function(Domain):
    def __init__(self, func: Callable):
        self.func = func

    def is_function(self):
        return True

    def _sample_one(self, spec, rng):
        import inspect

        try:
            n = len(inspect.signature(self.func).parameters)
        except (TypeError, ValueError):
            n = 1
        return self.func(spec) if n >= 1 else self.func()


class GridSearch(Domain):
    def __init__(self, values: Sequence):
        self.values = list(values)

    def is_grid(self):
        return True

    def _sample_one(self, spec, rng):
        raise RuntimeError("grid_search values are expanded, not sampled")


def uniform(lower: float, upper: float):
    return Float(lower, upper).uniform()


def quniform(lower: float, upper: float, q: float):
    return Float(lower, upper).uniform().quantized(q)


def loguniform(lower: float, upper: float, base: float = 10):
    return Float(lower, upper).loguniform(base)


def qloguniform(lower: float, upper: float, q: float, base: float = 10):
    return Float(lower, upper).loguniform(base).quantized(q)


def randn(mean: float = 0.0, sd: float = 1.0):
    return Float(None, None).normal(mean, sd)


def qrandn(mean: float, sd: float, q: float):
    return Float(None, None).normal(mean, sd).quantized(q)


def randint(lower: int, upper: int):
    return Integer(lower, upper).uniform()


def qrandint(lower: int, upper: int, q: int = 1):
    return Integer(lower, upper).uniform().quantized(q)


def lograndint(lower: int, upper: int, base: float = 10):
    return Integer(lower, upper).loguniform(base)


def qlograndint(lower: int, upper: int, q: int, base: float = 10):
    return Integer(lower, upper).loguniform(base).quantized(q)


def choice(categories: Sequence):
    return Categorical(categories).uniform()


def sample_from(func: Callable):
    return Function(func)


def grid_search(values: Sequence) -> Dict[str, List]:
    """Reference encoding: {"grid_search": [...]}."""
    return {"grid_search": list(values)}
