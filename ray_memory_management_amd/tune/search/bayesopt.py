"""Bayesian optimisation searcher on scikit-learn's Gaussian process.

Parity: reference python/ray/tune/search/bayesopt/bayesopt_search.py (BayesOptSearch(space, metric,
mode, utility_kwargs={"kind": "ucb", "kappa": 2.576, "xi": 0.0}, random_state,
random_search_steps, points_to_evaluate): continuous parameters only, a GP surrogate fitted to the
observed (config, metric) pairs, the next config maximises the acquisition (UCB / EI / POI);
usually wrapped in ConcurrencyLimiter). The reference wraps the `bayes_opt` package; here the GP
is sklearn's (Matérn-5/2 + white noise) and the acquisition is maximised over random candidates
in the unit cube (log-uniform parameters are modelled in log space).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

from ray_memory_management_amd.tune.search.sample import Domain, Float, Integer
from ray_memory_management_amd.tune.search.variant_generator import Searcher


def _flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "/"))
        else:
            out[key] = v
    return out


def _unflatten(flat):
    out: Dict = {}
    for k, v in flat.items():
        cur = out
        parts = k.split("/")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = v
    return out


class BayesOptSearch(Searcher):
    def __init__(self, space: Optional[Dict] = None, metric: Optional[str] = None, mode: Optional[str] = None,
                 points_to_evaluate: Optional[List[Dict]] = None, utility_kwargs: Optional[Dict] = None,
                 random_state: int = 42, random_search_steps: int = 10, n_candidates: int = 2048):
        super().__init__(metric, mode)
        self._ukw = {"kind": "ucb", "kappa": 2.576, "xi": 0.0, **(utility_kwargs or {})}
        self._rng = np.random.default_rng(random_state)
        self._random_steps = int(random_search_steps)
        self._n_cand = int(n_candidates)
        self._points = list(points_to_evaluate or [])
        self._X: List[np.ndarray] = []
        self._y: List[float] = []
        self._live: Dict[str, np.ndarray] = {}
        self._num_samples = None
        self._suggested = 0
        self._space = None
        if space:
            self._set_space(space)

    def _set_space(self, space):
        flat = _flatten(space)
        self._params, self._const = [], {}
        for k, v in flat.items():
            if isinstance(v, (Float, Integer)):
                if v.lower is None or v.upper is None or getattr(v, "_kind", "uniform") == "normal":
                    raise ValueError(f"BayesOptSearch needs bounded uniform / loguniform parameters ({k}: {v})")
                self._params.append((k, v))
            elif isinstance(v, Domain):
                raise ValueError(f"BayesOptSearch supports continuous (and integer) parameters only; {k} is {v}")
            else:
                self._const[k] = v
        if not self._params:
            raise ValueError("BayesOptSearch: the search space has no continuous parameters")
        self._space = space

    def set_search_properties(self, metric, mode, config, num_samples: Optional[int] = None, **kw) -> bool:
        super().set_search_properties(metric, mode, config)
        if self._space is None and config:
            self._set_space(config)
        if num_samples is not None:
            self._num_samples = int(num_samples)
        return True

    # ---- unit-cube encoding
    def _decode(self, u: np.ndarray) -> Dict:
        out = dict(self._const)
        for x, (k, d) in zip(u, self._params):
            log = getattr(d, "_kind", "uniform") == "loguniform"
            lo, hi = (math.log(d.lower), math.log(d.upper)) if log else (d.lower, d.upper)
            if isinstance(d, Integer):
                hi = hi - 1 if not log else math.log(d.upper - 1)
            v = lo + float(x) * (hi - lo)
            v = math.exp(v) if log else v
            out[k] = int(round(v)) if isinstance(d, Integer) else v
        return _unflatten(out)

    def _encode(self, cfg: Dict) -> np.ndarray:
        flat = _flatten(cfg)
        u = []
        for k, d in self._params:
            v = float(flat[k])
            log = getattr(d, "_kind", "uniform") == "loguniform"
            lo, hi = (math.log(d.lower), math.log(d.upper)) if log else (d.lower, d.upper)
            u.append(((math.log(v) if log else v) - lo) / max(hi - lo, 1e-12))
        return np.clip(np.asarray(u), 0.0, 1.0)

    def _acquisition(self, mu, sd, best):
        kind = self._ukw["kind"]
        if kind == "ucb":
            return mu + self._ukw["kappa"] * sd
        from scipy.stats import norm

        z = (mu - best - self._ukw["xi"]) / np.maximum(sd, 1e-9)
        if kind == "ei":
            return (mu - best - self._ukw["xi"]) * norm.cdf(z) + sd * norm.pdf(z)
        return norm.cdf(z)  # poi

    def suggest(self, trial_id: str):
        if self._num_samples is not None and self._suggested >= self._num_samples:
            return Searcher.FINISHED
        if self._points:
            u = self._encode(self._points.pop(0))
        elif len(self._y) < self._random_steps:
            u = self._rng.random(len(self._params))
        else:
            from sklearn.gaussian_process import GaussianProcessRegressor
            from sklearn.gaussian_process.kernels import Matern, WhiteKernel

            X, y = np.stack(self._X), np.asarray(self._y)
            ym, ys = y.mean(), y.std() + 1e-9
            gp = GaussianProcessRegressor(kernel=Matern(nu=2.5) + WhiteKernel(1e-3), normalize_y=False,
                                          n_restarts_optimizer=2, random_state=int(self._rng.integers(1 << 30)))
            gp.fit(X, (y - ym) / ys)
            cand = self._rng.random((self._n_cand, len(self._params)))
            mu, sd = gp.predict(cand, return_std=True)
            u = cand[int(np.argmax(self._acquisition(mu, sd, float(((y - ym) / ys).max()))))]
        self._live[trial_id] = u
        self._suggested += 1
        return self._decode(u)

    def on_trial_complete(self, trial_id: str, result: Optional[Dict] = None, error: bool = False):
        u = self._live.pop(trial_id, None)
        if u is None or error or not result or self._metric not in result:
            return
        v = float(result[self._metric])
        if not math.isfinite(v):
            return
        self._X.append(u)
        self._y.append(v if self._mode != "min" else -v)  # the GP always maximises

    def best(self):
        if not self._y:
            return None
        i = int(np.argmax(self._y))
        return self._decode(self._X[i]), (self._y[i] if self._mode != "min" else -self._y[i])
