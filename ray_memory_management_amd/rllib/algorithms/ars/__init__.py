"""ARS: augmented random search (Mania et al. 2018).

Parity: reference rllib/algorithms/ars/ars.py (ARSConfig: noise_stdev 0.02, num_rollouts 32
directions, rollouts_used 32 top directions ranked by max(r+, r-), sgd_stepsize 0.01, plain
gradient step scaled by the std of the returns used, eval_prob 0.03, MeanStdFilter, linear policy
by default) and ars_torch_policy.py. Runs on the ES worker/noise-table machinery
(`algorithms.es`): same shared store-resident noise table, same antithetic worker actors.
"""
from __future__ import annotations

import numpy as np

from ray_memory_management_amd.rllib.algorithms.es import ES, ESConfig


class ARSConfig(ESConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or ARS)
        self.action_noise_std = 0.0
        self.noise_stdev = 0.02
        self.num_rollouts = 32
        self.rollouts_used = 32
        self.num_workers = 2
        self.sgd_stepsize = 0.01
        self.observation_filter = "MeanStdFilter"
        self.eval_prob = 0.03
        self.episodes_per_batch = 0
        self.train_batch_size = 0
        self.offset = 0
        self.model = {**self.model, "fcnet_hiddens": [], "vf_share_layers": True}


class ARS(ES):
    _config_class = ARSConfig

    def _perturbations_per_worker(self, c) -> int:
        return max(1, -(-int(c.num_rollouts) // max(1, c.num_workers)))

    def _update(self, theta, idxs, returns, lengths) -> np.ndarray:
        c = self.algo_config
        returns = returns - float(c.offset) * lengths  # survival bonus offset (reference `offset`)
        k = min(int(c.rollouts_used), len(returns))
        top = np.argsort(np.max(returns, axis=1))[::-1][:k]
        r, idx = returns[top], [idxs[i] for i in top]
        sigma_r = float(r.std()) or 1.0
        dim = len(theta)
        g = np.zeros(dim, np.float32)
        for (rp, rn), i in zip(r, idx):
            g += (rp - rn) * self.noise[i:i + dim]
        g /= (k * sigma_r)
        return (theta + c.sgd_stepsize * g).astype(np.float32)


DEFAULT_CONFIG = ARSConfig().to_dict()
