"""Behaviour cloning = MARWIL with beta 0 (reference rllib/algorithms/bc/bc.py: BCConfig sets
beta = 0.0 and keeps MARWIL's training step)."""
from __future__ import annotations

from ray_memory_management_amd.rllib.algorithms.marwil import MARWIL, MARWILConfig


class BCConfig(MARWILConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or BC)
        self.beta = 0.0


class BC(MARWIL):
    _config_class = BCConfig

    def validate_config(self, c):
        super().validate_config(c)
        if c.beta != 0.0:
            raise ValueError("BC requires beta == 0 (use MARWIL for beta > 0)")


DEFAULT_CONFIG = BCConfig().to_dict()
