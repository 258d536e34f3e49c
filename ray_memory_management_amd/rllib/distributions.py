"""Action distributions. Parity: reference rllib/models/torch/torch_action_dist.py
(TorchCategorical, TorchDiagGaussian)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


class Categorical:
    def __init__(self, logits):
        self.logits = logits.float()
        self._logp = None

    @property
    def log_probs(self):
        if self._logp is None:
            self._logp = F.log_softmax(self.logits, dim=-1)
        return self._logp

    def sample(self):
        # Gumbel-max: one fused elementwise + argmax (no host sync, graph-capturable)
        u = torch.rand_like(self.logits).clamp_(1e-10, 1.0)
        return torch.argmax(self.logits - torch.log(-torch.log(u)), dim=-1)

    def deterministic_sample(self):
        return torch.argmax(self.logits, dim=-1)

    def logp(self, actions):
        return self.log_probs.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)

    def entropy(self):
        lp = self.log_probs
        return -(lp.exp() * lp).sum(-1)

    def kl(self, other: "Categorical"):
        lp, lq = self.log_probs, other.log_probs
        return (lp.exp() * (lp - lq)).sum(-1)


class DiagGaussian:
    def __init__(self, inputs):
        inputs = inputs.float()
        self.mean, self.log_std = torch.chunk(inputs, 2, dim=-1)
        self.std = self.log_std.exp()

    def sample(self):
        return self.mean + self.std * torch.randn_like(self.mean)

    def deterministic_sample(self):
        return self.mean

    def logp(self, x):
        return (-0.5 * (((x - self.mean) / self.std) ** 2).sum(-1) - 0.5 * math.log(2 * math.pi) * x.shape[-1]
                - self.log_std.sum(-1))

    def entropy(self):
        return (self.log_std + 0.5 * math.log(2 * math.pi * math.e)).sum(-1)

    def kl(self, other: "DiagGaussian"):
        return (other.log_std - self.log_std + (self.std ** 2 + (self.mean - other.mean) ** 2)
                / (2.0 * other.std ** 2) - 0.5).sum(-1)


def dist_class_for(action_space):
    return Categorical if hasattr(action_space, "n") else DiagGaussian
