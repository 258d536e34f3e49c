"""ComplexInputNetwork: one network over Dict / Tuple observations.

Parity: reference rllib/models/torch/complex_input_net.py:24 (ComplexInputNetwork): a sub-network
per observation component (conv stack for images, one-hot for Discrete, fully-connected for flat
Box), their outputs concatenated, a post-FC stack (``post_fcnet_hiddens``), then the logits and
value heads.

Here rollout workers flatten composite observations into one float32 vector per step
(modelv2.DictFlatteningPreprocessor), so observation columns stay ordinary [B, N] arrays through
the sample batch, the object store and the learner's row gathers; the network restores the
components with ``restore_original_dimensions`` as views of that one buffer.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.modelv2 import _component_size, restore_original_dimensions


def _act(name):
    from ray_memory_management_amd.rllib.models import _act as a

    return a(name)


class ConvTrunk(nn.Module):
    """Conv stack over one image component ([B, H, W, C] or [B, C, H, W]) → flat features."""

    def __init__(self, shape, filters=None, activation="relu", scale=1.0):
        super().__init__()
        from ray_memory_management_amd.rllib.models import ConvReLU, _same_pad

        h, w, c = (shape[0], shape[1], shape[2]) if shape[-1] <= 4 and shape[0] > 4 else (shape[1], shape[2], shape[0])
        self.channels_last = shape[-1] == c and shape[0] != c
        if filters is None:  # small images (reference get_filter_config covers 84/42/10; others: this)
            filters = [(16, 4, 2), (32, 4, 2), (64, 3, 1)] if min(h, w) >= 32 else [(16, 3, 1), (32, 3, 2)]
        layers, hw = [], h
        for out, k, s in filters:
            pad = _same_pad(hw, k, s)
            layers.append(ConvReLU(c, out, k, s, padding=pad))
            hw = (hw + 2 * pad - k) // s + 1
            c = out
        self.convs = nn.Sequential(*layers)
        self.out_dim = c * hw * hw
        self.scale = float(scale)

    def forward(self, x):
        if self.channels_last:
            x = x.permute(0, 3, 1, 2)
        return self.convs(x.float() * self.scale).flatten(1)


class ComplexInputNetwork(nn.Module):
    """(logits, value) over flat composite observations; ``features(obs)`` gives the post-FC
    features (the trunk the LSTM / attention wrappers put a memory on)."""

    def __init__(self, obs_space, num_outputs: int, model_config: Dict):
        super().__init__()
        self.obs_space = obs_space
        cfg = model_config or {}
        self.flat_dim = _component_size(obs_space)
        subs = obs_space.spaces.items() if isinstance(obs_space.spaces, dict) else enumerate(obs_space.spaces)
        self.keys: List = []
        self.kinds: List[str] = []
        nets = []
        concat = 0
        hid = list(cfg.get("fcnet_hiddens") or [256, 256])
        act = cfg.get("fcnet_activation", "tanh")
        for k, sp in subs:
            self.keys.append(k)
            if hasattr(sp, "n"):  # one-hot, no sub-network (reference: one_hot + flatten)
                self.kinds.append("onehot")
                nets.append(nn.Identity())
                concat += int(sp.n)
            elif hasattr(sp, "spaces"):  # nested composite: a ComplexInputNetwork of its own
                self.kinds.append("nested")
                sub = ComplexInputNetwork(sp, 0, cfg)
                nets.append(sub)
                concat += sub.out_dim
            elif len(sp.shape) == 3:  # image
                self.kinds.append("image")
                scale = 1.0 / 255.0 if np.dtype(sp.dtype) == np.uint8 else 1.0
                t = ConvTrunk(sp.shape, cfg.get("conv_filters"), cfg.get("conv_activation", "relu"), scale)
                nets.append(t)
                concat += t.out_dim
            else:  # flat Box: fully-connected stack (reference: FullyConnectedNetwork, no head)
                self.kinds.append("flat")
                layers, d = [], int(np.prod(sp.shape)) if sp.shape else 1
                for h in hid:
                    layers += [nn.Linear(d, h), _act(act)]
                    d = h
                nets.append(nn.Sequential(*layers))
                concat += d
        self.subnets = nn.ModuleList(nets)
        post, d = [], concat
        for h in cfg.get("post_fcnet_hiddens") or []:
            post += [nn.Linear(d, h), _act(cfg.get("post_fcnet_activation", "relu"))]
            d = h
        self.post = nn.Sequential(*post)
        self.out_dim = d
        self.num_outputs = int(num_outputs)
        if self.num_outputs:
            self.logits = nn.Linear(d, self.num_outputs)
            self.value = nn.Linear(d, 1)
            nn.init.orthogonal_(self.logits.weight, 0.01)
            nn.init.zeros_(self.logits.bias)

    def features(self, obs):
        obs = obs.reshape(obs.shape[0], -1).float() if not isinstance(obs, (dict, tuple, list)) else obs
        parts = restore_original_dimensions(obs, self.obs_space) if not isinstance(obs, (dict, tuple, list)) else obs
        outs = []
        for k, kind, net in zip(self.keys, self.kinds, self.subnets):
            x = parts[k]
            if kind == "nested":
                outs.append(net.features(x))
            elif kind == "flat":
                outs.append(net(x.reshape(x.shape[0], -1)))
            else:
                outs.append(net(x))
        return self.post(torch.cat(outs, dim=1))

    def forward(self, obs):
        h = self.features(obs)
        return self.logits(h), self.value(h).squeeze(-1)
