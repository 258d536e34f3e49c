"""Policies. Parity: reference rllib/policy/{policy.py, torch_policy.py} (compute_actions,
compute_single_action, postprocess_trajectory, learn_on_batch, get/set_weights)."""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from ray_memory_management_amd import ops
from ray_memory_management_amd.rllib.distributions import dist_class_for
from ray_memory_management_amd.rllib.models import build_model
from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class Policy:
    """Policy interface (reference rllib/policy/policy.py): map observations to actions and hold
    weights; learning lives in the algorithm's learner. Subclasses implement compute_actions."""

    def __init__(self, observation_space, action_space, config: Dict):
        self.observation_space, self.action_space, self.config = observation_space, action_space, config
        self.global_timestep = 0

    def compute_actions(self, obs_batch, explore: bool = True):
        raise NotImplementedError

    def compute_single_action(self, obs, explore: bool = False):
        a, _, _ = self.compute_actions([obs], explore=explore)
        return a[0]

    def postprocess_trajectory(self, sample_batch, other_agent_batches=None, episode=None):
        return sample_batch

    def get_weights(self):
        return {}

    def set_weights(self, weights) -> None:
        pass

    def get_state(self) -> Dict:
        return {"weights": self.get_weights(), "global_timestep": self.global_timestep}

    def set_state(self, state: Dict) -> None:
        self.set_weights(state["weights"])
        self.global_timestep = state.get("global_timestep", 0)


class TFPolicy(Policy):
    """Reference TFPolicy: TensorFlow is not part of the MI355X stack (PyTorch-ROCm only)."""

    def __init__(self, *a, **kw):
        raise ImportError("TFPolicy needs TensorFlow, which this framework does not use; use TorchPolicy")


class TorchPolicy(Policy):
    """Model + action distribution on a device (CPU for rollout workers, cuda for the learner)."""

    def __init__(self, observation_space, action_space, config: Dict, device="cpu"):
        self.observation_space, self.action_space = observation_space, action_space
        self.config = config
        self.device = torch.device(device)
        self.model = build_model(observation_space, action_space, config.get("model") or {}).to(self.device)
        self.dist_class = dist_class_for(action_space)
        self.global_timestep = 0

    @torch.no_grad()
    def compute_actions(self, obs_batch, explore: bool = True):
        obs = torch.as_tensor(np.asarray(obs_batch), device=self.device)
        logits, v = self.model(obs)
        dist = self.dist_class(logits.float())
        a = dist.sample() if explore else dist.deterministic_sample()
        extra = {SampleBatch.ACTION_LOGP: dist.logp(a).cpu().numpy(), SampleBatch.VF_PREDS: v.float().cpu().numpy(),
                 SampleBatch.ACTION_DIST_INPUTS: logits.float().cpu().numpy()}
        self.global_timestep += len(obs)
        return a.cpu().numpy(), [], extra

    def compute_single_action(self, obs, explore: bool = False):
        a, _, extra = self.compute_actions([obs], explore=explore)
        return a[0]

    @torch.no_grad()
    def value(self, obs_batch) -> np.ndarray:
        _, v = self.model(torch.as_tensor(np.asarray(obs_batch), device=self.device))
        return v.float().cpu().numpy()

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, weights):
        self.model.load_state_dict({k: v.to(self.device) for k, v in weights.items()})


def compute_gae_for_trajectories(rewards, vf_preds, dones, last_values, gamma, lam):
    """Time-major [T, B] numpy arrays → (advantages, value_targets) via the GAE op (HIP kernel
    on GPU tensors, fp32 torch scan on CPU). Reference: rllib/evaluation/postprocessing.py."""
    t = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32))  # noqa: E731
    adv, ret = ops.gae(t(rewards), t(vf_preds), t(dones), t(last_values), gamma, lam)
    return adv.numpy(), ret.numpy()
