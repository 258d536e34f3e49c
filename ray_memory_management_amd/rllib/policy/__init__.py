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

    def is_recurrent(self) -> bool:
        return bool(getattr(self.model, "is_recurrent", False))

    def get_initial_state(self):
        """Per-env initial recurrent state (no batch dim), [] for stateless models."""
        if not self.is_recurrent():
            return []
        return [s[0].cpu().numpy() for s in self.model.initial_state(1, self.device)]

    def _obs_tensor(self, obs_batch):
        from ray_memory_management_amd.rllib.modelv2 import flatten_observation

        if hasattr(self.observation_space, "spaces"):  # Dict / Tuple observations: flat float32 rows
            obs_batch = [o if isinstance(o, np.ndarray) and o.ndim == 1 else flatten_observation(
                self.observation_space, o) for o in obs_batch]
        return torch.as_tensor(np.asarray(obs_batch), device=self.device)

    @torch.no_grad()
    def compute_actions(self, obs_batch, state_batches=None, prev_action_batch=None, prev_reward_batch=None,
                        explore: bool = True, **kwargs):
        """(actions, state_outs, extra) — reference Policy.compute_actions. Recurrent models take and
        return the per-env state (list of [B, ...] arrays; the initial state when None)."""
        if not isinstance(state_batches, (list, tuple)) and state_batches is not None and not isinstance(
                state_batches, np.ndarray):
            explore = bool(state_batches)  # legacy positional call compute_actions(obs, explore)
            state_batches = None
        obs = self._obs_tensor(obs_batch)
        state_out = []
        if self.is_recurrent():
            st = [torch.as_tensor(np.asarray(s), device=self.device) for s in state_batches] if state_batches \
                else self.model.initial_state(obs.shape[0], self.device)
            pa = None if prev_action_batch is None else torch.as_tensor(np.asarray(prev_action_batch), device=self.device)
            pr = None if prev_reward_batch is None else torch.as_tensor(np.asarray(prev_reward_batch, np.float32),
                                                                        device=self.device)
            logits, v, new = self.model.step(obs, st, pa, pr)
            state_out = [s.cpu().numpy() for s in new]
        else:
            logits, v = self.model(obs)
        dist = self.dist_class(logits.float())
        a = dist.sample() if explore else dist.deterministic_sample()
        extra = {SampleBatch.ACTION_LOGP: dist.logp(a).cpu().numpy(), SampleBatch.VF_PREDS: v.float().cpu().numpy(),
                 SampleBatch.ACTION_DIST_INPUTS: logits.float().cpu().numpy()}
        self.global_timestep += len(obs)
        return a.cpu().numpy(), state_out, extra

    def compute_single_action(self, obs, state=None, prev_action=None, prev_reward=None, explore: bool = False,
                              **kwargs):
        """The action for one observation; with a recurrent model (or when `state` is given) the
        reference's (action, state_out, extra) tuple."""
        if self.is_recurrent() or state is not None:
            st = [np.asarray(s)[None] for s in (state if state is not None else self.get_initial_state())]
            a, so, extra = self.compute_actions(
                [obs], st, None if prev_action is None else [prev_action],
                None if prev_reward is None else [prev_reward], explore=explore)
            return a[0], [s[0] for s in so], {k: v[0] for k, v in extra.items()}
        a, _, extra = self.compute_actions([obs], explore=explore)
        return a[0]

    @torch.no_grad()
    def value(self, obs_batch) -> np.ndarray:
        _, v = self.model(self._obs_tensor(obs_batch))
        return v.float().cpu().numpy()

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, weights):
        self.model.load_state_dict({k: v.to(self.device) for k, v in weights.items()})

    # ------------------------------------------------------------------ learning (policy templates)
    # reference rllib/policy/torch_policy.py: loss → compute_gradients / apply_gradients /
    # learn_on_batch. The built-in algorithms train in their own (fused) learners; these are the
    # generic path used by policies built with build_policy_class and the execution-plan operators.
    def loss(self, model, dist_class, train_batch: SampleBatch):
        raise NotImplementedError(f"{type(self).__name__} defines no loss (build it with build_torch_policy)")

    def optimizer(self) -> torch.optim.Optimizer:
        opt = getattr(self, "_optimizer", None)
        if opt is None:
            opt = self._optimizer = torch.optim.Adam(self.model.parameters(), lr=float(self.config.get("lr", 5e-5)))
        return opt

    def stats_fn(self, train_batch: SampleBatch) -> Dict:
        return {}

    def extra_grad_info(self, train_batch: SampleBatch) -> Dict:
        return {}

    def _lazy_tensor_dict(self, batch) -> SampleBatch:
        out = SampleBatch({})
        for k, v in batch.items():
            if isinstance(v, torch.Tensor):
                out[k] = v.to(self.device)
            else:
                a = np.asarray(v)
                out[k] = torch.as_tensor(a, device=self.device) if a.dtype != object else v
        return out

    def _loss_value(self, train) -> torch.Tensor:
        out = self.loss(self.model, self.dist_class, train)
        if isinstance(out, (list, tuple)):
            out = sum(out)
        return out

    def compute_gradients(self, postprocessed_batch):
        """(list of numpy gradients in parameter order, info)."""
        train = self._lazy_tensor_dict(postprocessed_batch)
        params = [p for p in self.model.parameters() if p.requires_grad]
        self.model.zero_grad(set_to_none=True)
        loss = self._loss_value(train)
        loss.backward()
        gc = self.config.get("grad_clip")
        info = {}
        if gc:
            info["grad_gnorm"] = float(torch.nn.utils.clip_grad_norm_(params, gc))
        grads = [(p.grad.detach().cpu().numpy() if p.grad is not None else np.zeros(tuple(p.shape), np.float32))
                 for p in params]
        info.update(self.extra_grad_info(train))
        info["learner_stats"] = {**self.stats_fn(train), "total_loss": float(loss.detach())}
        return grads, info

    def apply_gradients(self, gradients) -> None:
        params = [p for p in self.model.parameters() if p.requires_grad]
        for p, g in zip(params, gradients):
            p.grad = torch.as_tensor(np.asarray(g), dtype=p.dtype, device=p.device)
        self.optimizer().step()

    def learn_on_batch(self, samples) -> Dict:
        grads, info = self.compute_gradients(samples)
        self.apply_gradients(grads)
        self.global_timestep += len(next(iter(samples.values()))) if len(samples) else 0
        return info


def compute_gae_for_trajectories(rewards, vf_preds, dones, last_values, gamma, lam):
    """Time-major [T, B] numpy arrays → (advantages, value_targets) via the GAE op (HIP kernel
    on GPU tensors, fp32 torch scan on CPU). Reference: rllib/evaluation/postprocessing.py."""
    t = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32))  # noqa: E731
    adv, ret = ops.gae(t(rewards), t(vf_preds), t(dones), t(last_values), gamma, lam)
    return adv.numpy(), ret.numpy()


from ray_memory_management_amd.rllib.policy.policy_template import (  # noqa: E402,F401
    build_policy_class, build_tf_policy, build_torch_policy)
