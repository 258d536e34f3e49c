"""DDPG (deterministic actor-critic with a replay buffer and Polyak-averaged target networks) and
the continuous-control off-policy scaffolding TD3 and SAC reuse.

Parity: reference rllib/algorithms/ddpg/ddpg.py (DDPGConfig defaults: twin_q, policy_delay,
smooth_target_policy, target_noise(_clip), n_step, actor/critic lrs, tau, l2_reg, use_huber,
random exploration steps, OrnsteinUhlenbeck noise), ddpg_torch_model.py (actor = MLP → tanh squash
onto the action bounds, critic = MLP on [obs, action]), ddpg_torch_policy.py (critic target
r + γⁿ(1-d)·min Q'(s', μ'(s') + clip(ε)), actor loss -Q(s, μ(s)), Polyak update every
`target_network_update_freq` steps) and rllib/utils/exploration/ornstein_uhlenbeck_noise.py.

MI355X design: the learner's networks, optimisers and (with ``num_gpus > 0``) the replay buffer live
on the GPU — a training batch is gathered from HBM with the K2 row-gather kernel, so the only
host→device traffic per iteration is the newly sampled rows. Target updates are ONE multi-tensor
``torch._foreach_lerp_`` over all parameters (a handful of fused launches, not one per tensor).
"""
from __future__ import annotations

import copy
from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch, concat_samples
from ray_memory_management_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer


def _mlp(sizes: List[int], act=nn.ReLU, out_act=None) -> nn.Sequential:
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers.append(act())
    if out_act is not None:
        layers.append(out_act())
    return nn.Sequential(*layers)


def _act_cls(name: str):
    return {"relu": nn.ReLU, "tanh": nn.Tanh, "elu": nn.ELU, "swish": nn.SiLU, "silu": nn.SiLU}[name]


def _bounds(action_space):
    low = torch.tensor(np.array(action_space.low, np.float32)).flatten()
    high = torch.tensor(np.array(action_space.high, np.float32)).flatten()
    return low, high


class ContinuousActorCritic(nn.Module):
    """Actor + (twin) Q critics. ``stochastic`` actors (SAC) emit mean and log-std of a
    tanh-squashed Gaussian; deterministic actors (DDPG/TD3) a tanh-squashed action."""

    def __init__(self, obs_dim: int, action_space, actor_hiddens=(400, 300), critic_hiddens=(400, 300),
                 actor_activation="relu", critic_activation="relu", twin_q: bool = False, stochastic: bool = False):
        super().__init__()
        low, high = _bounds(action_space)
        self.act_dim = int(low.numel())
        self.register_buffer("a_mid", (high + low) / 2.0)
        self.register_buffer("a_half", (high - low) / 2.0)
        self.stochastic = stochastic
        out = 2 * self.act_dim if stochastic else self.act_dim
        self.actor = _mlp([obs_dim, *actor_hiddens, out], _act_cls(actor_activation))
        self.q1 = _mlp([obs_dim + self.act_dim, *critic_hiddens, 1], _act_cls(critic_activation))
        self.q2 = _mlp([obs_dim + self.act_dim, *critic_hiddens, 1], _act_cls(critic_activation)) if twin_q else None

    def scale(self, squashed):  # [-1, 1] → [low, high]
        return self.a_mid + self.a_half * squashed

    def unscale(self, a):
        return (a - self.a_mid) / self.a_half

    def deterministic(self, obs):
        h = self.actor(obs.flatten(1).float())
        if self.stochastic:
            h = h[:, :self.act_dim]
        return self.scale(torch.tanh(h))

    def sample_squashed(self, obs, deterministic: bool = False):
        """SAC: reparameterised tanh-Gaussian sample and its log-prob (with the tanh Jacobian and the
        affine rescale to the action bounds)."""
        h = self.actor(obs.flatten(1).float())
        mean, log_std = h[:, :self.act_dim], h[:, self.act_dim:].clamp(-20.0, 2.0)
        std = log_std.exp()
        u = mean if deterministic else mean + std * torch.randn_like(mean)
        t = torch.tanh(u)
        logp = (-0.5 * ((u - mean) / std) ** 2 - log_std - 0.5 * np.log(2 * np.pi)).sum(-1)
        logp = logp - torch.log(1.0 - t.pow(2) + 1e-6).sum(-1) - torch.log(self.a_half).sum()
        return self.scale(t), logp

    def logp_of(self, obs, act):
        """log π(a|s) of given (dataset) actions under the tanh-squashed Gaussian (CQL's BC phase,
        CRR's weighted regression): invert the squash, Gaussian log-density plus the Jacobian."""
        h = self.actor(obs.flatten(1).float())
        mean, log_std = h[:, :self.act_dim], h[:, self.act_dim:].clamp(-20.0, 2.0)
        t = self.unscale(act.float()).clamp(-1 + 1e-6, 1 - 1e-6)
        u = torch.atanh(t)
        logp = (-0.5 * ((u - mean) / log_std.exp()) ** 2 - log_std - 0.5 * np.log(2 * np.pi)).sum(-1)
        return logp - torch.log(1.0 - t.pow(2) + 1e-6).sum(-1) - torch.log(self.a_half).sum()

    def q(self, obs, act):
        x = torch.cat([obs.flatten(1).float(), act.float()], dim=-1)
        return self.q1(x).squeeze(-1), (self.q2(x).squeeze(-1) if self.q2 is not None else None)


def build_actor_critic(obs_space, action_space, cfg: Dict, stochastic: bool) -> ContinuousActorCritic:
    if not hasattr(action_space, "low"):
        raise ValueError(f"{type(action_space).__name__} action space: DDPG/TD3/SAC need a continuous Box "
                         "action space")
    obs_dim = int(np.prod(obs_space.shape)) if obs_space.shape else 1
    return ContinuousActorCritic(obs_dim, action_space, tuple(cfg.get("actor_hiddens", (400, 300))),
                                 tuple(cfg.get("critic_hiddens", (400, 300))),
                                 cfg.get("actor_hidden_activation", "relu"),
                                 cfg.get("critic_hidden_activation", "relu"),
                                 twin_q=bool(cfg.get("twin_q", False)), stochastic=stochastic)


class ContinuousPolicy:
    """Rollout-side policy: actor network on the worker's CPU + exploration.
    Deterministic actors explore with Ornstein-Uhlenbeck or Gaussian noise after
    `random_timesteps` uniformly random steps (reference exploration/{ornstein_uhlenbeck_noise,
    gaussian_noise}.py); SAC samples its stochastic actor."""

    stochastic = False

    def __init__(self, observation_space, action_space, config: Dict, device="cpu"):
        self.observation_space, self.action_space = observation_space, action_space
        self.config = config
        self.device = torch.device(device)
        self.model = build_actor_critic(observation_space, action_space, config, self.stochastic).to(self.device)
        self.low, self.high = (np.asarray(action_space.low, np.float32), np.asarray(action_space.high, np.float32))
        ec = dict(config.get("exploration_config") or {})
        self.noise_type = ec.get("type", "OrnsteinUhlenbeckNoise")
        self.random_timesteps = int(ec.get("random_timesteps", 1000))
        self.ou_theta, self.ou_sigma = ec.get("ou_theta", 0.15), ec.get("ou_sigma", 0.2)
        self.ou_base_scale = ec.get("ou_base_scale", 0.1)
        self.stddev = ec.get("stddev", 0.1)
        self.scale = ec.get("initial_scale", 1.0)
        self._ou = None
        self._rng = np.random.default_rng(config.get("seed"))
        self.global_timestep = 0

    @torch.no_grad()
    def compute_actions(self, obs_batch, explore: bool = True):
        obs = torch.as_tensor(np.asarray(obs_batch, np.float32), device=self.device)
        n = obs.shape[0]
        if self.stochastic:
            a, logp = self.model.sample_squashed(obs, deterministic=not explore)
            a, logp = a.cpu().numpy(), logp.cpu().numpy()
        else:
            a = self.model.deterministic(obs).cpu().numpy()
            logp = np.zeros(n, np.float32)
            if explore:
                span = self.high - self.low
                if self.global_timestep < self.random_timesteps:
                    a = self._rng.uniform(self.low, self.high, size=a.shape).astype(np.float32)
                elif self.noise_type == "GaussianNoise":
                    a = a + self.scale * self.stddev * span * self._rng.standard_normal(a.shape)
                else:  # Ornstein-Uhlenbeck, one process per env slot
                    if self._ou is None or self._ou.shape != a.shape:
                        self._ou = np.zeros(a.shape, np.float32)
                    self._ou += self.ou_theta * -self._ou + self.ou_sigma * self._rng.standard_normal(a.shape)
                    a = a + self.scale * self.ou_base_scale * self._ou * span
                a = np.clip(a, self.low, self.high).astype(np.float32)
        self.global_timestep += n
        z = np.zeros(n, np.float32)
        return a.astype(np.float32), [], {SampleBatch.ACTION_LOGP: logp.astype(np.float32), SampleBatch.VF_PREDS: z,
                                          SampleBatch.ACTION_DIST_INPUTS: a.astype(np.float32)}

    def compute_single_action(self, obs, explore: bool = False):
        a, _, _ = self.compute_actions([obs], explore=explore)
        return a[0]

    def value(self, obs_batch):
        return np.zeros(len(obs_batch), np.float32)

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, weights):
        self.model.load_state_dict({k: torch.as_tensor(v).to(self.device) for k, v in weights.items()})


class DDPGConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or DDPG)
        self.twin_q = False
        self.policy_delay = 1
        self.smooth_target_policy = False
        self.target_noise = 0.2
        self.target_noise_clip = 0.5
        self.use_state_preprocessor = False
        self.actor_hiddens = [400, 300]
        self.actor_hidden_activation = "relu"
        self.critic_hiddens = [400, 300]
        self.critic_hidden_activation = "relu"
        self.n_step = 1
        self.critic_lr = 1e-3
        self.actor_lr = 1e-3
        self.tau = 0.002
        self.target_network_update_freq = 0
        self.use_huber = False
        self.huber_threshold = 1.0
        self.l2_reg = 1e-6
        self.grad_clip = None
        self.training_intensity = None
        self.num_steps_sampled_before_learning_starts = 1500
        self.train_batch_size = 256
        self.rollout_fragment_length = 1
        self.num_workers = 0
        self.min_sample_timesteps_per_iteration = 1000
        self.replay_buffer_config = {"type": "MultiAgentReplayBuffer", "capacity": 50000,
                                     "prioritized_replay_alpha": 0.6, "prioritized_replay_beta": 0.4,
                                     "prioritized_replay_eps": 1e-6}
        self.exploration_config = {"type": "OrnsteinUhlenbeckNoise", "random_timesteps": 1000,
                                   "ou_base_scale": 0.1, "ou_theta": 0.15, "ou_sigma": 0.2,
                                   "initial_scale": 1.0}
        self.policy_class = "ray_memory_management_amd.rllib.algorithms.ddpg.ContinuousPolicy"

    def training(self, *, replay_buffer_config=None, **kwargs) -> "DDPGConfig":
        super().training(**kwargs)
        if replay_buffer_config is not None:
            self.replay_buffer_config = {**self.replay_buffer_config, **replay_buffer_config}
        return self

    def exploration(self, *, explore=None, exploration_config=None, **kw) -> "DDPGConfig":
        if exploration_config is not None:
            exploration_config = {**self.exploration_config, **exploration_config}
        return super().exploration(explore=explore, exploration_config=exploration_config, **kw)


def polyak_update(target: nn.Module, source: nn.Module, tau: float):
    """θ' ← (1-τ)θ' + τθ for every parameter, as multi-tensor launches."""
    tp = [p for p in target.parameters()]
    sp = [p.detach() for p in source.parameters()]
    with torch.no_grad():
        if tau >= 1.0:
            torch._foreach_copy_(tp, sp)
        else:
            torch._foreach_lerp_(tp, sp, float(tau))


class DDPGLearner:
    """Actor, critic(s) and their targets + Adam optimisers on one device. One `update` = one critic
    step, and (every `policy_delay` critic steps) one actor step and one Polyak target update."""

    def __init__(self, model: ContinuousActorCritic, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.m = model.to(self.device)
        self.target = copy.deepcopy(self.m)
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.cfg = cfg
        critic_params = list(self.m.q1.parameters()) + (list(self.m.q2.parameters()) if self.m.q2 is not None else [])
        self.critic_params = critic_params
        self.actor_opt = torch.optim.Adam(self.m.actor.parameters(), lr=cfg["actor_lr"])
        self.critic_opt = torch.optim.Adam(critic_params, lr=cfg["critic_lr"])
        self.steps = 0

    def _tensors(self, b: SampleBatch):
        dev = self.device
        t = lambda k: torch.as_tensor(b[k], device=dev).float()  # noqa: E731
        w = t("weights") if "weights" in b else None
        return t(SampleBatch.OBS), t(SampleBatch.ACTIONS).reshape(len(b), -1), t(SampleBatch.REWARDS), \
            t(SampleBatch.DONES), t(SampleBatch.NEXT_OBS), w

    def _critic_err(self, td):
        c = self.cfg
        if c.get("use_huber"):
            d = float(c.get("huber_threshold", 1.0))
            return torch.where(td.abs() < d, 0.5 * td.pow(2), d * (td.abs() - 0.5 * d))
        return 0.5 * td.pow(2)

    def critic_target(self, nobs, rew, done):
        c = self.cfg
        with torch.no_grad():
            a2 = self.target.deterministic(nobs)
            if c.get("smooth_target_policy"):
                eps = (torch.randn_like(a2) * c["target_noise"]).clamp(-c["target_noise_clip"], c["target_noise_clip"])
                a2 = torch.max(torch.min(a2 + eps * self.m.a_half, self.m.a_mid + self.m.a_half),
                               self.m.a_mid - self.m.a_half)
            q1t, q2t = self.target.q(nobs, a2)
            qt = torch.min(q1t, q2t) if q2t is not None else q1t
            return rew + (c["gamma"] ** c["n_step"]) * (1.0 - done) * qt

    def update(self, b: SampleBatch) -> Dict:
        c = self.cfg
        obs, act, rew, done, nobs, w = self._tensors(b)
        target = self.critic_target(nobs, rew, done)
        q1, q2 = self.m.q(obs, act)
        td = q1 - target
        err = self._critic_err(td) + (self._critic_err(q2 - target) if q2 is not None else 0.0)
        critic_loss = (err * w).mean() if w is not None else err.mean()
        if c.get("l2_reg"):
            critic_loss = critic_loss + c["l2_reg"] * sum(p.pow(2).sum() for n, p in self.m.named_parameters()
                                                          if n.startswith("q") and n.endswith("weight"))
        self.critic_opt.zero_grad(set_to_none=True)
        critic_loss.backward()
        if c.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.critic_params, c["grad_clip"])
        self.critic_opt.step()
        self.steps += 1
        out = {"critic_loss": float(critic_loss.detach()), "mean_q": float(q1.detach().mean()),
               "td_error": td.detach().abs().cpu().numpy()}
        if self.steps % max(1, int(c.get("policy_delay", 1))) == 0:
            q_pi, _ = self.m.q(obs, self.m.deterministic(obs))
            actor_loss = -q_pi.mean()
            if c.get("l2_reg"):
                actor_loss = actor_loss + c["l2_reg"] * sum(p.pow(2).sum() for n, p in self.m.actor.named_parameters()
                                                            if n.endswith("weight"))
            self.actor_opt.zero_grad(set_to_none=True)
            actor_loss.backward()
            if c.get("grad_clip"):
                nn.utils.clip_grad_norm_(self.m.actor.parameters(), c["grad_clip"])
            self.actor_opt.step()
            self.critic_opt.zero_grad(set_to_none=True)  # actor loss back-propagated into the critics
            out["actor_loss"] = float(actor_loss.detach())
            if not c.get("target_network_update_freq"):
                polyak_update(self.target, self.m, c["tau"])
        return out

    def sync_target(self, tau: float = 1.0):
        polyak_update(self.target, self.m, tau)

    def actor_weights(self):
        return {k: v.detach().cpu() for k, v in self.m.state_dict().items()}

    def get_state(self):
        return {"model": {k: v.detach().cpu() for k, v in self.m.state_dict().items()},
                "target": {k: v.detach().cpu() for k, v in self.target.state_dict().items()}}

    def set_state(self, s):
        self.m.load_state_dict({k: torch.as_tensor(v) for k, v in s["model"].items()})
        self.target.load_state_dict({k: torch.as_tensor(v) for k, v in s["target"].items()})


class OffPolicyContinuousAlgorithm(Algorithm):
    """Shared training loop of DDPG/TD3/SAC (reference dqn.py training_step, which DDPG and SAC
    inherit): sample → replay buffer → `training_intensity`-scaled learner updates on replayed
    batches → priorities → hard target syncs every `target_network_update_freq` sampled steps
    (0 = Polyak after every actor step) → broadcast actor weights."""

    _learner_class = DDPGLearner

    def _learner_cfg(self, c) -> Dict:
        keys = ("gamma", "n_step", "twin_q", "policy_delay", "smooth_target_policy", "target_noise",
                "target_noise_clip", "critic_lr", "actor_lr", "tau", "use_huber", "huber_threshold", "l2_reg",
                "grad_clip", "target_network_update_freq")
        return {k: getattr(c, k) for k in keys if hasattr(c, k)}

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        local = self.workers.local_worker()
        self.learner = self._learner_class(copy.deepcopy(local.policy.model), self._learner_cfg(c), device=dev)
        rb = dict(c.replay_buffer_config)
        self._prioritized = "Prioritized" in str(rb.get("type", ""))
        buf_dev = dev if dev != "cpu" else None
        if self._prioritized:
            self.buffer = PrioritizedReplayBuffer(rb.get("capacity", 50000), alpha=rb.get("prioritized_replay_alpha", 0.6),
                                                  device=buf_dev, seed=c.seed)
        else:
            self.buffer = ReplayBuffer(rb.get("capacity", 50000), device=buf_dev, seed=c.seed)
        self._last_target_update = 0
        self._sync()

    def _sync(self):
        w = self.learner.actor_weights()
        self.workers.local_worker().set_weights(w)
        self.workers.sync_weights(w)

    def _sample(self) -> SampleBatch:
        if self.workers.remote_workers():
            return concat_samples(ray.get([w.sample.remote() for w in self.workers.remote_workers()]))
        return self.workers.local_worker().sample()

    def training_step(self) -> Dict:
        c = self.algo_config
        batch = self._sample()
        keep = [SampleBatch.OBS, SampleBatch.NEXT_OBS, SampleBatch.ACTIONS, SampleBatch.REWARDS, SampleBatch.DONES]
        batch = SampleBatch({k: batch[k] for k in keep})
        self.buffer.add(batch)
        n = batch.count
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        ts = self._counters["num_env_steps_sampled"]
        stats: Dict = {}
        if ts > c.num_steps_sampled_before_learning_starts:
            intensity = c.training_intensity
            n_updates = max(1, int(round(intensity * n / c.train_batch_size))) if intensity else 1
            rb = c.replay_buffer_config
            for _ in range(n_updates):
                tb = self.buffer.sample(c.train_batch_size, beta=rb.get("prioritized_replay_beta", 0.4))
                out = self.learner.update(tb)
                if self._prioritized:
                    self.buffer.update_priorities(tb["batch_indexes"],
                                                  out["td_error"] + rb.get("prioritized_replay_eps", 1e-6))
                stats.update({k: v for k, v in out.items() if k != "td_error"})
                self._counters["num_env_steps_trained"] += c.train_batch_size
            if c.target_network_update_freq and ts - self._last_target_update >= c.target_network_update_freq:
                self.learner.sync_target(c.tau)
                self._last_target_update = ts
                self._counters["num_target_updates"] += 1
            self._sync()
        stats["replay_buffer"] = self.buffer.stats()
        return stats

    def get_weights(self):
        return self.learner.actor_weights()

    def set_weights(self, weights):
        self.learner.m.load_state_dict({k: torch.as_tensor(v) for k, v in weights.items()})
        self.learner.sync_target(1.0)
        self._sync()

    def _extra_state(self):
        return {"learner": self.learner.get_state()}

    def _load_extra_state(self, s):
        if s.get("learner"):
            self.learner.set_state(s["learner"])
            self._sync()


class DDPG(OffPolicyContinuousAlgorithm):
    _config_class = DDPGConfig

    def validate_config(self, c):
        super().validate_config(c)
        if c.n_step < 1:
            raise ValueError("n_step must be >= 1")
        if c.policy_delay < 1:
            raise ValueError("policy_delay must be >= 1")


DEFAULT_CONFIG = DDPGConfig().to_dict()
