"""MAML: model-agnostic meta-learning for policy gradients.

Parity: reference rllib/algorithms/maml/maml.py (MAMLConfig: inner_adaptation_steps 1,
inner_lr 0.1, maml_optimizer_steps 5, lr 1e-3, use_meta_env (TaskSettableEnv: sample_tasks /
set_task), one task per rollout worker, training_step = per-worker pre-adaptation sampling →
inner policy-gradient step → post-adaptation sampling → meta update through the inner step) and
maml_torch_policy.py (second-order meta-gradient of the post-adaptation surrogate through
θ' = θ − α ∇θ L_inner(θ); PPO-style clipping of the outer surrogate, KL between pre/post).

The policy is a diagonal-Gaussian MLP evaluated functionally (torch.func.functional_call), so the
adapted parameters θ' stay differentiable w.r.t. θ; workers sample with the (detached) θ or θ'
shipped through the object store, the meta-gradient is taken on the driver.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn
from torch.func import functional_call

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.env import Box, Env, make_env, register_env


class GoalBanditEnv(Env):
    """TaskSettableEnv (reference rllib/env/apis/task_settable_env.py): a one-dimensional continuous
    bandit whose optimal action is a hidden per-task goal g ∈ [-1, 1]; reward −(a − g)², episodes of
    `episode_len` steps with a constant observation (the goal must be found by adaptation)."""

    def __init__(self, config=None):
        c = config or {}
        self.episode_len = int(c.get("episode_len", 5))
        self.observation_space = Box(-1.0, 1.0, shape=(1,), dtype=np.float32)
        self.action_space = Box(-2.0, 2.0, shape=(1,), dtype=np.float32)
        self.goal = float(c.get("goal", 0.5))
        self.rng = np.random.default_rng(c.get("seed"))
        self.t = 0

    def sample_tasks(self, n: int) -> List[float]:
        return [float(g) for g in self.rng.uniform(-1.0, 1.0, n)]

    def set_task(self, task):
        self.goal = float(task)

    def get_task(self):
        return self.goal

    def reset(self, *, seed=None):
        self.t = 0
        return np.ones(1, np.float32)

    def step(self, action):
        a = float(np.clip(np.asarray(action).reshape(-1)[0], -2.0, 2.0))
        self.t += 1
        return np.ones(1, np.float32), -(a - self.goal) ** 2, self.t >= self.episode_len, {}


register_env("GoalBandit-v0", GoalBanditEnv)


class GaussianPolicyNet(nn.Module):
    def __init__(self, obs_dim, act_dim, hiddens=(32,), init_log_std=0.0):
        super().__init__()
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), nn.Tanh()]
            d = h
        self.body = nn.Sequential(*layers)
        self.mu = nn.Linear(d, act_dim)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(init_log_std)))

    def forward(self, obs):
        return self.mu(self.body(obs)), self.log_std.expand(obs.shape[0], -1)


def _logp(net, params, obs, act):
    mu, log_std = functional_call(net, params, (obs,))
    return (-0.5 * ((act - mu) / log_std.exp()) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)


def _pg_loss(net, params, b):
    adv = (b["returns"] - b["returns"].mean()) / (b["returns"].std() + 1e-6)  # standardised advantages
    return -(_logp(net, params, b["obs"], b["actions"]) * adv).mean()


def maml_sample(worker, task, params: Dict[str, np.ndarray], episodes: int, hiddens, seed: int):
    """Runs inside a RolloutWorker: set the task, roll out `episodes` episodes with the given flat
    parameters; returns obs / actions / per-step reward-to-go and the mean episode return."""
    env = getattr(worker, "_maml_env", None)
    if env is None:
        env = worker._maml_env = make_env(worker.config.get("env"), worker.config.get("env_config") or {})
    env.set_task(task)
    net = getattr(worker, "_maml_net", None)
    if net is None:
        net = worker._maml_net = GaussianPolicyNet(env.observation_space.shape[0], env.action_space.shape[0],
                                                   tuple(hiddens))
    net.load_state_dict({k: torch.as_tensor(v) for k, v in params.items()})
    g = torch.Generator().manual_seed(int(seed))
    obs_l, act_l, ret_l, ep_rets = [], [], [], []
    with torch.no_grad():
        for _ in range(episodes):
            o, done, rews = env.reset(), False, []
            while not done:
                ot = torch.as_tensor(np.asarray(o, np.float32))[None]
                mu, log_std = net(ot)
                a = (mu + log_std.exp() * torch.randn(mu.shape, generator=g))[0]
                o2, r, done, _ = env.step(a.numpy())
                obs_l.append(ot[0].numpy())
                act_l.append(a.numpy())
                rews.append(r)
                o = o2
            rtg = np.cumsum(np.asarray(rews)[::-1])[::-1]
            ret_l += list(rtg)
            ep_rets.append(float(np.sum(rews)))
    return ({"obs": np.stack(obs_l).astype(np.float32), "actions": np.stack(act_l).astype(np.float32),
             "returns": np.asarray(ret_l, np.float32)}, float(np.mean(ep_rets)))


class MAMLConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or MAML)
        self.inner_adaptation_steps = 1
        self.inner_lr = 0.1
        self.maml_optimizer_steps = 5
        self.lr = 1e-3
        self.num_workers = 2
        self.episodes_per_task = 10
        self.clip_param = 0.3
        self.model = {"fcnet_hiddens": [32]}
        self.use_meta_env = True


class MAML(Algorithm):
    _config_class = MAMLConfig

    def validate_config(self, c):
        super().validate_config(c)
        if c.num_workers < 1:
            raise ValueError("MAML samples one task per rollout worker: num_rollout_workers >= 1")

    def _setup_learner(self):
        c = self.algo_config
        env = make_env(c.env, c.env_config)
        if not (hasattr(env, "sample_tasks") and hasattr(env, "set_task")):
            raise ValueError("MAML needs a TaskSettableEnv (sample_tasks / set_task)")
        self.task_env = env
        if c.seed is not None:
            torch.manual_seed(int(c.seed))
            env.rng = np.random.default_rng(int(c.seed))
        self.hiddens = tuple(c.model.get("fcnet_hiddens", (32,)))
        self.net = GaussianPolicyNet(env.observation_space.shape[0], env.action_space.shape[0], self.hiddens)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=c.lr)
        self._seed = int(c.seed or 0) * 100003

    def _params(self):
        return {k: v for k, v in self.net.named_parameters()}

    @staticmethod
    def _np(params):
        return {k: v.detach().cpu().numpy() for k, v in params.items()}

    @staticmethod
    def _t(b):
        return {k: torch.as_tensor(v) for k, v in b.items()}

    def adapt(self, params, batch, steps: int, create_graph: bool):
        """θ' after `steps` inner policy-gradient steps on `batch` (differentiable if create_graph)."""
        p = dict(params)
        for _ in range(steps):
            loss = _pg_loss(self.net, p, batch)
            grads = torch.autograd.grad(loss, list(p.values()), create_graph=create_graph)
            p = {k: v - self.algo_config.inner_lr * g for (k, v), g in zip(p.items(), grads)}
        return p

    def _sample(self, worker_tasks, params_list, tag):
        refs = []
        for i, (w, task) in enumerate(worker_tasks):
            self._seed += 1
            refs.append(w.apply.remote(maml_sample, task, self._np(params_list[i]), self.algo_config.episodes_per_task,
                                       self.hiddens, self._seed))
        return ray.get(refs)

    def training_step(self) -> Dict:
        c = self.algo_config
        workers = self.workers.remote_workers()
        tasks = self.task_env.sample_tasks(len(workers))
        wt = list(zip(workers, tasks))
        theta = self._params()
        pre = self._sample(wt, [theta] * len(wt), "pre")
        pre_b = [self._t(b) for b, _ in pre]
        # inner adaptation per task (first pass without graph just to sample post-adaptation data)
        adapted = [self.adapt(theta, b, c.inner_adaptation_steps, create_graph=False) for b in pre_b]
        post = self._sample(wt, adapted, "post")
        post_b = [self._t(b) for b, _ in post]
        with torch.no_grad():
            old_logp = [_logp(self.net, {k: v.detach() for k, v in a.items()}, pb["obs"], pb["actions"])
                        for a, pb in zip(adapted, post_b)]
        for _ in range(int(c.maml_optimizer_steps)):  # outer (meta) updates through the inner step
            theta = self._params()
            meta = 0.0
            for b_pre, b_post, lp_old in zip(pre_b, post_b, old_logp):
                th_i = self.adapt(theta, b_pre, c.inner_adaptation_steps, create_graph=True)
                adv = (b_post["returns"] - b_post["returns"].mean()) / (b_post["returns"].std() + 1e-6)
                ratio = torch.exp(_logp(self.net, th_i, b_post["obs"], b_post["actions"]) - lp_old)
                surr = torch.min(ratio * adv, ratio.clamp(1 - c.clip_param, 1 + c.clip_param) * adv)
                meta = meta - surr.mean()
            meta = meta / len(pre_b)
            self.opt.zero_grad(set_to_none=True)
            meta.backward()
            self.opt.step()
        n = sum(len(b["returns"]) for b, _ in pre) + sum(len(b["returns"]) for b, _ in post)
        self._counters["num_env_steps_sampled"] += n
        self._counters["num_env_steps_trained"] += n
        self._timesteps_total += n
        pre_r, post_r = float(np.mean([r for _, r in pre])), float(np.mean([r for _, r in post]))
        self._episode_history.append((post_r, 0))
        return {"meta_loss": float(meta.detach()), "episode_reward_mean_pre_adaptation": pre_r,
                "episode_reward_mean_post_adaptation": post_r, "adaptation_delta": post_r - pre_r}

    def adaptation_gain(self, n_tasks: int = 8, seed: int = 0):
        """Mean (pre, post) return on fresh tasks after one inner adaptation from the current θ."""
        rng = np.random.default_rng(seed)
        tasks = list(rng.uniform(-1, 1, n_tasks))
        workers = self.workers.remote_workers()
        pres, posts = [], []
        theta = {k: v.detach() for k, v in self._params().items()}
        for j in range(0, n_tasks, len(workers)):
            wt = list(zip(workers, tasks[j:j + len(workers)]))
            pre = self._sample(wt, [theta] * len(wt), "eval-pre")
            th = [self.adapt({k: v.requires_grad_(True) for k, v in theta.items()}, self._t(b),
                             self.algo_config.inner_adaptation_steps, create_graph=False) for b, _ in pre]
            post = self._sample(wt, th, "eval-post")
            pres += [r for _, r in pre]
            posts += [r for _, r in post]
        return float(np.mean(pres)), float(np.mean(posts))

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.net.state_dict().items()}

    def set_weights(self, w):
        self.net.load_state_dict(w)


DEFAULT_CONFIG = MAMLConfig().to_dict()
