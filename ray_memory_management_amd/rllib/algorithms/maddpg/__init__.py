"""MADDPG: multi-agent DDPG with centralised critics and decentralised actors.

Parity: reference rllib/algorithms/maddpg/maddpg.py (MADDPGConfig: agent_id per policy,
use_local_critic False, good/adv policy "maddpg", actor/critic hiddens [64, 64], n_step 1,
tau 0.01, actor_lr / critic_lr 1e-2, grad_norm_clipping 0.5, train_batch_size 1024) and
maddpg_torch_policy.py (critic_i(o_1..o_n, a_1..a_n); target y_i = r_i + γ(1−d) Q'_i(o', μ'_1(o'_1),
…, μ'_n(o'_n)); actor_i ascends Q_i with a_i replaced by μ_i(o_i); Polyak target updates).
Continuous (Box) actions. The team env is a MultiAgentEnv with a fixed agent set; joint
transitions live in one columnar replay buffer ([n_agents, …] per row).
"""
from __future__ import annotations

import collections
import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.algorithms.ddpg import _mlp, polyak_update
from ray_memory_management_amd.rllib.env import Box, MultiAgentEnv, make_env, register_env
from ray_memory_management_amd.rllib.sample_batch import SampleBatch
from ray_memory_management_amd.rllib.utils.replay_buffers import ReplayBuffer


class CoopTargetEnv(MultiAgentEnv):
    """Two agents see a shared target t ∈ [-1, 1] and must split it: team reward
    −(a_0 + a_1 − t)² − 0.5 (a_0 − a_1)² (optimum a_0 = a_1 = t/2, return 0)."""

    def __init__(self, config=None):
        config = config or {}
        self.episode_len = int(config.get("episode_len", 10))
        self._agent_ids = {0, 1}
        self.observation_space = Box(-1.0, 1.0, shape=(3,), dtype=np.float32)
        self.action_space = Box(-1.0, 1.0, shape=(1,), dtype=np.float32)
        self.rng = np.random.default_rng(config.get("seed"))
        self.t = 0
        self.target = 0.0

    def _obs(self):
        return {i: np.array([self.target, float(i == 0), float(i == 1)], np.float32) for i in (0, 1)}

    def reset(self, *, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.target = float(self.rng.uniform(-1, 1))
        return self._obs()

    def step(self, action_dict):
        a0, a1 = (float(np.clip(np.asarray(action_dict[i]).reshape(-1)[0], -1, 1)) for i in (0, 1))
        r = -(a0 + a1 - self.target) ** 2 - 0.5 * (a0 - a1) ** 2
        self.t += 1
        self.target = float(self.rng.uniform(-1, 1))
        d = self.t >= self.episode_len
        return self._obs(), {0: r, 1: r}, {0: d, 1: d, "__all__": d}, {}


register_env("CoopTarget-v0", CoopTargetEnv)


class MADDPGConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or MADDPG)
        self.use_local_critic = False
        self.actor_hiddens = [64, 64]
        self.critic_hiddens = [64, 64]
        self.n_step = 1
        self.tau = 0.01
        self.actor_lr = 1e-2
        self.critic_lr = 1e-2
        self.grad_norm_clipping = 0.5
        self.train_batch_size = 1024
        self.num_steps_sampled_before_learning_starts = 1024 * 25
        self.rollout_fragment_length = 100
        self.num_workers = 0
        self.min_sample_timesteps_per_iteration = 100
        self.exploration_noise = 0.1
        self.replay_buffer_config = {"capacity": 1000000}


class MADDPG(Algorithm):
    _config_class = MADDPGConfig

    def setup(self, config: Dict):
        import ray_memory_management_amd as ray

        if not ray.is_initialized():
            ray.init()
        c = self.algo_config
        self.validate_config(c)
        self.env = make_env(c.env, c.env_config)
        self.agents = sorted(self.env.get_agent_ids())
        n = len(self.agents)
        od, ad = int(np.prod(self.env.observation_space.shape)), int(np.prod(self.env.action_space.shape))
        self.low, self.high = np.asarray(self.env.action_space.low), np.asarray(self.env.action_space.high)
        if c.seed is not None:
            torch.manual_seed(int(c.seed))
        dev = torch.device("cuda" if c.num_gpus and torch.cuda.is_available() else "cpu")
        self.device = dev
        cin = (od + ad) if c.use_local_critic else n * (od + ad)
        self.actors = nn.ModuleList([_mlp([od, *c.actor_hiddens, ad], nn.ReLU, nn.Tanh) for _ in range(n)]).to(dev)
        self.critics = nn.ModuleList([_mlp([cin, *c.critic_hiddens, 1], nn.ReLU) for _ in range(n)]).to(dev)
        self.t_actors, self.t_critics = copy.deepcopy(self.actors), copy.deepcopy(self.critics)
        self.a_opts = [torch.optim.Adam(a.parameters(), lr=c.actor_lr) for a in self.actors]
        self.c_opts = [torch.optim.Adam(q.parameters(), lr=c.critic_lr) for q in self.critics]
        self.buffer = ReplayBuffer(int(c.replay_buffer_config.get("capacity", 1000000)), seed=c.seed)
        self.rng = np.random.default_rng(c.seed)
        self._obs = self.env.reset(seed=c.seed)
        self._ep_ret = 0.0
        self._episode_history = collections.deque(maxlen=100)
        self._counters = collections.Counter()
        self._timesteps_total = self._episodes_total = 0
        self.workers = None
        self._multi_agent = True
        self.callbacks = None
        self.od, self.ad, self.n = od, ad, n

    def _scale(self, a):
        return self.low + (a + 1.0) * 0.5 * (self.high - self.low)

    @torch.no_grad()
    def compute_actions(self, obs_dict, explore=True):
        out = {}
        for i, aid in enumerate(self.agents):
            a = self.actors[i](torch.as_tensor(obs_dict[aid], device=self.device).float().unsqueeze(0))[0].cpu().numpy()
            if explore:
                a = np.clip(a + self.algo_config.exploration_noise * self.rng.standard_normal(a.shape), -1, 1)
            out[aid] = self._scale(a).astype(np.float32)
        return out

    def _critic_in(self, obs, act, i):
        if self.algo_config.use_local_critic:
            return torch.cat([obs[:, i], act[:, i]], -1)
        return torch.cat([obs.flatten(1), act.flatten(1)], -1)

    def _learn(self, b) -> Dict:
        c, dev = self.algo_config, self.device
        t = lambda k: torch.as_tensor(np.asarray(b[k]), device=dev).float()  # noqa: E731
        obs, act, rew, nobs, done = t("obs"), t("actions"), t("rewards"), t("new_obs"), t("dones")
        with torch.no_grad():
            na = torch.stack([self.t_actors[j](nobs[:, j]) for j in range(self.n)], 1)
        stats = {}
        for i in range(self.n):
            with torch.no_grad():
                y = rew[:, i] + c.gamma * (1.0 - done) * self.t_critics[i](self._critic_in(nobs, na, i)).squeeze(-1)
            q = self.critics[i](self._critic_in(obs, act, i)).squeeze(-1)
            closs = ((q - y) ** 2).mean()
            self.c_opts[i].zero_grad(set_to_none=True)
            closs.backward()
            nn.utils.clip_grad_norm_(self.critics[i].parameters(), c.grad_norm_clipping)
            self.c_opts[i].step()
            a_new = act.clone()
            a_new[:, i] = self.actors[i](obs[:, i])
            aloss = -self.critics[i](self._critic_in(obs, a_new, i)).mean()
            self.a_opts[i].zero_grad(set_to_none=True)
            aloss.backward()
            nn.utils.clip_grad_norm_(self.actors[i].parameters(), c.grad_norm_clipping)
            self.a_opts[i].step()
            stats[f"agent_{i}"] = {"critic_loss": float(closs.detach()), "actor_loss": float(aloss.detach())}
        polyak_update(self.t_actors, self.actors, c.tau)
        polyak_update(self.t_critics, self.critics, c.tau)
        return stats

    def training_step(self) -> Dict:
        c = self.algo_config
        rows = collections.defaultdict(list)
        for _ in range(int(c.rollout_fragment_length)):
            acts = self.compute_actions(self._obs)
            nobs, rew, done, _ = self.env.step(acts)
            # stored actions are the actors' [-1, 1] outputs (before the bound rescale)
            norm = [2.0 * (acts[a] - self.low) / (self.high - self.low) - 1.0 for a in self.agents]
            rows["obs"].append(np.stack([self._obs[a] for a in self.agents]))
            rows["actions"].append(np.stack(norm))
            rows["rewards"].append(np.array([rew[a] for a in self.agents], np.float32))
            rows["new_obs"].append(np.stack([nobs[a] for a in self.agents]))
            rows["dones"].append(float(done["__all__"]))
            self._ep_ret += float(np.mean([rew[a] for a in self.agents]))
            if done["__all__"]:
                self._episode_history.append(self._ep_ret)
                self._episodes_total += 1
                self._ep_ret = 0.0
                nobs = self.env.reset()
            self._obs = nobs
        batch = SampleBatch({k: np.asarray(v, np.float32) for k, v in rows.items()})
        self.buffer.add(batch)
        self._counters["num_env_steps_sampled"] += batch.count
        self._timesteps_total += batch.count
        stats: Dict = {}
        if self._counters["num_env_steps_sampled"] > c.num_steps_sampled_before_learning_starts:
            for _ in range(max(1, batch.count // 10)):
                stats = self._learn(self.buffer.sample(c.train_batch_size))
                self._counters["num_env_steps_trained"] += c.train_batch_size
        return stats

    def step(self) -> Dict:
        c = self.algo_config
        ts0 = self._counters["num_env_steps_sampled"]
        res: Dict = {}
        while self._counters["num_env_steps_sampled"] - ts0 < (c.min_sample_timesteps_per_iteration or 1):
            res = self.training_step()
        h = list(self._episode_history)
        return {"episode_reward_mean": float(np.mean(h)) if h else float("nan"), "episodes_total": self._episodes_total,
                "timesteps_total": self._timesteps_total, "num_env_steps_sampled": self._counters["num_env_steps_sampled"],
                "num_env_steps_trained": self._counters["num_env_steps_trained"],
                "info": {"learner": res, **dict(self._counters)}}

    def evaluate_greedy(self, episodes: int = 10) -> float:
        env = make_env(self.algo_config.env, self.algo_config.env_config)
        tot = []
        for k in range(episodes):
            o, done, ret = env.reset(seed=1000 + k), False, 0.0
            while not done:
                o, r, d, _ = env.step(self.compute_actions(o, explore=False))
                ret += float(np.mean(list(r.values())))
                done = d["__all__"]
            tot.append(ret)
        return float(np.mean(tot))

    def get_weights(self):
        return {"actors": {k: v.cpu() for k, v in self.actors.state_dict().items()},
                "critics": {k: v.cpu() for k, v in self.critics.state_dict().items()}}

    def set_weights(self, w):
        self.actors.load_state_dict(w["actors"])
        self.critics.load_state_dict(w["critics"])

    def cleanup(self):
        pass


DEFAULT_CONFIG = MADDPGConfig().to_dict()
