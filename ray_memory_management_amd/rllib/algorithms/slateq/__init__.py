"""SlateQ: Q-learning for slate recommendation via item-wise Q decomposition.

Parity: reference rllib/algorithms/slateq/slateq.py (SlateQConfig: slate_size, fcnet hiddens for the
user/doc embeddings, lr 1e-3 (choice model lr 1e-3), target_network_update_freq, epsilon-greedy
over slates, replay buffer, double-Q off) and slateq_torch_policy.py / slateq_torch_model.py
(Q(s, A) = Σ_{i∈A} P(i | s, A) · Q̄(s, i) with a conditional-logit user choice model
P(i | s, A) = exp(v(s, i)) / (exp(v_no_click) + Σ_j exp(v(s, j))); Q̄ learned by TD on the clicked
item with target max over slates of Σ P·Q̄'; slate chosen greedily by the top-k of P·Q̄) and the
RecSim interest-evolution environment (replaced here by a synthetic user-interest env:
`SlateRecEnv`, since recsim is not installed).
"""
from __future__ import annotations

import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.env import make_env, register_env
from ray_memory_management_amd.rllib.utils.replay_buffers import ReplayBuffer
from ray_memory_management_amd.rllib.sample_batch import SampleBatch
from ray_memory_management_amd.rllib.utils.schedules import PiecewiseSchedule


class SlateRecEnv:
    """User with a unit interest vector u; each step offers `num_candidates` documents (unit topic
    vectors d_j, quality q_j); the agent shows `slate_size` of them; the user clicks item i with
    probability ∝ exp(β u·d_i) (or nothing, weight exp(β·no_click)); the reward is the clicked
    document's quality·(1 + u·d) engagement; interest drifts toward what was clicked. Episodes
    last `episode_len` steps. Observation: {"user": u, "doc": [N, dim], "quality": [N]}."""

    def __init__(self, config=None):
        c = config or {}
        self.dim, self.N, self.k = int(c.get("dim", 4)), int(c.get("num_candidates", 10)), int(c.get("slate_size", 2))
        self.beta, self.no_click = float(c.get("beta", 4.0)), float(c.get("no_click", 0.0))
        self.episode_len = int(c.get("episode_len", 20))
        self.rng = np.random.default_rng(c.get("seed"))

    def _docs(self):
        d = self.rng.standard_normal((self.N, self.dim))
        self.doc = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
        self.quality = self.rng.uniform(0.0, 1.0, self.N).astype(np.float32)

    def _obs(self):
        return {"user": self.u.copy(), "doc": self.doc.copy(), "quality": self.quality.copy()}

    def reset(self, *, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        u = self.rng.standard_normal(self.dim)
        self.u = (u / np.linalg.norm(u)).astype(np.float32)
        self.t = 0
        self._docs()
        return self._obs()

    def step(self, slate):
        slate = [int(i) for i in slate]
        logits = np.array([self.beta * float(self.u @ self.doc[i]) for i in slate] + [self.beta * self.no_click])
        p = np.exp(logits - logits.max())
        p /= p.sum()
        c = int(self.rng.choice(len(p), p=p))
        reward, clicked = 0.0, -1
        if c < len(slate):
            clicked = slate[c]
            reward = float(self.quality[clicked] * (1.0 + self.u @ self.doc[clicked]))
            u = self.u + 0.1 * self.doc[clicked]
            self.u = (u / np.linalg.norm(u)).astype(np.float32)
        self.t += 1
        self._docs()
        return self._obs(), reward, self.t >= self.episode_len, {"click": c if c < len(slate) else -1,
                                                                   "clicked_doc": clicked}


register_env("SlateRecEnv-v0", SlateRecEnv)


class SlateQModel(nn.Module):
    """Q̄(s, i) and the choice-model score v(s, i) from [user, doc, quality] features."""

    def __init__(self, dim: int, hidden: int = 64):
        super().__init__()
        f = 2 * dim + 1 + dim  # user, doc, quality, user*doc
        self.q = nn.Sequential(nn.Linear(f, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                               nn.Linear(hidden, 1))
        self.choice = nn.Linear(f, 1)
        self.no_click = nn.Parameter(torch.zeros(()))

    @staticmethod
    def feats(user, doc, quality):  # user [B, d], doc [B, N, d], quality [B, N]
        u = user.unsqueeze(1).expand_as(doc)
        return torch.cat([u, doc, quality.unsqueeze(-1), u * doc], -1)

    def forward(self, user, doc, quality):
        f = self.feats(user, doc, quality)
        return self.q(f).squeeze(-1), self.choice(f).squeeze(-1)  # [B, N] each


def slate_value(qbar, score, no_click, slates):
    """Σ_{i∈slate} P(i|s,slate) Q̄(s,i) for slates [B, k] (item indices)."""
    s = torch.gather(score, 1, slates)
    q = torch.gather(qbar, 1, slates)
    e = torch.exp(s - torch.maximum(s.max(1, keepdim=True).values, no_click.expand(s.shape[0], 1)))
    e0 = torch.exp(no_click - torch.maximum(s.max(1).values, no_click.expand(s.shape[0])))
    return (e * q).sum(1) / (e.sum(1) + e0)


def greedy_slates(qbar, score, k: int):
    """Top-k by exp(v)·Q̄ (the reference's greedy slate optimisation)."""
    return torch.topk(torch.exp(score - score.max(1, keepdim=True).values) * qbar, k, dim=1).indices


class SlateQConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or SlateQ)
        self.lr = 1e-3
        self.lr_choice_model = 1e-3
        self.gamma = 0.9
        self.slate_size = 2
        self.train_batch_size = 64
        self.target_network_update_freq = 800
        self.num_steps_sampled_before_learning_starts = 500
        self.rollout_fragment_length = 4
        self.num_workers = 0
        self.min_sample_timesteps_per_iteration = 500
        self.replay_buffer_config = {"capacity": 100000}
        self.exploration_config = {"initial_epsilon": 1.0, "final_epsilon": 0.05, "epsilon_timesteps": 5000}
        self.fcnet_hiddens_per_candidate = [64]


class SlateQ(Algorithm):
    _config_class = SlateQConfig

    def setup(self, config: Dict):
        import collections

        import ray_memory_management_amd as ray

        if not ray.is_initialized():
            ray.init()
        c = self.algo_config
        self.validate_config(c)
        self.env = make_env(c.env, {"slate_size": c.slate_size, **(c.env_config or {})})
        self._obs = self.env.reset(seed=c.seed)
        if c.seed is not None:
            torch.manual_seed(int(c.seed))
        self.m = SlateQModel(self.env.dim, int(c.fcnet_hiddens_per_candidate[0]))
        self.t = copy.deepcopy(self.m)
        self.q_opt = torch.optim.Adam(self.m.q.parameters(), lr=c.lr)
        self.c_opt = torch.optim.Adam(list(self.m.choice.parameters()) + [self.m.no_click], lr=c.lr_choice_model)
        self.buffer = ReplayBuffer(int(c.replay_buffer_config.get("capacity", 100000)), seed=c.seed)
        ec = c.exploration_config
        self.eps = PiecewiseSchedule([[0, ec.get("initial_epsilon", 1.0)],
                                      [ec.get("epsilon_timesteps", 5000), ec.get("final_epsilon", 0.05)]])
        self.rng = np.random.default_rng(c.seed)
        self._counters = collections.Counter()
        self._episode_history = collections.deque(maxlen=100)
        self._ret, self._timesteps_total, self._episodes_total = 0.0, 0, 0
        self._last_target = 0
        self.workers = None
        self._multi_agent = False
        self.callbacks = None

    @staticmethod
    def _t(o):
        return (torch.as_tensor(np.asarray(o["user"]))[None], torch.as_tensor(np.asarray(o["doc"]))[None],
                torch.as_tensor(np.asarray(o["quality"]))[None])

    @torch.no_grad()
    def compute_slate(self, obs, explore: bool = False):
        k = self.algo_config.slate_size
        if explore and self.rng.random() < self.eps(self._counters["num_env_steps_sampled"]):
            return self.rng.choice(len(obs["quality"]), size=k, replace=False)
        qbar, score = self.m(*self._t(obs))
        return greedy_slates(qbar, score, k)[0].numpy()

    def _learn(self, b) -> Dict:
        c = self.algo_config
        f = lambda k: torch.as_tensor(np.asarray(b[k]))  # noqa: E731
        user, doc, qual, slate, click = f("user"), f("doc"), f("quality"), f("slate").long(), f("click").long()
        rew, done = f("rewards").float(), f("dones").float()
        nuser, ndoc, nqual = f("n_user"), f("n_doc"), f("n_quality")
        qbar, score = self.m(user, doc, qual)
        # choice model: conditional logit over the shown slate + "no click"
        s = torch.gather(score, 1, slate)
        logits = torch.cat([s, self.m.no_click.expand(len(s), 1)], 1)
        tgt = torch.where(click >= 0, click, torch.full_like(click, slate.shape[1]))
        choice_loss = nn.functional.cross_entropy(logits, tgt)
        self.c_opt.zero_grad(set_to_none=True)
        choice_loss.backward()
        self.c_opt.step()
        # item-wise TD on the clicked document only (no click → no Q̄ update)
        with torch.no_grad():
            tq, ts = self.t(nuser, ndoc, nqual)
            _, cs = self.m(nuser, ndoc, nqual)
            nsl = greedy_slates(tq, cs, slate.shape[1])
            v_next = slate_value(tq, cs, self.m.no_click.detach(), nsl)
            y = rew + c.gamma * (1.0 - done) * v_next
        clicked = click >= 0
        qbar, _ = self.m(user, doc, qual)
        q_click = torch.gather(qbar, 1, torch.gather(slate, 1, tgt.clamp(max=slate.shape[1] - 1).unsqueeze(1))).squeeze(1)
        td = (q_click - y)[clicked]
        q_loss = (td ** 2).mean() if clicked.any() else torch.zeros((), requires_grad=True)
        self.q_opt.zero_grad(set_to_none=True)
        q_loss.backward()
        self.q_opt.step()
        return {"q_loss": float(q_loss.detach()), "choice_loss": float(choice_loss.detach())}

    def training_step(self) -> Dict:
        c = self.algo_config
        rows = {k: [] for k in ("user", "doc", "quality", "slate", "click", "rewards", "dones", "n_user", "n_doc",
                                "n_quality")}
        for _ in range(int(c.rollout_fragment_length)):
            sl = self.compute_slate(self._obs, explore=True)
            nobs, r, d, info = self.env.step(sl)
            clicked_pos = int(info["click"])
            for k, v in (("user", self._obs["user"]), ("doc", self._obs["doc"]), ("quality", self._obs["quality"]),
                         ("slate", np.asarray(sl, np.int64)), ("click", clicked_pos), ("rewards", r),
                         ("dones", float(d)), ("n_user", nobs["user"]), ("n_doc", nobs["doc"]),
                         ("n_quality", nobs["quality"])):
                rows[k].append(v)
            self._ret += r
            if d:
                self._episode_history.append(self._ret)
                self._episodes_total += 1
                self._ret = 0.0
                nobs = self.env.reset()
            self._obs = nobs
        b = SampleBatch({k: np.asarray(v) for k, v in rows.items()})
        self.buffer.add(b)
        self._counters["num_env_steps_sampled"] += b.count
        self._timesteps_total += b.count
        st: Dict = {}
        ts = self._counters["num_env_steps_sampled"]
        if ts > c.num_steps_sampled_before_learning_starts:
            st = self._learn(self.buffer.sample(c.train_batch_size))
            self._counters["num_env_steps_trained"] += c.train_batch_size
            if ts - self._last_target >= c.target_network_update_freq:
                self.t.load_state_dict(self.m.state_dict())
                self._last_target = ts
        return st

    def step(self) -> Dict:
        c = self.algo_config
        ts0 = self._counters["num_env_steps_sampled"]
        res: Dict = {}
        while self._counters["num_env_steps_sampled"] - ts0 < (c.min_sample_timesteps_per_iteration or 1):
            res = self.training_step()
        h = list(self._episode_history)
        return {"episode_reward_mean": float(np.mean(h)) if h else float("nan"), "episodes_total": self._episodes_total,
                "timesteps_total": self._timesteps_total, "num_env_steps_sampled": self._counters["num_env_steps_sampled"],
                "info": {"learner": {"default_policy": {"learner_stats": res}}, **dict(self._counters)}}

    def evaluate_policy(self, episodes: int = 20, random_slates: bool = False) -> float:
        env = make_env(self.algo_config.env, {"slate_size": self.algo_config.slate_size,
                                              **(self.algo_config.env_config or {})})
        rng = np.random.default_rng(123)
        tot = []
        for k in range(episodes):
            o, done, ret = env.reset(seed=5000 + k), False, 0.0
            while not done:
                sl = rng.choice(len(o["quality"]), size=self.algo_config.slate_size, replace=False) if random_slates \
                    else self.compute_slate(o)
                o, r, done, _ = env.step(sl)
                ret += r
            tot.append(ret)
        return float(np.mean(tot))

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.m.state_dict().items()}

    def set_weights(self, w):
        self.m.load_state_dict(w)

    def cleanup(self):
        pass


DEFAULT_CONFIG = SlateQConfig().to_dict()
