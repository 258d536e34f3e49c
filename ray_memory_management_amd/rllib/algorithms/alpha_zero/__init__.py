"""AlphaZero (single-player): MCTS guided by a policy/value network, trained on the search's visit
distributions and ranked episode returns.

Parity: reference rllib/algorithms/alpha_zero/alpha_zero.py (AlphaZeroConfig: mcts_config
{puct_coefficient 1.0, num_simulations 30, temperature 1.5, dirichlet_epsilon 0.25,
dirichlet_noise 0.03, argmax_tree_policy False, add_dirichlet_noise True}, ranked_rewards
{enable, percentile 75, buffer_max_length 1000, initialize_buffer 100}, replay of whole episodes,
num_sgd_iter 30, sgd_minibatch_size 128, lr 5e-5), mcts.py (Node / RootParentNode, PUCT selection,
expansion with network priors, backup of the value), ranked_rewards.py (R2: +1 above the running
percentile, −1 below), alpha_zero_policy.py (loss = −Σ π_mcts log π + (v − z)²) and
rllib/examples/env/cartpole_sparse_rewards.py (CartPole with the return paid at the end, cloneable
via get_state / set_state).
"""
from __future__ import annotations

import collections
import copy
import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.env import CartPoleEnv, make_env, register_env
from ray_memory_management_amd.rllib.sample_batch import SampleBatch, concat_samples


class CartPoleSparseRewards(CartPoleEnv):
    """CartPole whose reward is paid in one lump when the episode ends; state clone/restore."""

    def __init__(self, config=None):
        super().__init__(config)
        self._ret = 0.0

    def reset(self, *, seed=None):
        self._ret = 0.0
        return super().reset(seed=seed)

    def step(self, action):
        o, r, d, i = super().step(action)
        self._ret += r
        return o, (self._ret if d else 0.0), d, i

    def get_state(self):
        return (self.state.copy(), self.steps, self._ret)

    def set_state(self, st):
        self.state, self.steps, self._ret = st[0].copy(), st[1], st[2]
        return self.state.astype(np.float32)


register_env("CartPoleSparseRewards-v1", CartPoleSparseRewards)


class PolicyValueNet(nn.Module):
    def __init__(self, obs_dim, n_actions, hiddens=(64, 64)):
        super().__init__()
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), nn.ReLU()]
            d = h
        self.body = nn.Sequential(*layers)
        self.pi = nn.Linear(d, n_actions)
        self.v = nn.Linear(d, 1)

    def forward(self, obs):
        h = self.body(obs.float())
        return self.pi(h), torch.tanh(self.v(h)).squeeze(-1)

    @torch.no_grad()
    def evaluate(self, obs):
        logits, v = self(torch.as_tensor(np.asarray(obs, np.float32))[None])
        return torch.softmax(logits, -1)[0].numpy(), float(v[0])


class Node:
    __slots__ = ("state", "obs", "reward", "done", "parent", "action", "children", "prior", "N", "W", "expanded")

    def __init__(self, state, obs, reward, done, parent, action, n_actions):
        self.state, self.obs, self.reward, self.done = state, obs, reward, done
        self.parent, self.action = parent, action
        self.children: Dict[int, "Node"] = {}
        self.prior = np.zeros(n_actions, np.float64)
        self.N = np.zeros(n_actions, np.float64)
        self.W = np.zeros(n_actions, np.float64)
        self.expanded = False


class MCTS:
    def __init__(self, model: PolicyValueNet, env, cfg: Dict, rng):
        self.model, self.env, self.c, self.rng = model, env, cfg, rng
        self.A = env.action_space.n

    def _child(self, node: Node, a: int) -> Node:
        ch = node.children.get(a)
        if ch is None:
            self.env.set_state(node.state)
            o, r, d, _ = self.env.step(a)
            ch = node.children[a] = Node(self.env.get_state(), o, r, d, node, a, self.A)
        return ch

    def search(self, root: Node):
        """Runs num_simulations; returns (visit-count policy, chosen action)."""
        c = self.c
        if not root.expanded:
            p, _ = self.model.evaluate(root.obs)
            root.prior, root.expanded = p, True
        if c.get("add_dirichlet_noise", True):
            noise = self.rng.dirichlet([c.get("dirichlet_noise", 0.03)] * self.A)
            eps = c.get("dirichlet_epsilon", 0.25)
            root.prior = (1 - eps) * root.prior + eps * noise
        for _ in range(int(c.get("num_simulations", 30))):
            node = root
            while node.expanded and not node.done:  # PUCT selection
                q = np.where(node.N > 0, node.W / np.maximum(node.N, 1), 0.0)
                u = c.get("puct_coefficient", 1.0) * node.prior * math.sqrt(node.N.sum() + 1) / (1 + node.N)
                node = self._child(node, int(np.argmax(q + u)))
            if node.done:
                value = self._terminal_value(node)
            else:
                p, value = self.model.evaluate(node.obs)
                node.prior, node.expanded = p, True
            while node.parent is not None:  # backup
                a, node = node.action, node.parent
                node.N[a] += 1
                node.W[a] += value
        counts = root.N
        if c.get("argmax_tree_policy", False):
            pi = np.eye(self.A)[int(np.argmax(counts))]
        else:
            t = float(c.get("temperature", 1.5))
            x = counts ** (1.0 / t)
            pi = x / x.sum() if x.sum() > 0 else np.full(self.A, 1.0 / self.A)
        a = int(self.rng.choice(self.A, p=pi))
        return pi, a

    def _terminal_value(self, node: Node) -> float:
        return float(self.c["value_fn"](node.reward)) if "value_fn" in self.c else float(np.sign(node.reward))


class RankedRewards:
    """R2 buffer: an episode return maps to +1 above the running percentile, −1 below (ties ±1 at
    random), so the value target is a self-play-like win/loss signal."""

    def __init__(self, percentile=75, maxlen=1000, rng=None):
        self.buf = collections.deque(maxlen=maxlen)
        self.percentile, self.rng = percentile, rng or np.random.default_rng()

    def add(self, r):
        self.buf.append(r)

    def normalize(self, r) -> float:
        if not self.buf:
            return 0.0
        thr = float(np.percentile(np.asarray(self.buf), self.percentile))
        if r > thr:
            return 1.0
        if r < thr:
            return -1.0
        return float(self.rng.choice([-1.0, 1.0]))


def play_episodes(worker, weights, cfg: Dict, n_episodes: int, ranked_state):
    """Runs inside a RolloutWorker: MCTS self-play episodes with the given network weights.
    Returns (batch with obs / mcts_policies / returns, episode returns)."""
    env = getattr(worker, "_az_env", None)
    if env is None:
        ec = worker.config.get("env_config") or {}
        env = worker._az_env = make_env(worker.config.get("env"), ec)
        worker._az_rng = np.random.default_rng(worker.config.get("seed"))
        o = env.reset()
        worker._az_model = PolicyValueNet(len(o), env.action_space.n, tuple((worker.config.get("model") or {})
                                                                           .get("fcnet_hiddens", (64, 64))))
    model, rng = worker._az_model, worker._az_rng
    model.load_state_dict({k: torch.as_tensor(v) for k, v in weights.items()})
    rr = RankedRewards(cfg.get("percentile", 75), rng=rng)
    for r in ranked_state:
        rr.add(r)
    mcfg = dict(cfg["mcts_config"])
    if cfg.get("ranked_rewards", True):
        mcfg["value_fn"] = rr.normalize
    batches, rets = [], []
    for _ in range(n_episodes):
        o = env.reset()
        root = Node(env.get_state(), o, 0.0, False, None, None, env.action_space.n)
        tree = MCTS(model, env, mcfg, rng)
        obs, pis, done, ret, r = [], [], False, 0.0, 0.0
        while not done:
            pi, a = tree.search(root)
            obs.append(np.asarray(root.obs, np.float32))
            pis.append(pi.astype(np.float32))
            root = tree._child(root, a)
            root.parent = None  # re-root: keep the subtree statistics
            r, done = root.reward, root.done
            ret += r
        rets.append(ret)
        z = rr.normalize(ret) if cfg.get("ranked_rewards", True) else ret
        rr.add(ret)
        batches.append(SampleBatch({"obs": np.stack(obs), "mcts_policies": np.stack(pis),
                                    "value_label": np.full(len(obs), z, np.float32)}))
    return concat_samples(batches), rets


class AlphaZeroConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or AlphaZero)
        self.sgd_minibatch_size = 128
        self.shuffle_sequences = True
        self.num_sgd_iter = 30
        self.lr = 5e-5
        self.train_batch_size = 4000
        self.rollout_fragment_length = 200
        self.num_workers = 2
        self.episodes_per_worker = 1
        self.replay_buffer_config = {"capacity": 1000}  # episodes
        self.mcts_config = {"puct_coefficient": 1.0, "num_simulations": 30, "temperature": 1.5,
                            "dirichlet_epsilon": 0.25, "dirichlet_noise": 0.03, "argmax_tree_policy": False,
                            "add_dirichlet_noise": True}
        self.ranked_rewards = {"enable": True, "percentile": 75, "buffer_max_length": 1000, "initialize_buffer": 100}
        self.model = {"fcnet_hiddens": [64, 64]}


class AlphaZero(Algorithm):
    _config_class = AlphaZeroConfig

    def _setup_learner(self):
        c = self.algo_config
        env = make_env(c.env, c.env_config)
        if not (hasattr(env, "get_state") and hasattr(env, "set_state")):
            raise ValueError("AlphaZero needs a cloneable env (get_state / set_state)")
        o = env.reset()
        if c.seed is not None:
            torch.manual_seed(int(c.seed))
        self.net = PolicyValueNet(len(o), env.action_space.n, tuple(c.model.get("fcnet_hiddens", (64, 64))))
        self.opt = torch.optim.Adam(self.net.parameters(), lr=c.lr)
        self.replay: collections.deque = collections.deque(maxlen=int(c.replay_buffer_config.get("capacity", 1000)))
        self.ranked = collections.deque(maxlen=int(c.ranked_rewards.get("buffer_max_length", 1000)))
        self.rng = np.random.default_rng(c.seed)
        self.eval_env = env

    def _weights(self):
        return {k: v.detach().cpu() for k, v in self.net.state_dict().items()}

    def training_step(self) -> Dict:
        c = self.algo_config
        cfg = {"mcts_config": c.mcts_config, "ranked_rewards": c.ranked_rewards.get("enable", True),
               "percentile": c.ranked_rewards.get("percentile", 75)}
        w = self._weights()
        ranked = list(self.ranked)
        workers = self.workers.remote_workers()
        if workers:
            wref = ray.put(w)
            outs = ray.get([wk.apply.remote(play_episodes, wref, cfg, c.episodes_per_worker, ranked) for wk in workers])
        else:
            outs = [play_episodes(self.workers.local_worker(), w, cfg, c.episodes_per_worker, ranked)]
        n = 0
        for b, rets in outs:
            self.replay.append(b)
            for r in rets:
                self.ranked.append(r)
                self._episode_history.append((r, 0))
                self._episodes_total += 1
            n += b.count
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        stats: Dict = {}
        if len(self.ranked) >= min(int(c.ranked_rewards.get("initialize_buffer", 100)), 10 ** 9) or \
                not c.ranked_rewards.get("enable", True):
            data = concat_samples(list(self.replay))
            obs = torch.as_tensor(np.asarray(data["obs"]))
            pis = torch.as_tensor(np.asarray(data["mcts_policies"]))
            z = torch.as_tensor(np.asarray(data["value_label"]))
            mb = min(int(c.sgd_minibatch_size), len(z))
            for _ in range(int(c.num_sgd_iter)):
                idx = torch.as_tensor(self.rng.permutation(len(z))[:mb])
                logits, v = self.net(obs[idx])
                pl = -(pis[idx] * torch.log_softmax(logits, -1)).sum(-1).mean()
                vl = ((v - z[idx]) ** 2).mean()
                self.opt.zero_grad(set_to_none=True)
                (pl + vl).backward()
                self.opt.step()
                stats = {"policy_loss": float(pl.detach()), "value_loss": float(vl.detach())}
            self._counters["num_env_steps_trained"] += mb * int(c.num_sgd_iter)
        return stats

    def compute_single_action(self, observation, *, explore=None, **kw):
        p, _ = self.net.evaluate(observation)
        return int(np.argmax(p))

    def get_weights(self):
        return self._weights()

    def set_weights(self, w):
        self.net.load_state_dict(w)


DEFAULT_CONFIG = AlphaZeroConfig().to_dict()
