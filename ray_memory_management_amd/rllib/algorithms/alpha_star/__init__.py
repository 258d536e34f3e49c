"""AlphaStar-style league training.

Parity: reference rllib/algorithms/alpha_star/alpha_star.py (AlphaStarConfig: a league of
main agents, main exploiters and league exploiters, frozen snapshots added to the league when a
learner's win rate passes `win_rate_threshold_for_new_snapshot`, `max_num_policies_to_train`;
training_step: sample matches, update every trainable policy, update the win-rate table, let the
league builder add snapshots and re-route matchmaking), league_builder.py (AlphaStarLeagueBuilder:
prioritised fictitious self-play — main agents sample opponents with weight (1 − p_win)², main
exploiters play the current main agent, league exploiters play the whole league) and
rllib/examples/env/rock_paper_scissors.py (the competitive 2-player test env).

Here each learner policy trains with the multi-agent PG/A2C machinery (`Algorithm._ma_*`):
rollout workers hold a growing policy map (`add_policy`) and a matchmaking function that pairs
agent 0 (a trainable league member, round-robin) with a PFSP-sampled opponent for agent 1.
"""
from __future__ import annotations

import collections
import copy
import random
from typing import Dict, List

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.a2c import A2C, A2CConfig
from ray_memory_management_amd.rllib.env import Box, Discrete, MultiAgentEnv, register_env


class RockPaperScissorsEnv(MultiAgentEnv):
    """Two players, `episode_len` rounds; obs = one-hot of the opponent's previous move (+ "none");
    reward +1 win / −1 loss / 0 draw per round (zero-sum)."""

    BEATS = {0: 2, 1: 0, 2: 1}  # rock beats scissors, paper beats rock, scissors beat paper

    def __init__(self, config=None):
        c = config or {}
        self.episode_len = int(c.get("episode_len", 10))
        self._agent_ids = {0, 1}
        self.observation_space = Box(0.0, 1.0, shape=(4,), dtype=np.float32)
        self.action_space = Discrete(3)
        self.t = 0
        self.last = {0: 3, 1: 3}

    def _obs(self):
        return {i: np.eye(4, dtype=np.float32)[self.last[1 - i]] for i in (0, 1)}

    def reset(self, *, seed=None):
        self.t, self.last = 0, {0: 3, 1: 3}
        return self._obs()

    def step(self, action_dict):
        a0, a1 = int(action_dict[0]), int(action_dict[1])
        r0 = 0.0 if a0 == a1 else (1.0 if self.BEATS[a0] == a1 else -1.0)
        self.last = {0: a0, 1: a1}
        self.t += 1
        d = self.t >= self.episode_len
        return self._obs(), {0: r0, 1: -r0}, {0: d, 1: d, "__all__": d}, {}


register_env("RockPaperScissors-v0", RockPaperScissorsEnv)


class _Matchmaker:
    """Picklable policy-mapping function carrying the league's matchmaking table."""

    def __init__(self, learners: List[str], opponents: Dict[str, List], seed: int = 0):
        self.learners, self.opponents = learners, opponents  # learner -> [(opponent, weight)]
        self.rng = random.Random(seed)
        self._pair = {}

    def __call__(self, agent_id, episode=None, worker=None, **kw):
        pair = self._pair.get(episode)
        if pair is None:
            learner = self.learners[(episode or 0) % len(self.learners)]
            opps = self.opponents.get(learner) or [(learner, 1.0)]
            names, w = zip(*opps)
            pair = self._pair[episode] = (learner, self.rng.choices(names, weights=w)[0])
            if len(self._pair) > 64:
                self._pair.pop(next(iter(self._pair)))
        return pair[0] if agent_id == 0 else pair[1]


class AlphaStarConfig(A2CConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or AlphaStar)
        self.league_builder_config = {"num_main_exploiters": 1, "num_league_exploiters": 1,
                                      "win_rate_threshold_for_new_snapshot": 0.9, "min_matches_for_snapshot": 20,
                                      "num_random_policies": 1}
        self.max_num_policies_to_train = 8
        self.num_workers = 2
        self.rollout_fragment_length = 50
        self.train_batch_size = 400
        self.lr = 3e-3
        self.entropy_coeff = 0.01
        self.model = {**self.model, "fcnet_hiddens": [32]}


class _RandomPolicy:
    """League seed opponent: uniformly random moves (reference num_random_policies)."""

    def __init__(self, observation_space, action_space, config, device="cpu"):
        from ray_memory_management_amd.rllib.policy import TorchPolicy

        self._p = TorchPolicy(observation_space, action_space, config, device)
        self.model = self._p.model
        self.action_space = action_space
        self.global_timestep = 0
        self._rng = np.random.default_rng(config.get("seed"))
        p = config.get("league_random_policy_probs")  # optional move bias of the seed opponents
        self._probs = None if p is None else np.asarray(p, np.float64) / np.sum(p)

    def compute_actions(self, obs_batch, explore=True):
        from ray_memory_management_amd.rllib.sample_batch import SampleBatch

        n = len(obs_batch)
        probs = self._probs if self._probs is not None else None
        a = self._rng.choice(self.action_space.n, size=n, p=probs)
        z = np.zeros(n, np.float32)
        return a, [], {SampleBatch.ACTION_LOGP: z - np.log(self.action_space.n), SampleBatch.VF_PREDS: z,
                       SampleBatch.ACTION_DIST_INPUTS: np.zeros((n, self.action_space.n), np.float32)}

    def value(self, obs_batch):
        return np.zeros(len(obs_batch), np.float32)

    def get_weights(self):
        return self._p.get_weights()

    def set_weights(self, w):
        self._p.set_weights(w)


class AlphaStar(A2C):
    _config_class = AlphaStarConfig

    @classmethod
    def _initial_policies(cls, lb):
        learners = ["main_0"] + [f"main_exploiter_{i}" for i in range(lb.get("num_main_exploiters", 1))] + \
                   [f"league_exploiter_{i}" for i in range(lb.get("num_league_exploiters", 1))]
        frozen = [f"random_{i}" for i in range(lb.get("num_random_policies", 1))]
        return learners, frozen

    def setup(self, config):
        c = self.algo_config
        learners, frozen = self._initial_policies(c.league_builder_config)
        pols = {p: None for p in learners}
        pols.update({p: (_RandomPolicy, None, None, {}) for p in frozen})
        c.multiagent = {"policies": pols, "policy_mapping_fn": _Matchmaker(learners, {}, c.seed or 0),
                        "policies_to_train": learners}
        self.learners, self.league = list(learners), list(frozen)
        self.win = collections.defaultdict(lambda: [0.0, 0])  # (a, b) -> [a's wins + 0.5 draws, games]
        self._snapshots = 0
        super().setup(config)
        self._push_matchmaking()

    def _p_win(self, a, b) -> float:
        w, n = self.win[(a, b)]
        return (w + 0.5) / (n + 1.0)

    def _opponents(self) -> Dict[str, List]:
        everyone = self.league + self.learners
        out = {}
        for lp in self.learners:
            if lp.startswith("main_exploiter"):
                cands = [(p, 1.0) for p in self.learners if p.startswith("main_")] or [("main_0", 1.0)]
            elif lp.startswith("league_exploiter"):
                cands = [(p, 1.0) for p in everyone if p != lp]
            else:  # main agents: prioritised fictitious self-play over the whole league
                cands = [(p, (1.0 - self._p_win(lp, p)) ** 2 + 1e-3) for p in everyone]
            out[lp] = cands
        return out

    def _push_matchmaking(self):
        mm = _Matchmaker(self.learners, self._opponents(), random.randrange(1 << 30))
        self.workers.local_worker().set_policy_mapping_fn(mm)
        if self.workers.remote_workers():
            ray.get([w.set_policy_mapping_fn.remote(mm) for w in self.workers.remote_workers()])

    def _record_matches(self):
        res = list(self.workers.local_worker().take_match_results())
        if self.workers.remote_workers():
            for r in ray.get([w.take_match_results.remote() for w in self.workers.remote_workers()]):
                res += r
        for _, rets in res:
            if len(rets) != 2:
                continue
            (a, ra), (b, rb) = rets.items()
            score = 1.0 if ra > rb else (0.5 if ra == rb else 0.0)
            self.win[(a, b)][0] += score
            self.win[(a, b)][1] += 1
            self.win[(b, a)][0] += 1.0 - score
            self.win[(b, a)][1] += 1
        return len(res)

    def _maybe_snapshot(self) -> List[str]:
        lb = self.algo_config.league_builder_config
        added = []
        for lp in list(self.learners):
            games = sum(self.win[(lp, o)][1] for o in self.league + self.learners if o != lp)
            if games < lb.get("min_matches_for_snapshot", 20):
                continue
            wr = sum(self.win[(lp, o)][0] for o in self.league) / max(1, sum(self.win[(lp, o)][1] for o in self.league))
            if wr >= lb.get("win_rate_threshold_for_new_snapshot", 0.9) and len(self.league) < 64:
                name = f"{lp}_v{self._snapshots}"
                self._snapshots += 1
                w = self.ma_learners[lp].get_weights()
                from ray_memory_management_amd.rllib.policy import TorchPolicy

                self.workers.local_worker().add_policy(name, TorchPolicy, weights=w)
                wref = ray.put(w)
                if self.workers.remote_workers():
                    ray.get([wk.add_policy.remote(name, TorchPolicy, None, None, None, wref)
                             for wk in self.workers.remote_workers()])
                self.league.append(name)
                for o in self.league + self.learners:  # a fresh snapshot starts with a clean record
                    self.win.pop((lp, o), None)
                added.append(name)
        return added

    def training_step(self) -> Dict:
        stats = self._ma_training_step()
        n = self._record_matches()
        added = self._maybe_snapshot()
        self._push_matchmaking()
        league = {f"win_rate/{lp}_vs_{o}": round(self._p_win(lp, o), 3)
                  for lp in self.learners for o in self.league}
        out = {pid: dict(st) for pid, st in stats.items()}
        out["league"] = {"size": len(self.league) + len(self.learners), "matches": n, "snapshots_added": added,
                         **league}
        return out


DEFAULT_CONFIG = AlphaStarConfig().to_dict()
