"""R2D2: recurrent replay distributed DQN.

Parity: reference rllib/algorithms/r2d2/r2d2.py (R2D2Config: LSTM Q-model (lstm_cell_size 64,
max_seq_len 20), replay of fixed-length SEQUENCES with their stored initial recurrent state,
burn_in steps that only warm the state, zero_init_states, value rescaling
h(x) = sign(x)(sqrt(|x|+1) − 1) + εx (use_h_function, h_function_epsilon 1e-3), double-Q targets
from the target network, sequence priorities η·max|δ| + (1−η)·mean|δ|) and r2d2_torch_policy.py.

Sequences are columnar replay rows: one row = [L+1] observations, [L] actions / rewards / dones
and the LSTM (h, c) at the sequence start, so a training batch is one gather per column (the K2
row gather when the buffer lives in HBM). The learner unrolls an LSTMCell over the sequence and
resets the state after every `done`.
"""
from __future__ import annotations

import copy
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.dqn import DQN, DQNConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch
from ray_memory_management_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer
from ray_memory_management_amd.rllib.utils.schedules import PiecewiseSchedule


def h_function(x, eps: float = 1e-3):
    return torch.sign(x) * (torch.sqrt(torch.abs(x) + 1.0) - 1.0) + eps * x


def h_inverse(x, eps: float = 1e-3):
    two_eps = 2.0 * eps
    return torch.sign(x) * (((torch.sqrt(1.0 + 4.0 * eps * (torch.abs(x) + 1.0 + eps)) - 1.0) / two_eps) ** 2 - 1.0)


class RecurrentQModel(nn.Module):
    """obs → MLP → LSTMCell → (dueling) Q head."""

    def __init__(self, obs_dim: int, num_actions: int, hiddens=(64,), cell: int = 64, dueling: bool = True):
        super().__init__()
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), nn.ReLU()]
            d = h
        self.enc = nn.Sequential(*layers)
        self.lstm = nn.LSTMCell(d, cell)
        self.adv = nn.Linear(cell, num_actions)
        self.val = nn.Linear(cell, 1) if dueling else None
        self.cell = cell

    def initial_state(self, n: int, device=None):
        z = torch.zeros(n, self.cell, device=device)
        return z, z.clone()

    def step(self, obs, state):
        h, c = self.lstm(self.enc(obs.flatten(1).float()), state)
        a = self.adv(h)
        q = a if self.val is None else self.val(h) + a - a.mean(-1, keepdim=True)
        return q, (h, c)

    def unroll(self, obs_seq, state, resets):
        """obs_seq [B, L, ...], resets [B, L] (1 → zero the state BEFORE step t). Returns Q [B, L, A]."""
        h, c = state
        qs = []
        for t in range(obs_seq.shape[1]):
            keep = (1.0 - resets[:, t]).unsqueeze(-1)
            q, (h, c) = self.step(obs_seq[:, t], (h * keep, c * keep))
            qs.append(q)
        return torch.stack(qs, 1)


class R2D2Policy:
    """Epsilon-greedy recurrent policy for rollout workers (state kept per env slot)."""

    def __init__(self, observation_space, action_space, config: Dict, device="cpu"):
        self.observation_space, self.action_space, self.config = observation_space, action_space, config
        m = config.get("model") or {}
        self.model = RecurrentQModel(int(np.prod(observation_space.shape)), action_space.n,
                                     tuple(m.get("fcnet_hiddens", (64,))), int(m.get("lstm_cell_size", 64)),
                                     bool(config.get("dueling", True)))
        ec = dict(config.get("exploration_config") or {})
        self.eps = PiecewiseSchedule([[0, ec.get("initial_epsilon", 1.0)],
                                      [ec.get("epsilon_timesteps", 10000), ec.get("final_epsilon", 0.02)]])
        self._rng = np.random.default_rng(config.get("seed"))
        self.global_timestep = 0
        self.state = None

    @torch.no_grad()
    def act(self, obs, state, explore=True):
        q, state = self.model.step(torch.as_tensor(np.asarray(obs, np.float32)), state)
        a = q.argmax(-1).numpy()
        if explore:
            e = self.eps(self.global_timestep)
            rnd = self._rng.random(len(a)) < e
            a = np.where(rnd, self._rng.integers(0, q.shape[-1], size=len(a)), a)
        self.global_timestep += len(a)
        return a, state

    def compute_actions(self, obs_batch, explore: bool = True):  # stateless single-step API
        a, _ = self.act(obs_batch, self.model.initial_state(len(obs_batch)), explore)
        z = np.zeros(len(a), np.float32)
        return a, [], {SampleBatch.ACTION_LOGP: z, SampleBatch.VF_PREDS: z,
                       SampleBatch.ACTION_DIST_INPUTS: np.zeros((len(a), self.action_space.n), np.float32)}

    def compute_single_action(self, obs, explore: bool = False):
        if self.state is None:
            self.state = self.model.initial_state(1)
        a, self.state = self.act(np.asarray(obs)[None], self.state, explore)
        return int(a[0])

    def value(self, obs_batch):
        return np.zeros(len(obs_batch), np.float32)

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        self.model.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})


def sample_sequences(worker, L: int, explore: bool = True):
    """Runs inside a RolloutWorker: step every env L times with the recurrent policy and return
    one sequence row per env (obs [L+1], actions/rewards/dones [L], LSTM state at the start)."""
    pol = worker.policy
    env = worker.env
    n = env.num_envs
    if getattr(worker, "_r2d2_state", None) is None:
        worker._r2d2_state = pol.model.initial_state(n)
    h0, c0 = (x.clone() for x in worker._r2d2_state)
    obs_buf, act, rew, dn = [], [], [], []
    state = worker._r2d2_state
    obs = np.stack([np.asarray(o, np.float32) for o in worker._obs])
    for _ in range(L):
        a, state = pol.act(obs, state, explore)
        nobs, r, d, _ = env.vector_step(list(a))
        obs_buf.append(obs)
        act.append(a)
        rew.append(np.asarray(r, np.float32))
        dn.append(np.asarray(d, np.float32))
        worker._ep_reward += np.asarray(r, np.float64)
        worker._ep_len += 1
        keep = torch.ones(n, 1)
        for i in range(n):
            if d[i]:
                worker._completed.append((float(worker._ep_reward[i]), int(worker._ep_len[i])))
                worker._ep_reward[i], worker._ep_len[i] = 0.0, 0
                nobs[i] = env.reset_at(i)
                keep[i] = 0.0
        state = (state[0] * keep, state[1] * keep)  # zero_init_states on episode start
        obs = np.stack([np.asarray(o, np.float32) for o in nobs])
    worker._obs = list(obs)
    worker._r2d2_state = state
    # the observation after step t is obs_buf[t+1] unless the episode ended there (then the
    # target is masked by done), so [L+1] observations suffice
    obs_buf.append(obs)
    sw = lambda x: np.swapaxes(np.stack(x), 0, 1)  # noqa: E731  [L, n] -> [n, L]
    return SampleBatch({"obs_seq": sw(obs_buf), "act_seq": sw(act).astype(np.int64), "rew_seq": sw(rew),
                        "done_seq": sw(dn), "state_h": h0.numpy(), "state_c": c0.numpy()})


class R2D2Config(DQNConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or R2D2)
        self.zero_init_states = True
        self.use_h_function = True
        self.h_function_epsilon = 1e-3
        self.burn_in = 0
        self.replay_sequence_length = 20
        self.lr = 1e-4
        self.train_batch_size = 64  # sequences
        self.target_network_update_freq = 2500
        self.num_steps_sampled_before_learning_starts = 1000
        self.priority_eta = 0.9
        self.n_step = 1
        self.model = {**self.model, "use_lstm": True, "lstm_cell_size": 64, "max_seq_len": 20, "fcnet_hiddens": [64]}
        self.replay_buffer_config = {"type": "MultiAgentPrioritizedReplayBuffer", "capacity": 100000,
                                     "storage_unit": "sequences", "prioritized_replay_alpha": 0.6,
                                     "prioritized_replay_beta": 0.4, "prioritized_replay_eps": 1e-6}
        self.policy_class = "ray_memory_management_amd.rllib.algorithms.r2d2.R2D2Policy"


class R2D2Learner:
    def __init__(self, model: RecurrentQModel, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.q = model.to(self.device)
        self.target = copy.deepcopy(self.q)
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.cfg = cfg
        self.opt = torch.optim.Adam(self.q.parameters(), lr=cfg["lr"])

    def update(self, b: SampleBatch) -> Dict:
        c, dev = self.cfg, self.device
        t = lambda k, dt=torch.float32: torch.as_tensor(np.asarray(b[k]), device=dev).to(dt)  # noqa: E731
        obs, act, rew, done = t("obs_seq"), t("act_seq", torch.int64), t("rew_seq"), t("done_seq")
        B, L = act.shape
        state = (t("state_h"), t("state_c"))
        if c.get("zero_init_states", True):
            state = (torch.zeros_like(state[0]), torch.zeros_like(state[1]))
        # resets[t] = 1 if step t starts a new episode (the previous step ended one)
        resets = torch.cat([torch.zeros(B, 1, device=dev), done[:, :-1]], 1)
        resets_full = torch.cat([resets, done[:, -1:]], 1)
        q_all = self.q.unroll(obs, state, resets_full)  # [B, L+1, A]
        with torch.no_grad():
            qt_all = self.target.unroll(obs, state, resets_full)
            a_star = q_all[:, 1:].argmax(-1, keepdim=True)
            q_next = qt_all[:, 1:].gather(2, a_star).squeeze(2)
            eps = float(c.get("h_function_epsilon", 1e-3))
            if c.get("use_h_function", True):
                q_next = h_inverse(q_next, eps)
            y = rew + c["gamma"] * (1.0 - done) * q_next
            if c.get("use_h_function", True):
                y = h_function(y, eps)
        q_sel = q_all[:, :-1].gather(2, act.unsqueeze(2)).squeeze(2)
        burn = int(c.get("burn_in", 0))
        mask = torch.ones(B, L, device=dev)
        mask[:, :burn] = 0.0
        td = (q_sel - y) * mask
        w = t("weights") if "weights" in b else torch.ones(B, device=dev)
        loss = (w.unsqueeze(1) * torch.nn.functional.huber_loss(q_sel, y, reduction="none", delta=1.0) * mask).sum() \
            / mask.sum()
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if c.get("grad_clip"):
            nn.utils.clip_grad_norm_(self.q.parameters(), c["grad_clip"])
        self.opt.step()
        a = td.detach().abs()
        eta = float(c.get("priority_eta", 0.9))
        prio = eta * a.max(1).values + (1 - eta) * a.sum(1) / mask.sum(1).clamp_min(1.0)
        return {"loss": float(loss.detach()), "mean_q": float(q_sel.detach().mean()), "td_error": prio.cpu().numpy()}

    def sync_target(self):
        self.target.load_state_dict(self.q.state_dict())

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.q.state_dict().items()}

    def set_weights(self, w):
        self.q.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})
        self.sync_target()


class R2D2(DQN):
    _config_class = R2D2Config
    _supports_sequence_models = True  # its own recurrent Q-model (RecurrentQModel)

    def validate_config(self, c):
        super().validate_config(c)
        if c.burn_in >= c.replay_sequence_length:
            raise ValueError("burn_in must be shorter than replay_sequence_length")

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        local = self.workers.local_worker()
        self.learner = R2D2Learner(copy.deepcopy(local.policy.model),
                                   dict(lr=c.lr, gamma=c.gamma, grad_clip=c.grad_clip, burn_in=c.burn_in,
                                        use_h_function=c.use_h_function, h_function_epsilon=c.h_function_epsilon,
                                        zero_init_states=c.zero_init_states, priority_eta=c.priority_eta),
                                   device=dev)
        rb = dict(c.replay_buffer_config)
        self._prioritized = "Prioritized" in str(rb.get("type", ""))
        cap = max(1, int(rb.get("capacity", 100000)) // max(1, c.replay_sequence_length))
        self.buffer = (PrioritizedReplayBuffer(cap, alpha=rb.get("prioritized_replay_alpha", 0.6), seed=c.seed)
                       if self._prioritized else ReplayBuffer(cap, seed=c.seed))
        self._last_target_update = 0
        self._sync()

    def _sample(self) -> SampleBatch:
        from ray_memory_management_amd.rllib.sample_batch import concat_samples

        L = self.algo_config.replay_sequence_length
        if self.workers.remote_workers():
            return concat_samples(ray.get([w.apply.remote(sample_sequences, L) for w in self.workers.remote_workers()]))
        return sample_sequences(self.workers.local_worker(), L)

    def training_step(self) -> Dict:
        c = self.algo_config
        seqs = self._sample()
        self.buffer.add(seqs)
        n = seqs.count * c.replay_sequence_length  # env steps
        self._counters["num_env_steps_sampled"] += n
        self._timesteps_total += n
        ts = self._counters["num_env_steps_sampled"]
        stats: Dict = {}
        if ts > c.num_steps_sampled_before_learning_starts and len(self.buffer) >= c.train_batch_size:
            intensity = c.training_intensity
            n_up = max(1, int(round(intensity * n / (c.train_batch_size * c.replay_sequence_length)))) \
                if intensity else 1
            rb = c.replay_buffer_config
            for _ in range(n_up):
                tb = self.buffer.sample(c.train_batch_size, beta=rb.get("prioritized_replay_beta", 0.4)) \
                    if self._prioritized else self.buffer.sample(c.train_batch_size)
                out = self.learner.update(tb)
                if self._prioritized:
                    self.buffer.update_priorities(tb["batch_indexes"], out["td_error"] + rb.get("prioritized_replay_eps",
                                                                                              1e-6))
                stats = {k: v for k, v in out.items() if k != "td_error"}
                self._counters["num_env_steps_trained"] += c.train_batch_size * c.replay_sequence_length
            if ts - self._last_target_update >= c.target_network_update_freq:
                self.learner.sync_target()
                self._last_target_update = ts
                self._counters["num_target_updates"] += 1
            self._sync()
        stats["replay_buffer"] = self.buffer.stats()
        return stats


DEFAULT_CONFIG = R2D2Config().to_dict()
