"""Decision Transformer (offline RL as return-conditioned sequence modelling).

Parity: reference rllib/algorithms/dt/dt.py (DTConfig: target_return, horizon, embed_dim 128,
num_layers 2, num_heads 1, max_seq_len K 5, embed/attention/residual dropout 0.1, lr 1e-4,
lr warmup, train_batch_size 128 segments, loss_coef_actions 1; training_step = sample segments from
the offline episodes → one gradient step), segmentation_buffer.py (K-step windows of whole
episodes, left-padded with an attention mask, returns-to-go per step), dt_torch_model.py (tokens
(R̂_t, s_t, a_t) + timestep embeddings → causal GPT → action predicted from the state token) and
dt_torch_policy.py (evaluation: condition on the target return, subtract each reward).

On MI355X the transformer is plain torch (SDPA attention, bf16 autocast on the GPU); the episode
store is columnar numpy and a training batch is one fancy-index gather per column.
"""
from __future__ import annotations

import collections
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.env import make_env
from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class DTConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or DT)
        self.target_return = None
        self.horizon = None
        self.embed_dim = 128
        self.num_layers = 2
        self.num_heads = 1
        self.embed_pdrop = 0.1
        self.resid_pdrop = 0.1
        self.attn_pdrop = 0.1
        self.max_seq_len = 5
        self.lr = 1e-4
        self.lr_warmup_steps = 0
        self.weight_decay = 1e-4
        self.grad_clip = 0.25
        self.train_batch_size = 128
        self.loss_coef_actions = 1.0
        self.num_workers = 0
        self.min_train_timesteps_per_iteration = 0
        self.input_ = "sampler"


class DTModel(nn.Module):
    def __init__(self, obs_dim: int, num_actions: int, K: int, horizon: int, E: int, layers: int, heads: int,
                 pdrop: float, attn_pdrop: float):
        super().__init__()
        self.K, self.E, self.A = K, E, num_actions
        self.embed_t = nn.Embedding(horizon + 1, E)
        self.embed_r = nn.Linear(1, E)
        self.embed_s = nn.Linear(obs_dim, E)
        self.embed_a = nn.Embedding(num_actions + 1, E)  # last id = padding / unknown action
        self.ln = nn.LayerNorm(E)
        self.drop = nn.Dropout(pdrop)
        layer = nn.TransformerEncoderLayer(E, heads, 4 * E, dropout=attn_pdrop, activation="gelu", batch_first=True,
                                           norm_first=True)
        self.gpt = nn.TransformerEncoder(layer, layers)
        self.head = nn.Linear(E, num_actions)
        # dataset observation statistics (states are normalised before embedding, as in the DT paper)
        self.register_buffer("obs_mean", torch.zeros(obs_dim))
        self.register_buffer("obs_std", torch.ones(obs_dim))
        for mod in self.modules():  # GPT-2 initialisation
            if isinstance(mod, (nn.Linear, nn.Embedding)):
                nn.init.normal_(mod.weight, 0.0, 0.02)
                if isinstance(mod, nn.Linear) and mod.bias is not None:
                    nn.init.zeros_(mod.bias)

    def forward(self, rtg, obs, act, ts, mask):
        """rtg [B,K], obs [B,K,d], act [B,K] (−1 → unknown), ts [B,K], mask [B,K] (1 = real step).
        Returns action logits [B,K,A] read at the state tokens."""
        B, K = act.shape
        te = self.embed_t(ts)
        a = torch.where(act < 0, torch.full_like(act, self.A), act)
        s = (obs.flatten(2).float() - self.obs_mean) / self.obs_std
        tok = torch.stack([self.embed_r(rtg.unsqueeze(-1)) + te, self.embed_s(s) + te,
                           self.embed_a(a) + te], dim=2).reshape(B, 3 * K, self.E)
        tok = self.drop(self.ln(tok))
        causal = torch.triu(torch.ones(3 * K, 3 * K, dtype=torch.bool, device=tok.device), 1)
        pad = ~(mask.bool().unsqueeze(-1).expand(B, K, 3).reshape(B, 3 * K))
        h = self.gpt(tok, mask=causal, src_key_padding_mask=pad)
        return self.head(h.reshape(B, K, 3, self.E)[:, :, 1])


def episodes_from_batches(batches: List[SampleBatch]) -> List[Dict[str, np.ndarray]]:
    """Whole episodes (rows grouped by eps_id in recording order; episodes that never reached a
    done are dropped)."""
    rows = collections.OrderedDict()
    for b in batches:
        eps = np.asarray(b[SampleBatch.EPS_ID])
        for e in np.unique(eps):
            sel = eps == e
            d = rows.setdefault(int(e), {k: [] for k in ("obs", "actions", "rewards", "dones")})
            for k in d:
                d[k].append(np.asarray(b[k])[sel])
    out = []
    for d in rows.values():
        ep = {k: np.concatenate(v) for k, v in d.items()}
        if len(ep["dones"]) and ep["dones"][-1] > 0:
            r = ep["rewards"].astype(np.float64)
            ep["rtg"] = np.cumsum(r[::-1])[::-1].astype(np.float32)
            out.append(ep)
    return out


class DT(Algorithm):
    _config_class = DTConfig

    def validate_config(self, c):
        super().validate_config(c)
        if not c.input_ or c.input_ == "sampler":
            raise ValueError("DT is an offline algorithm: set config.offline_data(input_=<recorded episodes>)")
        if c.target_return is None:
            raise ValueError("DT needs config.target_return (the return to condition evaluation on)")

    def _setup_learner(self):
        from ray_memory_management_amd.rllib.offline import JsonReader

        c = self.algo_config
        env = make_env(c.env, c.env_config)
        self.episodes = episodes_from_batches(JsonReader(c.input_).read_all())
        if not self.episodes:
            raise ValueError("no complete episodes in the offline input")
        self.horizon = int(c.horizon or max(len(e["dones"]) for e in self.episodes))
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        self.device = torch.device(dev)
        obs_dim = int(np.prod(env.observation_space.shape))
        if c.seed is not None:
            torch.manual_seed(int(c.seed))
        self.model = DTModel(obs_dim, env.action_space.n, c.max_seq_len, self.horizon, c.embed_dim, c.num_layers,
                             c.num_heads, c.embed_pdrop, c.attn_pdrop).to(self.device)
        allobs = np.concatenate([e["obs"].reshape(len(e["obs"]), -1) for e in self.episodes]).astype(np.float64)
        self.model.obs_mean.copy_(torch.as_tensor(allobs.mean(0), dtype=torch.float32))
        self.model.obs_std.copy_(torch.as_tensor(allobs.std(0) + 1e-6, dtype=torch.float32))
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=c.lr, weight_decay=c.weight_decay)
        self.rng = np.random.default_rng(c.seed)
        lens = np.array([len(e["dones"]) for e in self.episodes], np.float64)
        self._p = lens / lens.sum()  # sample windows uniformly over timesteps
        self.rtg_scale = float(max(1.0, np.abs(np.concatenate([e["rtg"] for e in self.episodes])).max()))
        self._steps = 0

    def _segments(self, n: int):
        c, K = self.algo_config, self.algo_config.max_seq_len
        obs_dim = self.episodes[0]["obs"].shape[1:]
        R = np.zeros((n, K), np.float32)
        S = np.zeros((n, K) + obs_dim, np.float32)
        A = np.full((n, K), -1, np.int64)
        T = np.zeros((n, K), np.int64)
        M = np.zeros((n, K), np.float32)
        for i, e in enumerate(self.rng.choice(len(self.episodes), size=n, p=self._p)):
            ep = self.episodes[e]
            L = len(ep["dones"])
            end = int(self.rng.integers(1, L + 1))
            st = max(0, end - K)
            k = end - st  # left-pad to K
            R[i, K - k:] = ep["rtg"][st:end] / self.rtg_scale
            S[i, K - k:] = ep["obs"][st:end]
            A[i, K - k:] = ep["actions"][st:end]
            T[i, K - k:] = np.minimum(np.arange(st, end), self.horizon)
            M[i, K - k:] = 1.0
        return R, S, A, T, M

    def training_step(self) -> Dict:
        c, dev = self.algo_config, self.device
        R, S, A, T, M = (torch.as_tensor(x, device=dev) for x in self._segments(c.train_batch_size))
        self.model.train()
        if c.lr_warmup_steps:
            for g in self.opt.param_groups:
                g["lr"] = c.lr * min(1.0, (self._steps + 1) / c.lr_warmup_steps)
        logits = self.model(R, S, A, T, M)
        tgt = torch.where(M > 0, A, torch.full_like(A, -100))
        loss = c.loss_coef_actions * nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(),
                                                                 tgt.reshape(-1), ignore_index=-100)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if c.grad_clip:
            nn.utils.clip_grad_norm_(self.model.parameters(), c.grad_clip)
        self.opt.step()
        self._steps += 1
        n = int(M.sum())
        self._counters["num_env_steps_trained"] += n
        self._counters["num_env_steps_sampled"] += n
        return {"loss": float(loss.detach()), "cur_lr": self.opt.param_groups[0]["lr"]}

    @torch.no_grad()
    def evaluate(self, episodes: int = 5, target_return: Optional[float] = None) -> Dict:
        c, dev, K = self.algo_config, self.device, self.algo_config.max_seq_len
        self.model.eval()
        env = make_env(c.env, c.env_config)
        rets = []
        for k in range(episodes):
            o = env.reset(seed=10_000 + k)
            R = [float(target_return if target_return is not None else c.target_return)]
            S, A, ret, t, done = [np.asarray(o, np.float32)], [], 0.0, 0, False
            while not done and t < self.horizon:
                n = len(S)
                st = max(0, n - K)
                k_ = n - st
                r_t = torch.zeros(1, K, device=dev)
                s_t = torch.zeros((1, K) + S[0].shape, device=dev)
                a_t = torch.full((1, K), -1, dtype=torch.int64, device=dev)
                ts = torch.zeros(1, K, dtype=torch.int64, device=dev)
                m = torch.zeros(1, K, device=dev)
                r_t[0, K - k_:] = torch.tensor(R[st:n], device=dev) / self.rtg_scale
                s_t[0, K - k_:] = torch.as_tensor(np.stack(S[st:n]), device=dev)
                if A[st:]:
                    a_t[0, K - k_:K - k_ + len(A[st:])] = torch.tensor(A[st:], device=dev)
                ts[0, K - k_:] = torch.arange(st, n, device=dev).clamp(max=self.horizon)
                m[0, K - k_:] = 1.0
                a = int(self.model(r_t, s_t, a_t, ts, m)[0, -1].argmax())
                o, r, done, _ = env.step(a)
                ret += r
                t += 1
                A.append(a)
                S.append(np.asarray(o, np.float32))
                R.append(R[-1] - r)
            rets.append(ret)
        return {"evaluation": {"episode_reward_mean": float(np.mean(rets)), "episode_reward_max": float(np.max(rets)),
                               "episodes_this_iter": episodes}}

    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        self.model.load_state_dict(w)


DEFAULT_CONFIG = DTConfig().to_dict()
