"""IMPALA: asynchronous sampling + a background learner with V-trace off-policy correction.

Parity: reference rllib/algorithms/impala/impala.py (ImpalaConfig defaults; training_step: keep
`max_sample_requests_in_flight_per_worker` sample requests in flight per rollout worker, turn the
ready ones into train batches of `train_batch_size`, feed the learner thread's queue, broadcast
new weights to the workers that just returned a batch every `broadcast_interval` learner updates,
optional replay of past batches via `replay_proportion` / `replay_buffer_num_slots`),
rllib/execution/learner_thread.py (LearnerThread: inqueue → SGD → outqueue) and
rllib/algorithms/impala/vtrace_torch_policy.py (VTraceLoss: -sum(logp * pg_adv) +
vf_coeff * 0.5 sum((vs - V)^2) - entropy_coeff * sum(H)).

MI355X design: fragments travel worker → shm object store → learner as time-major [T, n] blocks;
the learner concatenates them along the env axis, runs ONE forward over every observation plus the
bootstrap observations, and computes the V-trace targets with the K18 kernel (the whole backward
recursion in one launch instead of T sequential torch ops). The learner runs in a background
thread so HIP work overlaps the driver's sample bookkeeping; torch releases the GIL inside kernels.
"""
from __future__ import annotations

import collections
import copy
import queue
import random
import threading
import time
from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

import ray_memory_management_amd as ray
from ray_memory_management_amd import ops
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_memory_management_amd.rllib.utils.schedules import make_schedule


class ImpalaConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or Impala)
        self.vtrace = True
        self.vtrace_clip_rho_threshold = 1.0
        self.vtrace_clip_pg_rho_threshold = 1.0
        self.num_sgd_iter = 1
        self.minibatch_buffer_size = 1
        self.replay_proportion = 0.0
        self.replay_buffer_num_slots = 0
        self.learner_queue_size = 16
        self.learner_queue_timeout = 300
        self.max_sample_requests_in_flight_per_worker = 2
        self.broadcast_interval = 1
        self.grad_clip = 40.0
        self.opt_type = "adam"
        self.lr_schedule = None
        self.decay = 0.99
        self.momentum = 0.0
        self.epsilon = 0.1
        self.vf_loss_coeff = 0.5
        self.entropy_coeff = 0.01
        self.entropy_coeff_schedule = None
        self.rollout_fragment_length = 50
        self.train_batch_size = 500
        self.num_workers = 2
        self.lr = 0.0005
        self.min_time_s_per_iteration = 10
        self.learner_thread = True  # False: update inline in training_step (deterministic; tests)

    def training(self, **kwargs) -> "ImpalaConfig":
        return super().training(**kwargs)


class VTraceLearner:
    """Model + optimizer on the learner device; `update(fragments)` = one SGD step on a train
    batch assembled from time-major fragments. Thread-safe w.r.t. get_weights."""

    def __init__(self, model: nn.Module, cfg: Dict, device="cpu"):
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.cfg = cfg
        params = list(self.model.parameters())
        if cfg.get("opt_type", "adam") == "rmsprop":
            self.opt = torch.optim.RMSprop(params, lr=cfg["lr"], alpha=cfg.get("decay", 0.99),
                                           momentum=cfg.get("momentum", 0.0), eps=cfg.get("epsilon", 0.1))
        else:
            self.opt = torch.optim.Adam(params, lr=cfg["lr"])
        self.lr_sched = make_schedule(cfg.get("lr_schedule"), cfg["lr"])
        self.ent_sched = make_schedule(cfg.get("entropy_coeff_schedule"), cfg.get("entropy_coeff", 0.01))
        self.lock = threading.Lock()
        self.version = 0
        self.num_steps_trained = 0

    # ---- batch assembly: [T, n_i] fragments -> [T, B] device tensors (B = sum n_i)
    def _assemble(self, frags: List[Dict]):
        T = int(frags[0]["T"])
        if any(int(f["T"]) != T for f in frags):
            raise ValueError("all fragments of a train batch need the same rollout_fragment_length")
        dev = self.device
        nb = self.device.type == "cuda"

        def cat(k, axis=1):  # fragments fetched from the store are read-only views: one copy here
            a = np.concatenate([np.asarray(f[k]) for f in frags], axis=axis) if len(frags) > 1 else \
                np.array(frags[0][k], copy=True)
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=nb)

        keys = ["obs", "actions", "action_logp", "action_dist_inputs", "rewards", "dones"]
        b = {k: cat(k) for k in keys}
        if "state_in" in frags[0]:  # recurrent unrolls (RolloutWorker.sample_time_major)
            for k in ("prev_actions", "prev_rewards", "resets"):
                b[k] = cat(k)
            for k in ("last_prev_actions", "last_prev_rewards"):
                b[k] = cat(k, axis=0)
            b["state_in"] = [torch.from_numpy(np.ascontiguousarray(np.concatenate(
                [np.asarray(f["state_in"][i]) for f in frags], axis=0))).to(dev).float()
                for i in range(len(frags[0]["state_in"]))]
        return T, b, cat("last_obs", axis=0)

    def _forward(self, model, b, last_obs):
        obs = b["obs"]
        T, B = obs.shape[:2]
        if getattr(model, "is_recurrent", False):
            # the unroll re-run from its start state ([B, T] sequences, resets at episode starts), then
            # one step on the bootstrap observation from the final state
            bt = lambda x: x.transpose(0, 1)  # noqa: E731
            logits, values, st = model.seq(bt(obs), b["state_in"], bt(b["resets"]), bt(b["prev_actions"]),
                                           bt(b["prev_rewards"]))
            st = model.reset_state(st, b["dones"][-1] > 0)
            _, boot, _ = model.step(last_obs, st, b["last_prev_actions"], b["last_prev_rewards"])
            return bt(logits.float()), bt(values.float()), boot.float()
        x = torch.cat([obs.reshape((T * B,) + tuple(obs.shape[2:])), last_obs.to(obs.dtype)], 0)
        logits, values = model(x)
        logits, values = logits.float(), values.float()
        return logits[:T * B].view(T, B, -1), values[:T * B].view(T, B), values[T * B:]

    def loss(self, T, b, last_obs):
        c = self.cfg
        logits, values, boot = self._forward(self.model, b, last_obs)
        lsm = torch.log_softmax(logits, -1)
        tlogp = lsm.gather(2, b["actions"].unsqueeze(-1)).squeeze(-1)
        with torch.no_grad():
            if c.get("vtrace", True):
                vs, pg = ops.vtrace(b["action_logp"], tlogp, b["rewards"], values, b["dones"], boot, c["gamma"],
                                    c["vtrace_clip_rho_threshold"], c["vtrace_clip_pg_rho_threshold"])
            else:  # on-policy n-step returns (rho = 1)
                vs, pg = ops.vtrace(tlogp, tlogp, b["rewards"], values, b["dones"], boot, c["gamma"], None, None)
        ent = -(lsm.exp() * lsm).sum(-1)
        pi_loss = -(tlogp * pg).sum()
        vf_loss = 0.5 * ((vs - values) ** 2).sum()
        ent_coeff = self.ent_sched(self.num_steps_trained)
        total = pi_loss + c["vf_loss_coeff"] * vf_loss - ent_coeff * ent.sum()
        n = float(T * values.shape[1])
        return total, {"policy_loss": float(pi_loss.detach()) / n, "vf_loss": float(vf_loss.detach()) / n,
                       "entropy": float(ent.detach().mean()), "entropy_coeff": float(ent_coeff),
                       "mean_rho": float(torch.exp(tlogp.detach() - b["action_logp"]).mean()),
                       "vs_mean": float(vs.mean())}

    def update(self, frags: List[Dict]) -> Dict:
        T, b, last_obs = self._assemble(frags)
        stats = {}
        with self.lock:
            for g in self.opt.param_groups:
                g["lr"] = self.lr_sched(self.num_steps_trained)
            for _ in range(int(self.cfg.get("num_sgd_iter", 1))):
                total, stats = self.loss(T, b, last_obs)
                self.opt.zero_grad(set_to_none=True)
                total.backward()
                gn = nn.utils.clip_grad_norm_(self.model.parameters(), self.cfg["grad_clip"]) \
                    if self.cfg.get("grad_clip") else None
                self.opt.step()
                if gn is not None:
                    stats["grad_gnorm"] = float(gn)
            rows = T * b["rewards"].shape[1]
            self.num_steps_trained += rows
            self.after_update(stats, rows)
            self.version += 1
        stats["cur_lr"] = self.opt.param_groups[0]["lr"]
        return stats

    def after_update(self, stats: Dict, rows: int):
        pass

    def get_weights(self):
        with self.lock:
            return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}

    def set_weights(self, w):
        with self.lock:
            self.model.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})


class LearnerThread(threading.Thread):
    """Background SGD over train batches from `inqueue` (reference rllib/execution/learner_thread.py)."""

    def __init__(self, learner: VTraceLearner, queue_size: int, timeout: float):
        super().__init__(daemon=True, name="impala-learner")
        self.learner = learner
        self.inqueue: "queue.Queue" = queue.Queue(maxsize=queue_size)
        self.outqueue: "queue.Queue" = queue.Queue()
        self.timeout = timeout
        self.stopped = False
        self.error = None
        self.busy = False
        self.queue_sizes = collections.deque(maxlen=100)

    def run(self):
        while not self.stopped:
            try:
                frags = self.inqueue.get(timeout=0.1)
            except queue.Empty:
                continue
            self.busy = True
            try:
                self.queue_sizes.append(self.inqueue.qsize())
                stats = self.learner.update(frags)
                self.outqueue.put((sum(int(f["T"]) * int(f["n"]) for f in frags), stats))
            except Exception as e:  # surfaced by the driver's next training_step
                self.error = e
                self.stopped = True
            finally:
                self.busy = False


class Impala(Algorithm):
    _config_class = ImpalaConfig
    _learner_class = VTraceLearner
    _supports_sequence_models = True

    def validate_config(self, c):
        super().validate_config(c)
        if c.train_batch_size < c.rollout_fragment_length:
            raise ValueError("train_batch_size must be >= rollout_fragment_length")
        if c.max_sample_requests_in_flight_per_worker < 1:
            raise ValueError("max_sample_requests_in_flight_per_worker must be >= 1")

    def _learner_cfg(self) -> Dict:
        c = self.algo_config
        keys = ("lr", "gamma", "grad_clip", "opt_type", "decay", "momentum", "epsilon", "vf_loss_coeff", "entropy_coeff",
                "entropy_coeff_schedule", "lr_schedule", "vtrace", "vtrace_clip_rho_threshold",
                "vtrace_clip_pg_rho_threshold", "num_sgd_iter")
        return {k: getattr(c, k) for k in keys}

    def _setup_learner(self):
        c = self.algo_config
        dev = "cuda" if c.num_gpus and torch.cuda.is_available() else "cpu"
        local = self.workers.local_worker()
        self.learner = self._learner_class(copy.deepcopy(local.policy.model), self._learner_cfg(), device=dev)
        self._thread = None
        if c.learner_thread:
            self._thread = LearnerThread(self.learner, c.learner_queue_size, c.learner_queue_timeout)
            self._thread.start()
        self._in_flight: Dict = {}  # ObjectRef -> worker index
        self._pending: List[Dict] = []  # fragments not yet in a train batch
        self._pending_rows = 0
        self._replay = collections.deque(maxlen=max(1, int(c.replay_buffer_num_slots or 1)))
        self._worker_version = [0] * len(self.workers.remote_workers())
        self._updates_since_bcast = [0] * len(self.workers.remote_workers())
        self._weights_ref, self._weights_ref_version = None, -1
        self._learner_stats: Dict = {}
        self._rng = random.Random(c.seed)

    # ---- sampling
    def _kick(self, i):
        w = self.workers.remote_workers()[i]
        self._in_flight[w.sample_time_major.remote()] = i

    def _current_weights_ref(self):
        v = self.learner.version
        if self._weights_ref_version != v:
            self._weights_ref = ray.put(self.learner.get_weights())
            self._weights_ref_version = v
            self._counters["num_weight_broadcasts"] += 1
        return self._weights_ref

    def _gather_ready(self) -> List[Dict]:
        c = self.algo_config
        remotes = self.workers.remote_workers()
        if not remotes:
            return [self.workers.local_worker().sample_time_major()]
        for i in range(len(remotes)):
            have = sum(1 for j in self._in_flight.values() if j == i)
            for _ in range(c.max_sample_requests_in_flight_per_worker - have):
                self._kick(i)
        ready, rest = ray.wait(list(self._in_flight), num_returns=1, timeout=None)
        if rest:
            more, _ = ray.wait(rest, num_returns=len(rest), timeout=0)
            ready = list(ready) + list(more)
        frags = ray.get(ready)
        for r in ready:
            i = self._in_flight.pop(r)
            # weights to the worker that just returned, every `broadcast_interval` learner updates
            if self.learner.version - self._worker_version[i] >= c.broadcast_interval:
                remotes[i].set_weights.remote(self._current_weights_ref())
                self._worker_version[i] = self.learner.version
            self._kick(i)
        return frags

    def _train_batches(self, frags: List[Dict]) -> List[List[Dict]]:
        c = self.algo_config
        out = []
        for f in frags:
            self._pending.append(f)
            self._pending_rows += int(f["T"]) * int(f["n"])
            if self._pending_rows >= c.train_batch_size:
                out.append(self._pending)
                self._pending, self._pending_rows = [], 0
        if c.replay_proportion and c.replay_buffer_num_slots:
            mixed = []
            for b in out:
                mixed.append(b)
                self._replay.append(b)
                k = np.random.default_rng(self._rng.getrandbits(32)).poisson(c.replay_proportion)
                for _ in range(k):
                    mixed.append(self._rng.choice(list(self._replay)))
                    self._counters["num_replayed_batches"] += 1
            out = mixed
        return out

    def training_step(self) -> Dict:
        c = self.algo_config
        if self._thread is not None and self._thread.error is not None:
            raise RuntimeError("learner thread failed") from self._thread.error
        frags = self._gather_ready()
        n = sum(int(f["T"]) * int(f["n"]) for f in frags)
        self._counters["num_env_steps_sampled"] += n
        self._counters["num_agent_steps_sampled"] += n
        self._timesteps_total += n
        for batch in self._train_batches(frags):
            if self._thread is None:
                self._on_learned(sum(int(f["T"]) * int(f["n"]) for f in batch), self.learner.update(batch))
            else:
                self._thread.inqueue.put(batch, timeout=c.learner_queue_timeout)
        if self._thread is not None:
            while True:
                try:
                    self._on_learned(*self._thread.outqueue.get_nowait())
                except queue.Empty:
                    break
        if not self.workers.remote_workers() or self.learner.version != getattr(self, "_local_version", -1):
            self.workers.local_worker().set_weights(self.learner.get_weights())
            self._local_version = self.learner.version
        out = dict(self._learner_stats)
        if self._thread is not None:
            qs = self._thread.queue_sizes
            out["learner_queue"] = {"size_mean": float(np.mean(qs)) if qs else 0.0,
                                    "size_now": self._thread.inqueue.qsize()}
        return out

    def _on_learned(self, rows: int, stats: Dict):
        self._counters["num_env_steps_trained"] += rows
        self._counters["num_agent_steps_trained"] += rows
        self._counters["num_training_step_calls_learner"] += 1
        self._learner_stats = stats

    def wait_for_learner(self, timeout: float = 60.0):
        """Block until every queued train batch has been learned (tests / checkpoints)."""
        if self._thread is None:
            return
        t0 = time.time()
        while (not self._thread.inqueue.empty() or self._thread.busy) and time.time() - t0 < timeout \
                and self._thread.error is None:
            time.sleep(0.01)
        while True:
            try:
                self._on_learned(*self._thread.outqueue.get_nowait())
            except queue.Empty:
                break

    def get_weights(self):
        return self.learner.get_weights()

    def set_weights(self, weights):
        self.learner.set_weights(weights)
        self.workers.local_worker().set_weights(weights)
        self.workers.sync_weights(weights)

    def cleanup(self):
        if getattr(self, "_thread", None) is not None:
            self._thread.stopped = True
            self._thread.join(timeout=10)
        super().cleanup()


Impala.__name__ = "Impala"
IMPALA = Impala
DEFAULT_CONFIG = ImpalaConfig().to_dict()
