"""Execution-plan operators (the iterator-based training-loop API).

Parity: reference rllib/execution/{rollout_ops, train_ops, concurrency_ops, metric_ops,
replay_ops, learner_thread, multi_gpu_learner_thread, minibatch_buffer, buffers/}.py. An execution
plan composes these on ``util.iter.LocalIterator``::

    rollouts = ParallelRollouts(workers, mode="bulk_sync")
    train_op = rollouts.combine(ConcatBatches(min_batch_size=4000)) \\
                       .for_each(StandardizeFields(["advantages"])) \\
                       .for_each(TrainOneStep(workers, num_sgd_iter=10, sgd_minibatch_size=128))
    for result in StandardMetricsReporting(train_op, workers, config):
        ...

Counters / timers shared by the operators of one plan live in a per-process MetricsContext
(``_get_shared_metrics()``), as in the reference. Learning goes through the policy's
``learn_on_batch`` / ``compute_gradients`` / ``apply_gradients`` (policy templates); the built-in
algorithms' fused GPU learners keep their own ``training_step``.
"""
from __future__ import annotations

import collections
import queue
import random
import threading
import time
from typing import Any, Callable, Dict, List, Optional

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples
from ray_memory_management_amd.util.iter import LocalIterator

STEPS_SAMPLED_COUNTER = "num_steps_sampled"
AGENT_STEPS_SAMPLED_COUNTER = "num_agent_steps_sampled"
STEPS_TRAINED_COUNTER = "num_steps_trained"
STEPS_TRAINED_THIS_ITER_COUNTER = "num_steps_trained_this_iter"
AGENT_STEPS_TRAINED_COUNTER = "num_agent_steps_trained"
LAST_TARGET_UPDATE_TS = "last_target_update_ts"
NUM_TARGET_UPDATES = "num_target_updates"
SAMPLE_TIMER = "sample"
LEARN_ON_BATCH_TIMER = "learn"
GRAD_WAIT_TIMER = "grad_wait"
APPLY_GRADS_TIMER = "apply_grad"
WORKER_UPDATE_TIMER = "update"
LOAD_BATCH_TIMER = "load"


class TimerStat:
    """Mean wall time of a repeated section (reference rllib/utils/timer.py)."""

    def __init__(self, window: int = 100):
        self._samples = collections.deque(maxlen=window)
        self._start = None
        self.count = 0
        self._units = collections.deque(maxlen=window)

    def __enter__(self):
        self._start = time.perf_counter()
        return self

    def __exit__(self, *a):
        self._samples.append(time.perf_counter() - self._start)
        self.count += 1

    def push_units_processed(self, n):
        self._units.append(n)

    @property
    def mean(self) -> float:
        return float(np.mean(self._samples)) if self._samples else 0.0

    @property
    def mean_throughput(self) -> float:
        t = float(np.sum(self._samples)) if self._samples else 0.0
        return float(np.sum(self._units)) / t if t > 0 and self._units else 0.0


class MetricsContext:
    """Counters / timers / info shared by the operators of an execution plan."""

    def __init__(self):
        self.counters: Dict[str, int] = collections.defaultdict(int)
        self.timers: Dict[str, TimerStat] = collections.defaultdict(TimerStat)
        self.info: Dict[str, Any] = {}
        self.current_actor = None

    def save(self):
        return dict(self.counters), dict(self.info)

    def restore(self, state):
        self.counters.clear()
        self.counters.update(state[0])
        self.info = dict(state[1])


_METRICS = threading.local()


def _get_shared_metrics() -> MetricsContext:
    m = getattr(_METRICS, "ctx", None)
    if m is None:
        m = _METRICS.ctx = MetricsContext()
    return m


def reset_shared_metrics() -> MetricsContext:
    _METRICS.ctx = MetricsContext()
    return _METRICS.ctx


def _count(batch) -> int:
    return int(batch.count) if hasattr(batch, "count") else len(batch)


def _agent_steps(batch) -> int:
    if isinstance(batch, MultiAgentBatch):
        return sum(_count(b) for b in batch.policy_batches.values())
    return _count(batch)


# ============================================================================ rollout ops
def synchronous_parallel_sample(worker_set=None, *, max_agent_steps: Optional[int] = None,
                                max_env_steps: Optional[int] = None, concat: bool = True):
    """reference rollout_ops.py:36: sample from every remote worker (or the local one) until the
    requested steps are collected."""
    steps = max_env_steps or max_agent_steps or 0
    out = worker_set.synchronous_parallel_sample(max(steps, 1), concat=False)
    if not concat:
        return out
    return concat_samples(out) if not isinstance(out[0], MultiAgentBatch) else MultiAgentBatch.concat_samples(out)


def ParallelRollouts(workers, *, mode: str = "bulk_sync", num_async: int = 1) -> LocalIterator:
    """Iterator of experience batches from the workers. ``bulk_sync``: one concatenated batch per
    round of all workers; ``async``: each worker's batch as it arrives (``num_async`` requests in
    flight per worker); ``raw``: a list of the round's per-worker batches."""
    metrics = reset_shared_metrics()
    remote = workers.remote_workers()

    def report(batch):
        metrics.counters[STEPS_SAMPLED_COUNTER] += _count(batch)
        metrics.counters[AGENT_STEPS_SAMPLED_COUNTER] += _agent_steps(batch)
        return batch

    if not remote:
        def local_gen():
            while True:
                with metrics.timers[SAMPLE_TIMER]:
                    b = workers.local_worker().sample()
                yield report(b)
        return LocalIterator(local_gen, "ParallelRollouts[local]")
    if mode in ("bulk_sync", "raw"):
        def bulk_gen():
            while True:
                with metrics.timers[SAMPLE_TIMER]:
                    bs = ray.get([w.sample.remote() for w in remote])
                if mode == "raw":
                    for b in bs:
                        report(b)
                    yield bs
                else:
                    yield report(concat_samples(bs) if not isinstance(bs[0], MultiAgentBatch)
                                 else MultiAgentBatch.concat_samples(bs))
        return LocalIterator(bulk_gen, f"ParallelRollouts[{mode}]")
    if mode == "async":
        def async_gen():
            pending = {}
            for w in remote:
                for _ in range(num_async):
                    pending[w.sample.remote()] = w
            while True:
                ready, _ = ray.wait(list(pending), num_returns=1)
                r = ready[0]
                w = pending.pop(r)
                metrics.current_actor = w
                b = ray.get(r)
                pending[w.sample.remote()] = w
                yield report(b)
        return LocalIterator(async_gen, "ParallelRollouts[async]")
    raise ValueError(f"mode must be one of bulk_sync / async / raw, got {mode!r}")


class ConcatBatches:
    """Accumulate batches until ``min_batch_size`` steps (use with ``.combine()``)."""

    def __init__(self, min_batch_size: int, count_steps_by: str = "env_steps"):
        self.min_batch_size = int(min_batch_size)
        self.count_steps_by = count_steps_by
        self.buffer: List = []
        self.count = 0
        self.last_batch_time = time.perf_counter()

    def __call__(self, batch) -> List:
        self.buffer.append(batch)
        self.count += _count(batch) if self.count_steps_by == "env_steps" else _agent_steps(batch)
        if self.count < self.min_batch_size:
            return []
        out = (concat_samples(self.buffer) if not isinstance(self.buffer[0], MultiAgentBatch)
               else MultiAgentBatch.concat_samples(self.buffer))
        _get_shared_metrics().timers["sample_throughput"].push_units_processed(self.count)
        self.buffer, self.count = [], 0
        self.last_batch_time = time.perf_counter()
        return [out]


class SelectExperiences:
    """Keep only the given policies' batches of a MultiAgentBatch."""

    def __init__(self, policy_ids: Optional[List[str]] = None, local_worker=None):
        self.policy_ids = set(policy_ids or [])

    def __call__(self, samples):
        if not isinstance(samples, MultiAgentBatch):
            return samples
        return MultiAgentBatch({k: v for k, v in samples.policy_batches.items() if k in self.policy_ids},
                               samples.count)


class StandardizeFields:
    """Zero-mean / unit-std the given columns (e.g. advantages) of every (policy) batch."""

    def __init__(self, fields: List[str]):
        self.fields = list(fields)

    def _std(self, b):
        for f in self.fields:
            if f in b:
                v = np.asarray(b[f], dtype=np.float32)
                b[f] = (v - v.mean()) / max(float(v.std()), 1e-4)
        return b

    def __call__(self, samples):
        if isinstance(samples, MultiAgentBatch):
            for b in samples.policy_batches.values():
                self._std(b)
            return samples
        return self._std(samples)


# ============================================================================ train ops
def _minibatches(batch: SampleBatch, size: int, num_iters: int):
    n = _count(batch)
    if not size or size >= n:
        for _ in range(num_iters):
            yield batch
        return
    for _ in range(num_iters):
        perm = np.random.permutation(n)
        for s in range(0, n - size + 1, size):
            idx = perm[s:s + size]
            yield SampleBatch({k: (np.asarray(v)[idx] if np.ndim(v) and len(v) == n else v) for k, v in batch.items()})


def _learn(worker, batch, num_sgd_iter: int, sgd_minibatch_size: int, policies=None) -> Dict:
    info: Dict = {}
    if isinstance(batch, MultiAgentBatch):
        for pid, b in batch.policy_batches.items():
            if policies and pid not in policies:
                continue
            pol = worker.get_policy(pid)
            for mb in _minibatches(b, sgd_minibatch_size, num_sgd_iter):
                info[pid] = pol.learn_on_batch(mb)
        return info
    pol = worker.get_policy()
    for mb in _minibatches(batch, sgd_minibatch_size, num_sgd_iter):
        info[DEFAULT_POLICY_ID] = pol.learn_on_batch(mb)
    return info


def train_one_step(algorithm, train_batch, policies_to_train=None) -> Dict:
    """reference train_ops.py: learn on the local worker (num_sgd_iter x minibatches)."""
    cfg = getattr(algorithm, "config", {}) or {}
    workers = algorithm.workers
    metrics = _get_shared_metrics()
    with metrics.timers[LEARN_ON_BATCH_TIMER]:
        info = _learn(workers.local_worker(), train_batch, int(cfg.get("num_sgd_iter", 1) or 1),
                      int(cfg.get("sgd_minibatch_size", 0) or 0), policies_to_train)
    metrics.counters[STEPS_TRAINED_COUNTER] += _count(train_batch)
    metrics.counters[AGENT_STEPS_TRAINED_COUNTER] += _agent_steps(train_batch)
    return info


class TrainOneStep:
    """Learn on the local worker's policies, then broadcast the weights to the remote workers."""

    def __init__(self, workers, policies: Optional[List[str]] = None, num_sgd_iter: int = 1,
                 sgd_minibatch_size: int = 0):
        self.workers, self.policies = workers, list(policies or [])
        self.num_sgd_iter, self.sgd_minibatch_size = int(num_sgd_iter), int(sgd_minibatch_size)

    def __call__(self, batch):
        metrics = _get_shared_metrics()
        with metrics.timers[LEARN_ON_BATCH_TIMER]:
            info = _learn(self.workers.local_worker(), batch, self.num_sgd_iter, self.sgd_minibatch_size,
                          self.policies)
        metrics.counters[STEPS_TRAINED_COUNTER] += _count(batch)
        metrics.counters[STEPS_TRAINED_THIS_ITER_COUNTER] = _count(batch)
        metrics.counters[AGENT_STEPS_TRAINED_COUNTER] += _agent_steps(batch)
        metrics.info["learner"] = info
        if self.workers.remote_workers():
            with metrics.timers[WORKER_UPDATE_TIMER]:
                self.workers.sync_weights()
        return batch, info


class MultiGPUTrainOneStep(TrainOneStep):
    """reference train_ops.MultiGPUTrainOneStep. The local worker's policy learns on its own
    device; multi-GPU data parallelism of the built-in algorithms is the learner actors'
    (execution/learner_group.py), not this operator's."""

    def __init__(self, *, workers, sgd_minibatch_size: int = 0, num_sgd_iter: int = 1, num_gpus: int = 0,
                 _fake_gpus: bool = False, shuffle_sequences: bool = True, policies=None, **kw):
        super().__init__(workers, policies, num_sgd_iter, sgd_minibatch_size)


class ComputeGradients:
    """batch → (gradients, count) on the worker the item came from (the local one by default)."""

    def __init__(self, workers):
        self.workers = workers

    def __call__(self, samples):
        metrics = _get_shared_metrics()
        with metrics.timers["compute_grads"]:
            grads, info = self.workers.local_worker().compute_gradients(samples)
        metrics.info["learner"] = info.get("learner_stats", info)
        return grads, _count(samples)


class ApplyGradients:
    """(gradients, count) → apply on the local worker; broadcast weights (all workers, or only to
    the worker that produced the gradients when ``update_all=False``)."""

    def __init__(self, workers, policies: Optional[List[str]] = None, update_all: bool = True):
        self.workers, self.policies, self.update_all = workers, list(policies or []), update_all

    def __call__(self, item):
        grads, count = item
        metrics = _get_shared_metrics()
        metrics.counters[STEPS_TRAINED_COUNTER] += count
        with metrics.timers[APPLY_GRADS_TIMER]:
            self.workers.local_worker().apply_gradients(grads)
        if self.update_all:
            if self.workers.remote_workers():
                with metrics.timers[WORKER_UPDATE_TIMER]:
                    self.workers.sync_weights()
        elif metrics.current_actor is not None:
            metrics.current_actor.set_weights.remote(self.workers.local_worker().get_weights())
        return item


class AverageGradients:
    """list of (gradients, count) → (average gradients, total count)."""

    def __call__(self, gradients):
        acc, total = None, 0
        for grads, count in gradients:
            acc = [np.asarray(g, dtype=np.float64) for g in grads] if acc is None else \
                [a + np.asarray(g) for a, g in zip(acc, grads)]
            total += count
        n = max(len(gradients), 1)
        return [(a / n).astype(np.float32) for a in acc], total


def AsyncGradients(workers) -> LocalIterator:
    """Gradients computed on the remote workers from their own samples, as they arrive."""
    metrics = reset_shared_metrics()

    def _grad(w):
        b = w.sample()
        g, info = w.compute_gradients(b)
        return g, info, _count(b)

    def gen():
        remote = workers.remote_workers()
        pending = {w.apply.remote(_grad): w for w in remote}
        while True:
            ready, _ = ray.wait(list(pending), num_returns=1)
            w = pending.pop(ready[0])
            with metrics.timers[GRAD_WAIT_TIMER]:
                grads, info, count = ray.get(ready[0])
            metrics.current_actor = w
            metrics.counters[STEPS_SAMPLED_COUNTER] += count
            metrics.info["learner"] = info.get("learner_stats", info)
            pending[w.apply.remote(_grad)] = w
            yield grads, count

    return LocalIterator(gen, "AsyncGradients")


class UpdateTargetNetwork:
    """Call ``policy.update_target()`` every ``target_update_freq`` trained steps."""

    def __init__(self, workers, target_update_freq: int, by_steps_trained: bool = False, policies=None):
        self.workers, self.freq, self.by_trained = workers, int(target_update_freq), by_steps_trained
        self.policies = list(policies or [])

    def __call__(self, item):
        metrics = _get_shared_metrics()
        cur = metrics.counters[STEPS_TRAINED_COUNTER if self.by_trained else STEPS_SAMPLED_COUNTER]
        if cur - metrics.counters[LAST_TARGET_UPDATE_TS] >= self.freq:
            self.workers.local_worker().foreach_policy(
                lambda p, pid: p.update_target() if hasattr(p, "update_target") and
                (not self.policies or pid in self.policies) else None)
            metrics.counters[NUM_TARGET_UPDATES] += 1
            metrics.counters[LAST_TARGET_UPDATE_TS] = cur
        return item


# ============================================================================ concurrency ops
def Concurrently(ops: List[LocalIterator], *, mode: str = "round_robin", output_indexes: Optional[List[int]] = None,
                 round_robin_weights: Optional[List] = None) -> LocalIterator:
    """Run several iterators interleaved; yield only the outputs of ``output_indexes``."""
    if mode not in ("round_robin", "async"):
        raise ValueError(f"mode must be round_robin or async, got {mode!r}")
    if round_robin_weights is not None and len(round_robin_weights) != len(ops):
        raise ValueError("round_robin_weights must have one entry per op")
    tagged = [op.for_each(lambda x, i=i: (i, x)) for i, op in enumerate(ops)]
    u = tagged[0].union(*tagged[1:], round_robin_weights=round_robin_weights)
    keep = set(range(len(ops)) if output_indexes is None else output_indexes)
    return u.filter(lambda ix: ix[0] in keep).for_each(lambda ix: ix[1])


class Enqueue:
    """Put each item into a (thread) queue; the item passes through."""

    def __init__(self, output_queue: "queue.Queue"):
        self.queue = output_queue

    def __call__(self, x):
        try:
            self.queue.put(x, timeout=0.001)
        except queue.Full:
            return None
        return x


def Dequeue(input_queue: "queue.Queue", check: Callable[[], bool] = lambda: True) -> LocalIterator:
    def gen():
        while check():
            try:
                yield input_queue.get(timeout=0.001)
            except queue.Empty:
                yield None  # lets a round-robin union make progress
    return LocalIterator(gen, "Dequeue").filter(lambda x: x is not None)


class OncePerTimeInterval:
    def __init__(self, delay: Optional[float] = None):
        self.delay = delay or 0.0
        self.last_returned = 0.0

    def __call__(self, item) -> bool:
        if self.delay <= 0:
            return True
        now = time.time()
        if now - self.last_returned > self.delay:
            self.last_returned = now
            return True
        return False


class OncePerTimestepsElapsed:
    def __init__(self, delay_steps: int, by_steps_trained: bool = False):
        self.delay_steps, self.by_trained = int(delay_steps), by_steps_trained
        self.last_called = 0

    def __call__(self, item) -> bool:
        if self.delay_steps <= 0:
            return True
        m = _get_shared_metrics()
        now = m.counters[STEPS_TRAINED_COUNTER if self.by_trained else STEPS_SAMPLED_COUNTER]
        if now - self.last_called >= self.delay_steps:
            self.last_called = now
            return True
        return False


# ============================================================================ metric ops
class CollectMetrics:
    """Turn the pipeline's items into training results (episode stats from the workers,
    counters, timers, learner info)."""

    def __init__(self, workers, min_history: int = 100, timeout_seconds: int = 180, keep_per_episode_custom_metrics=False,
                 selected_workers=None, by_steps_trained: bool = False):
        self.workers, self.min_history = workers, int(min_history)
        self.episode_history: collections.deque = collections.deque(maxlen=max(self.min_history, 1))
        self.selected_workers = selected_workers

    def __call__(self, _) -> Dict:
        from ray_memory_management_amd.rllib.evaluation.metrics import summarize_episodes

        eps = self.workers.collect_metrics()
        self.episode_history.extend(eps)
        use = eps if len(eps) >= self.min_history else list(self.episode_history)
        res = summarize_episodes(use)
        m = _get_shared_metrics()
        res["timesteps_total"] = m.counters[STEPS_SAMPLED_COUNTER]
        res["agent_timesteps_total"] = m.counters[AGENT_STEPS_SAMPLED_COUNTER]
        res["timers"] = {f"{k}_time_ms": round(t.mean * 1e3, 3) for k, t in m.timers.items()}
        res["info"] = {**{k: v for k, v in m.info.items()}, **dict(m.counters)}
        res["counters"] = dict(m.counters)
        return res


def StandardMetricsReporting(train_op: LocalIterator, workers, config: Dict, selected_workers=None,
                             by_steps_trained: bool = False) -> LocalIterator:
    """Report at most once per ``min_time_s_per_iteration`` and ``timesteps_per_iteration``."""
    cfg = config or {}
    return (train_op
            .filter(OncePerTimestepsElapsed(int(cfg.get("min_sample_timesteps_per_iteration",
                                                        cfg.get("timesteps_per_iteration", 0)) or 0),
                                            by_steps_trained=by_steps_trained))
            .filter(OncePerTimeInterval(float(cfg.get("min_time_s_per_iteration", 0) or 0)))
            .for_each(CollectMetrics(workers, min_history=int(cfg.get("metrics_num_episodes_for_smoothing", 100)),
                                     timeout_seconds=int(cfg.get("metrics_episode_collection_timeout_s", 180)))))


# ============================================================================ replay ops
class SimpleReplayBuffer:
    """Ring of whole batches, replayed uniformly (reference execution/buffers/simple_replay_buffer)."""

    def __init__(self, num_slots: int, replay_proportion: Optional[float] = None):
        self.num_slots, self.replay_proportion = int(num_slots), replay_proportion
        self.replay_batches: List = []
        self.replay_index = 0

    def add_batch(self, sample_batch) -> None:
        if self.num_slots <= 0:
            return
        if len(self.replay_batches) < self.num_slots:
            self.replay_batches.append(sample_batch)
        else:
            self.replay_batches[self.replay_index] = sample_batch
            self.replay_index = (self.replay_index + 1) % self.num_slots

    def replay(self):
        return random.choice(self.replay_batches) if self.replay_batches else None

    def __len__(self):
        return len(self.replay_batches)


class StoreToReplayBuffer:
    def __init__(self, *, local_buffer=None, actors=None):
        if (local_buffer is None) == (actors is None):
            raise ValueError("exactly one of local_buffer / actors")
        self.local_buffer, self.actors = local_buffer, actors

    def __call__(self, batch):
        if self.local_buffer is not None:
            (self.local_buffer.add_batch if hasattr(self.local_buffer, "add_batch") else self.local_buffer.add)(batch)
        else:
            random.choice(self.actors).add.remote(batch)
        return batch


def Replay(*, local_buffer=None, num_items_to_replay: int = 1, actors=None, num_async: int = 4) -> LocalIterator:
    """Iterator of replayed batches from a local buffer (or replay actors)."""
    if (local_buffer is None) == (actors is None):
        raise ValueError("exactly one of local_buffer / actors")

    def gen():
        while True:
            if local_buffer is not None:
                if hasattr(local_buffer, "replay"):
                    item = local_buffer.replay()
                else:
                    item = local_buffer.sample(num_items_to_replay)
            else:
                item = ray.get(random.choice(actors).sample.remote(num_items_to_replay))
            yield item if item is not None else None

    return LocalIterator(gen, "Replay").filter(lambda x: x is not None)


class MixInReplay:
    """Each new batch comes out together with ``replay_ratio``-proportioned replayed batches."""

    def __init__(self, num_slots: int, replay_proportion: float):
        if replay_proportion > 0 and num_slots == 0:
            raise ValueError("replay_proportion > 0 needs num_slots > 0")
        self.replay_buffer = SimpleReplayBuffer(num_slots)
        self.replay_proportion = float(replay_proportion)

    def __call__(self, sample_batch) -> List:
        self.replay_buffer.add_batch(sample_batch)
        out = [sample_batch]
        f = self.replay_proportion
        while random.random() < f:
            f -= 1
            r = self.replay_buffer.replay()
            if r is not None:
                out.append(r)
        return out


# ============================================================================ learner threads
class MinibatchBuffer:
    """Re-serve each batch of an input queue ``num_passes`` times (reference minibatch_buffer.py)."""

    def __init__(self, inqueue: "queue.Queue", size: int, timeout: float, num_passes: int, init_num_passes: int = 1):
        self.inqueue, self.size, self.timeout = inqueue, int(size), float(timeout)
        self.max_ttl, self.cur_max_ttl = int(num_passes), int(init_num_passes)
        self.buffers: List = [None] * self.size
        self.ttl = [0] * self.size
        self.idx = 0

    def get(self):
        if self.ttl[self.idx] <= 0:
            self.buffers[self.idx] = self.inqueue.get(timeout=self.timeout)
            self.ttl[self.idx] = self.cur_max_ttl
            if self.cur_max_ttl < self.max_ttl:
                self.cur_max_ttl += 1
        buf = self.buffers[self.idx]
        self.ttl[self.idx] -= 1
        released = self.ttl[self.idx] <= 0
        if released:
            self.buffers[self.idx] = None
        self.idx = (self.idx + 1) % len(self.buffers)
        return buf, released


class LearnerThread(threading.Thread):
    """Background learner consuming batches from ``inqueue`` (reference learner_thread.py)."""

    def __init__(self, local_worker, minibatch_buffer_size: int = 1, num_sgd_iter: int = 1,
                 learner_queue_size: int = 16, learner_queue_timeout: float = 300):
        super().__init__(daemon=True, name="rllib-learner")
        self.local_worker = local_worker
        self.inqueue: "queue.Queue" = queue.Queue(maxsize=learner_queue_size)
        self.outqueue: "queue.Queue" = queue.Queue()
        self.minibatch_buffer = MinibatchBuffer(self.inqueue, minibatch_buffer_size, learner_queue_timeout,
                                                num_sgd_iter)
        self.queue_timer, self.grad_timer = TimerStat(), TimerStat()
        self.stopped = False
        self.learner_info: Dict = {}
        self.num_steps = 0

    def run(self):
        while not self.stopped:
            self.step()

    def step(self):
        with self.queue_timer:
            try:
                batch, _ = self.minibatch_buffer.get()
            except queue.Empty:
                return
        with self.grad_timer:
            self.learner_info = _learn(self.local_worker, batch, 1, 0)
            self.num_steps += 1
        self.outqueue.put((_count(batch), self.learner_info))

    def add_learner_metrics(self, result: Dict) -> Dict:
        result.setdefault("info", {}).update(learner_queue={"size": self.inqueue.qsize()},
                                             timing_breakdown={"learner_grad_time_ms": self.grad_timer.mean * 1e3,
                                                               "learner_dequeue_time_ms": self.queue_timer.mean * 1e3})
        return result


class MultiGPULearnerThread(LearnerThread):
    """reference multi_gpu_learner_thread.py. The local worker's policy learns on its own device;
    the MI355X multi-GPU learner of the built-in algorithms is execution/learner_group.py."""

    def __init__(self, local_worker, num_gpus: int = 1, lr=None, train_batch_size: int = 500,
                 num_multi_gpu_tower_stacks: int = 1, num_sgd_iter: int = 1, learner_queue_size: int = 16,
                 learner_queue_timeout: float = 300, num_data_load_threads: int = 16, _fake_gpus: bool = False,
                 minibatch_buffer_size=None):
        super().__init__(local_worker, 1, num_sgd_iter, learner_queue_size, learner_queue_timeout)
        self.num_gpus = num_gpus
