"""Episode metrics. Parity: reference rllib/evaluation/metrics.py (collect_episodes,
summarize_episodes, collect_metrics). Episodes are (total_reward, length) records gathered from the
workers' ``get_metrics()``."""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np


def collect_episodes(local_worker=None, remote_workers=(), to_be_collected=(), timeout_seconds: int = 180) -> List:
    import ray_memory_management_amd as ray

    eps = list(local_worker.get_metrics()) if local_worker is not None else []
    if remote_workers:
        for m in ray.get([w.get_metrics.remote() for w in remote_workers], timeout=timeout_seconds):
            eps += m
    return eps


def summarize_episodes(episodes: Sequence, new_episodes: Sequence = None, keep_custom_metrics: bool = False) -> Dict:
    eps = list(episodes)
    rewards = [float(e[0]) for e in eps]
    lens = [int(e[1]) for e in eps]
    nan = float("nan")
    return {
        "episode_reward_max": max(rewards) if rewards else nan,
        "episode_reward_min": min(rewards) if rewards else nan,
        "episode_reward_mean": float(np.mean(rewards)) if rewards else nan,
        "episode_len_mean": float(np.mean(lens)) if lens else nan,
        "episodes_this_iter": len(new_episodes if new_episodes is not None else eps),
        "hist_stats": {"episode_reward": rewards, "episode_lengths": lens},
        "custom_metrics": {},
        "policy_reward_min": {}, "policy_reward_max": {}, "policy_reward_mean": {},
        "sampler_perf": {},
    }


def collect_metrics(local_worker=None, remote_workers=(), to_be_collected=(), timeout_seconds: int = 180,
                    keep_custom_metrics: bool = False) -> Dict:
    """Episode stats of a worker set (or of a local worker + remote workers)."""
    if hasattr(local_worker, "collect_metrics") and not remote_workers:  # a WorkerSet
        eps = local_worker.collect_metrics()
    else:
        eps = collect_episodes(local_worker, remote_workers, to_be_collected, timeout_seconds)
    return summarize_episodes(eps)
