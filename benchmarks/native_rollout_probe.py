"""Per-fragment time of ONE HybridRolloutWorker (native env + native rollout loop by default) in
isolation on one MI355X: ms per fragment and µs per env step for a given envs-per-worker, fragment
length and env-group split. Usage: python benchmarks/native_rollout_probe.py [n_envs] [T] [groups]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n: int = 50, T: int = 100, groups: int = 1, frags: int = 20):
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    w = HybridRolloutWorker(config={"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 1000},
                                    "num_envs_per_worker": n, "rollout_fragment_length": T, "seed": 1,
                                    "rollout_double_buffer": groups > 1})
    for _ in range(3):
        w.sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frags):
        w.sample()
    dt = (time.perf_counter() - t0) / frags
    from ray_memory_management_amd._native import require_hip

    ph = [round(x / T, 2) for x in require_hip().hybrid_rollout_phases()] if getattr(w, "_native_desc", None) else None
    print(json.dumps({"n_envs": n, "T": T, "groups": len(w.groups), "native_loop": getattr(w, "_native_desc", None) is not None,
                      "ms_per_fragment": round(dt * 1e3, 3), "us_per_step": round(dt / T * 1e6, 2),
                      "us_per_step_wait_env_launch": ph}), flush=True)


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
