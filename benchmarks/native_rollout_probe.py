"""Per-fragment time of ONE HybridRolloutWorker (native env + native rollout loop by default) in
isolation on one MI355X: ms per fragment and µs per env step for a given envs-per-worker, fragment
length and env-group split. Usage: python benchmarks/native_rollout_probe.py [n_envs] [T] [groups] [dtype]
(dtype bf16 or fp32: the policy's compute precision; fp32 runs the x3 kernels)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n: int = 50, T: int = 100, groups: int = 1, dtype: str = "bf16", frags: int = 20):
    import torch

    from ray_memory_management_amd.rllib.evaluation.gpu_rollout_worker import HybridRolloutWorker

    w = HybridRolloutWorker(config={"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 1000},
                                    "num_envs_per_worker": n, "rollout_fragment_length": T, "seed": 1,
                                    "rollout_double_buffer": groups > 1, "compute_dtype": dtype})
    for _ in range(3):
        w.sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(frags):
        w.sample()
    dt = (time.perf_counter() - t0) / frags
    from ray_memory_management_amd._native import require_hip

    srv = getattr(w, "_server_cache", None) is not None
    ph = ([round(x / T, 2) for x in require_hip().hybrid_rollout_phases()]
          if (getattr(w, "_native_desc", None) or srv) else None)
    prof = getattr(w, "_server_prof", None)
    if prof is not None:  # K21 stamps (100 MHz): go seen → trunk done → barrier 1 → barrier 2 → actions signalled
        p = prof.cpu().double()
        d = (p[1:, 1:] - p[1:, :-1]).mean(0) / 100.0  # µs, steps 1.. (step 0 includes the weight staging)
        gap = (p[1:, 0] - p[:-1, 4]).mean() / 100.0  # actions signalled → next step's go seen (host round trip)
        print(json.dumps({"server_us": {"trunk": round(float(d[0]), 2), "barrier1": round(float(d[1]), 2),
                                        "dense": round(float(d[2]), 2), "heads_signal": round(float(d[3]), 2),
                                        "host_round_trip": round(float(gap), 2)}}), flush=True)
    print(json.dumps({"n_envs": n, "T": T, "groups": len(w.groups), "dtype": dtype, "native_loop": getattr(w, "_native_desc", None) is not None,
                      "ms_per_fragment": round(dt * 1e3, 3), "us_per_step": round(dt / T * 1e6, 2),
                      "us_per_step_wait_env_launch": ph}), flush=True)


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:4]] + sys.argv[4:5]
    main(*a)
