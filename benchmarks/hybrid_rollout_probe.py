"""Per-step timing of one HybridRolloutWorker (CPU env + GPU policy) in isolation: total per env
step, time blocked on the GPU (event waits) and time in the CPU env step, for 1 vs 2 env groups."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")

from ray_memory_management_amd.rllib.evaluation import gpu_rollout_worker as G  # noqa: E402


def main():
    waits = {"sync": 0.0, "env": 0.0}
    orig_step = G._EnvGroup.env_step

    def env_step(self, t, completed):
        t0 = time.perf_counter()
        orig_step(self, t, completed)
        waits["env"] += time.perf_counter() - t0

    G._EnvGroup.env_step = env_step
    orig_sync = torch.cuda.Event.synchronize

    def sync(self):
        t0 = time.perf_counter()
        orig_sync(self)
        waits["sync"] += time.perf_counter() - t0

    torch.cuda.Event.synchronize = sync
    for n, dbl in ((25, False), (25, True), (50, True)):
        w = G.HybridRolloutWorker(config={"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 1000},
                                          "num_envs_per_worker": n, "rollout_fragment_length": 100, "seed": 1,
                                          "rollout_double_buffer": dbl})
        w.sample()
        waits["sync"] = waits["env"] = 0.0
        k = 5
        t0 = time.perf_counter()
        for _ in range(k):
            w.sample()
        el = (time.perf_counter() - t0) / k
        print(f"n={n} double_buffer={dbl}: {el * 1e3:.2f} ms/fragment = {el / 100 * 1e6:.1f} us/step; "
              f"gpu-wait {waits['sync'] / k / 100 * 1e6:.1f} us/step, env {waits['env'] / k / 100 * 1e6:.1f} us/step",
              flush=True)


if __name__ == "__main__":
    main()
