"""Three fragments of one HybridRolloutWorker (n=25, one env group) for a kernel trace: run under
`rocprofv3 --kernel-trace` and read the per-step GPU span and the gaps between the step's kernels.
argv[1] = "graph" (default) or "eager"; argv[2] = "double" for the default two env groups (12 + 13)."""
import sys

sys.path.insert(0, ".")

from ray_memory_management_amd.rllib.evaluation import gpu_rollout_worker as G  # noqa: E402


def main():
    graphs = (sys.argv[1] if len(sys.argv) > 1 else "graph") == "graph"
    double = len(sys.argv) > 2 and sys.argv[2] == "double"
    w = G.HybridRolloutWorker(config={"env": "SyntheticAtariVec-v0", "env_config": {"episode_len": 1000},
                                      "num_envs_per_worker": 25, "rollout_fragment_length": 100, "seed": 1,
                                      "rollout_double_buffer": double, "rollout_graphs": graphs})
    for _ in range(3):
        w.sample()
    print("done", flush=True)


if __name__ == "__main__":
    main()
