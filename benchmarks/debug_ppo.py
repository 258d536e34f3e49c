"""Stage-by-stage finiteness check of the fused PPO path at bench scale (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv  # noqa: E402
from ray_memory_management_amd.rllib.models import VisionNetwork  # noqa: E402
from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner  # noqa: E402


def fin(name, t):
    ok = bool(torch.isfinite(t.float()).all())
    print(f"  {name}: finite={ok} absmax={float(t.float().abs().max()):.4g}", flush=True)
    return ok


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(int(os.environ.get("SEED", "0")))
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    mbs = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    env = GPUSyntheticAtariVectorEnv(envs, dev, num_actions=4)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": mbs, "num_sgd_iter": 10}, device=dev,
                   action_space=env.action_space)
    S = GPURolloutSampler(env, L.model, fragment=100, use_graphs=not os.environ.get("NO_SAMPLER_GRAPH"))
    if os.environ.get("NO_LEARNER_GRAPH"):
        L.graphs = False
    if os.environ.get("SYNC_EACH"):
        import torch.cuda.graphs as tg

        orig_replay = tg.CUDAGraph.replay

        def replay(self):
            orig_replay(self)
            torch.cuda.synchronize()

        tg.CUDAGraph.replay = replay
    print("graphs", L.graphs, S.graphs)
    for it in range(int(os.environ.get("ITERS", "4"))):
        b = S.sample()
        print(f"iter {it}")
        for k in ("action_logp", "vf_preds", "action_dist_inputs", "advantages", "value_targets"):
            fin(k, b[k])
        st = L.update(b)
        print("  stats", st)
        fin("master", L.master)
        fin("w_bf16", L.w_bf16)
        fin("m2", L.m2)
        fin("flat_grad", L.flat_grad)


if __name__ == "__main__":
    main()
