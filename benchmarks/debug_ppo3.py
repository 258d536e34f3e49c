"""Compare the captured SGD step's gradients with an eager step on identical inputs (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv  # noqa: E402
from ray_memory_management_amd.rllib.models import VisionNetwork  # noqa: E402
from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    env = GPUSyntheticAtariVectorEnv(50, dev, num_actions=4)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 500, "num_sgd_iter": 1}, device=dev,
                   action_space=env.action_space)
    S = GPURolloutSampler(env, L.model, fragment=100, use_graphs=False)
    b = S.sample()
    L.update(b)  # captures
    names = [n for n, _ in L.model.named_parameters()]
    sizes = [p.numel() for p in L.params]
    for trial in range(6):
        b = S.sample()
        packed = L._pack(b)
        for k in ("obs", "cols", "actions"):
            L._static[k].copy_(packed[k])
        idx = torch.randperm(5000, device=dev)[:500]
        state = [t.clone() for t in (L.master, L.m1, L.m2, L.hp, L.w_bf16)]
        L._sidx.copy_(idx)
        L.acc.zero_()
        L._fast_step(L._static, L._sidx, False)
        torch.cuda.synchronize()
        ge = L.flat_grad.float().clone()
        acc_e = L.acc.clone()
        for dst, src in zip((L.master, L.m1, L.m2, L.hp, L.w_bf16), state):
            dst.copy_(src)
        L.acc.zero_()
        L._graph.replay()
        torch.cuda.synchronize()
        gg = L.flat_grad.float().clone()
        acc_g = L.acc.clone()
        for dst, src in zip((L.master, L.m1, L.m2, L.hp, L.w_bf16), state):
            dst.copy_(src)
        off = 0
        print(f"trial {trial}: stats eager {acc_e.tolist()}\n          graph {acc_g.tolist()}", flush=True)
        for n, k in zip(names, sizes):
            a, c = ge[off:off + k], gg[off:off + k]
            d = float((a - c).abs().max())
            print(f"   {n:24s} n={k:8d} |g|max={float(a.abs().max()):.3e} maxdiff={d:.3e} "
                  f"finite_g={bool(torch.isfinite(c).all())}", flush=True)
            off += k


if __name__ == "__main__":
    main()
