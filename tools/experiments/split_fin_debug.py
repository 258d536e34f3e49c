"""Where do tail+deferred-finalize and split K12 -> finalize -> K6 differ? One eager update each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner  # noqa: E402
from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv  # noqa: E402
from ray_memory_management_amd.rllib.models import VisionNetwork  # noqa: E402

cuda = torch.device("cuda:0")
os.environ["RMM_K12_SPLIT"] = "2"
graphs = len(sys.argv) > 1 and sys.argv[1] == "graphs"
env = GPUSyntheticAtariVectorEnv(16, cuda, num_actions=4, seed=0)
torch.manual_seed(0)
base = VisionNetwork(4)
cfg = {"sgd_minibatch_size": 128, "num_sgd_iter": int(os.environ.get("DBG_ITERS", "1")), "use_graphs": graphs}
L = {}
for tail in ("0", "1"):
    os.environ["RMM_TAIL_ADAM"] = tail
    m = VisionNetwork(4)
    m.load_state_dict(base.state_dict())
    L[tail] = PPOLearner(m, dict(cfg), device=cuda, action_space=env.action_space)
sampler = GPURolloutSampler(env, L["0"].model, fragment=16, use_graphs=False)
first = sampler.sample()
Batch = type(first)
batches = [{k: v.clone() for k, v in first.items()}, {k: v.clone() for k, v in sampler.sample().items()}]
snaps = {}
for tail, ln in L.items():
    os.environ["RMM_TAIL_ADAM"] = tail
    for i, b in enumerate(batches[:int(os.environ.get("DBG_UPDATES", "1"))]):
        torch.manual_seed(100 + i)
        ln.update(Batch({k: v.clone() for k, v in b.items()}))
        snaps[(tail, i)] = ln.master.clone()
    print("tail", tail, "split_fin", ln._split_fin(), "graphs", ln.graphs, "chain", getattr(ln, "_chain", None),
          "ctr", ln.ctr.tolist())
a = L["0"]
names = {id(p): n for n, p in a.model.named_parameters()}
for i in range(int(os.environ.get("DBG_UPDATES", "1"))):
    off = 0
    for p in a.params:
        n = p.numel()
        d = (snaps[("0", i)][off:off + n] - snaps[("1", i)][off:off + n]).abs()
        print(f"update {i} {names[id(p)]:22s} max|d| {float(d.max()):.3e} ndiff {int((d > 0).sum())}")
        off += n
