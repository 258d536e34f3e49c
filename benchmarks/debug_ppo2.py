"""Find the first SGD step that produces a non-finite value (debug aid; eager, synchronising)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["RMM_NO_GRAPHS"] = "1"
import torch  # noqa: E402

from ray_memory_management_amd import ops  # noqa: E402
from ray_memory_management_amd.rllib import ppo_learner as PL  # noqa: E402
from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv  # noqa: E402
from ray_memory_management_amd.rllib.models import VisionNetwork  # noqa: E402

state = {"step": 0, "done": False}


def checked_step(self, full, idx, with_opt):
    if state["done"]:
        return orig(self, full, idx, with_opt)
    x = ops.frames_to_nhwc(full["obs"], idx)
    cols = ops.gather_rows(full["cols"], idx)
    act = ops.gather_rows(full["actions"], idx)
    A = full["A"]
    logits, v = self.model(x, prescaled=True)
    bad = []
    for n, t in (("x", x), ("cols", cols), ("logits", logits), ("v", v)):
        if not torch.isfinite(t.float()).all():
            bad.append(n)
    orig(self, full, idx, with_opt)
    for n, t in (("flat_grad", self.flat_grad), ("master", self.master), ("m2", self.m2)):
        if not torch.isfinite(t.float()).all():
            bad.append(n)
    state["step"] += 1
    if bad:
        print(f"step {state['step']}: non-finite {bad}; logits absmax {float(logits.float().abs().max()):.3g} "
              f"v absmax {float(v.float().abs().max()):.3g} grad absmax {float(self.flat_grad.float().abs().max()):.3g}"
              f" hp {self.hp.tolist()}", flush=True)
        h = self.model
        for name, p in h.named_parameters():
            print("   ", name, float(p.float().abs().max()), flush=True)
        state["done"] = True
    elif state["step"] % 100 == 0:
        print(f"step {state['step']} ok: logits {float(logits.float().abs().max()):.3g} v {float(v.float().abs().max()):.3g}"
              f" grad {float(self.flat_grad.float().abs().max()):.3g} m2max {float(self.m2.max()):.3g}", flush=True)


orig = PL.PPOLearner._fast_step
PL.PPOLearner._fast_step = checked_step


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    env = GPUSyntheticAtariVectorEnv(50, dev, num_actions=4)
    L = PL.PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 500, "num_sgd_iter": 10}, device=dev,
                      action_space=env.action_space)
    S = PL.GPURolloutSampler(env, L.model, fragment=100)
    for it in range(14):
        b = S.sample()
        st = L.update(b)
        print(it, {k: round(v, 4) if isinstance(v, float) else v for k, v in st.items()}, flush=True)
        if state["done"]:
            break


if __name__ == "__main__":
    main()
