"""Hand-off latencies of the runtime PPO iteration (rollout fragment -> learner update -> next sample) from
wall-clock stamps in the rollout worker, the learner actor and their task executors:
    python benchmarks/handoff_probe.py [--steps 20] [--dtype fp32]"""
import sys, argparse
sys.path.insert(0, ".")
import bench
import ray_memory_management_amd as ray

ap = argparse.ArgumentParser(); ap.add_argument("--dtype", default="fp32"); ap.add_argument("--steps", type=int, default=20)
a0 = ap.parse_args()
args = argparse.Namespace(rollout="hybrid", workers_per_learner=0, env_threads=1, fragment=100, minibatch=500,
                          sgd_iters=10, store_gb=8, dist_backend="nccl", dtype=a0.dtype, same_device=False,
                          learners_per_gpu=1, warmup=3)
algo, info = bench._runtime(args, 1)
w = algo.workers.remote_workers()[0]
l = algo.learner_group.learners[0]
ray.get([w.phase_stamps.remote(True), l.phase_stamps.remote(True)])
for _ in range(a0.steps):
    algo.train()
ws = ray.get(w.phase_stamps.remote(False)); ls = ray.get(l.phase_stamps.remote(False))
tasks_w = [t for t in ws if t[0] == "task"]; tasks_l = [t for t in ls if t[0] == "task"]
ws = [t for t in ws if t[0] != "task"]; ls = [t for t in ls if t[0] != "task"]
def show(tag, ts):
    for t in ts[-4:]:
        _, name, a, r, m, st = t
        print(f"{tag} {name}: resolve {1e3*(r-a):.3f} ms, method {1e3*(m-r):.3f} ms, store {1e3*(st-m):.3f} ms")
show("worker", [t for t in tasks_w if t[1] == "sample"]); show("learner", [t for t in tasks_l if t[1] == "update"])
ev = sorted(ws + ls, key=lambda e: e[1])
a, b = [], []
for (n1, t1), (n2, t2) in zip(ev, ev[1:]):
    if n1 == "sample_end" and n2 == "update_start":
        a.append(t2 - t1)
    if n1 == "update_end" and n2 == "sample_start":
        b.append(t2 - t1)
med = lambda x: sorted(x)[len(x) // 2] * 1e3 if x else float("nan")
print(f"sample_end->update_start median {med(a):.3f} ms (n={len(a)}); update_end->sample_start median {med(b):.3f} ms (n={len(b)})")
print("events:", [(n, round((t - ev[0][1]) * 1e3, 2)) for n, t in ev[:12]])
algo.stop(); ray.shutdown()
