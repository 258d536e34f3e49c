"""Phase breakdown of one runtime PPO iteration (bench.py's hybrid configuration on 1 MI355X):
driver wall per algo.train(), rollout workers' sample() and set_weights() time, learner update
time, learner get_weights (weight publish) time. Usage: python benchmarks/ppo_phase_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(iters: int = 10, warmup: int = 3, workers: int = 1):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    ray.init(num_cpus=16, num_gpus=1, object_store_memory=8 << 30, _system_config={"prestart_workers": 0})
    try:
        algo = (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"num_actions": 4, "episode_len": 1000})
                .rollouts(num_rollout_workers=workers, num_envs_per_worker=50 // workers, rollout_fragment_length=100,
                          postprocess_on_learner=True)
                .training(train_batch_size=5000, sgd_minibatch_size=500, num_sgd_iter=10, lr=5e-5, lambda_=0.95,
                          kl_coeff=0.5, clip_param=0.1, vf_clip_param=10.0, entropy_coeff=0.01)
                .resources(num_learner_workers=1, num_gpus_per_learner_worker=0.5, num_gpus_per_worker=0.5 / workers)
                .debugging(seed=0)).build()
        for _ in range(warmup):
            algo.train()
        ws = algo.workers.remote_workers()
        t_w0 = ray.get([w.timing.remote() for w in ws])
        upd = 0.0
        t0 = time.perf_counter()
        for _ in range(iters):
            r = algo.train()
            upd += r["info"]["learner"]["default_policy"]["learner_stats"]["learner_update_s"]
        wall = (time.perf_counter() - t0) / iters
        t_w1 = ray.get([w.timing.remote() for w in ws])
        l0 = algo.learner_group.learners[0]
        tg = time.perf_counter()
        for _ in range(5):
            ray.get(l0.get_weights.remote())
        get_w = (time.perf_counter() - tg) / 5
        out = {"iter_ms": round(wall * 1e3, 2), "learner_update_ms": round(upd / iters * 1e3, 2),
               "learner_get_weights_ms": round(get_w * 1e3, 2)}
        for i, (a, b) in enumerate(zip(t_w0, t_w1)):
            out[f"worker{i}_sample_ms"] = round((b["sample_s"] - a["sample_s"]) / iters * 1e3, 2)
            out[f"worker{i}_set_weights_ms"] = round((b["set_weights_s"] - a["set_weights_s"]) / iters * 1e3, 2)
        print(json.dumps(out), flush=True)
        algo.stop()
    finally:
        ray.shutdown()


if __name__ == "__main__":
    main(workers=int(sys.argv[1]) if len(sys.argv) > 1 else 1)
