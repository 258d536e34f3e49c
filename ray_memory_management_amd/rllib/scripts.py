"""`rllib train` / `rllib evaluate` command line. Parity: reference rllib/scripts.py, rllib/train.py
(--run ALGO --env ENV --config JSON --stop JSON [--checkpoint-freq N --checkpoint-at-end] via Tune,
or -f tuned_example.yaml) and rllib/evaluate.py (restore a checkpoint, roll out N episodes greedily,
optionally write them with --out).

    python -m ray_memory_management_amd.rllib train --run PPO --env CartPole-v1 \\
        --stop '{"training_iteration": 5}' --config '{"num_workers": 2}'
    python -m ray_memory_management_amd.rllib evaluate <checkpoint_dir> --run PPO --env CartPole-v1 --episodes 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional


def _load_yaml(path: str) -> dict:
    import yaml

    with open(path) as f:
        return yaml.safe_load(f)


def cmd_train(a) -> int:
    import ray_memory_management_amd as ray
    from ray_memory_management_amd import tune
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    experiments = {}
    if a.config_file:
        experiments = _load_yaml(a.config_file)
    else:
        if not a.run or not a.env:
            print("train: --run and --env (or -f FILE) are required", file=sys.stderr)
            return 2
        experiments = {a.experiment_name or "default": {
            "run": a.run, "env": a.env, "config": json.loads(a.config or "{}"),
            "stop": json.loads(a.stop or "{}"), "checkpoint_freq": a.checkpoint_freq,
            "checkpoint_at_end": a.checkpoint_at_end}}
    if not ray.is_initialized():
        ray.init(num_cpus=a.num_cpus, num_gpus=a.num_gpus)
    last = None
    for name, spec in experiments.items():
        cls = get_algorithm_class(spec["run"])
        cfg = dict(spec.get("config") or {})
        if spec.get("env") is not None:
            cfg["env"] = spec["env"]
        analysis = tune.run(cls, name=name, config=cfg, stop=spec.get("stop") or {"training_iteration": 1},
                            checkpoint_freq=int(spec.get("checkpoint_freq", 0) or 0),
                            checkpoint_at_end=bool(spec.get("checkpoint_at_end", False)),
                            local_dir=a.local_dir, verbose=0)
        for t in analysis.trials:
            r = t.last_result or {}
            print(json.dumps({"experiment": name, "trial": t.trial_id,
                              "training_iteration": r.get("training_iteration"),
                              "episode_reward_mean": r.get("episode_reward_mean"),
                              "timesteps_total": r.get("timesteps_total"), "logdir": t.logdir,
                              "checkpoint": t.saved_checkpoints[-1][0] if t.saved_checkpoints else None}),
                  flush=True)
        last = analysis
    return 0 if last is not None else 1


def cmd_evaluate(a) -> int:
    import numpy as np

    import ray_memory_management_amd as ray
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class
    from ray_memory_management_amd.rllib.env import make_env

    if not ray.is_initialized():
        ray.init(num_cpus=a.num_cpus)
    cfg = json.loads(a.config or "{}")
    cfg["env"] = a.env
    cfg.setdefault("num_workers", 0)
    algo = get_algorithm_class(a.run)(config=cfg)
    algo.restore(a.checkpoint)
    env = make_env(a.env, cfg.get("env_config") or {})
    rets, rows = [], []
    for k in range(a.episodes):
        o, done, ret, steps = env.reset(seed=k), False, 0.0, 0
        while not done and steps < a.max_steps:
            act = algo.compute_single_action(o, explore=False)
            o2, r, done, _ = env.step(act)
            rows.append({"episode": k, "obs": np.asarray(o).tolist(), "action": np.asarray(act).tolist(), "reward": r})
            o, ret, steps = o2, ret + r, steps + 1
        rets.append(ret)
        print(json.dumps({"episode": k, "reward": ret, "length": steps}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for row in rows:
                f.write(json.dumps(row) + "\n")
    print(json.dumps({"episode_reward_mean": float(np.mean(rets)), "episodes": len(rets)}), flush=True)
    algo.stop()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="rllib")
    sub = p.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train", help="train an algorithm through Tune")
    t.add_argument("--run", default=None)
    t.add_argument("--env", default=None)
    t.add_argument("--config", default=None, help="JSON algorithm config")
    t.add_argument("--stop", default=None, help='JSON stop criteria, e.g. {"training_iteration": 5}')
    t.add_argument("-f", "--config-file", default=None, help="tuned-example YAML (experiments by name)")
    t.add_argument("--experiment-name", default=None)
    t.add_argument("--checkpoint-freq", type=int, default=0)
    t.add_argument("--checkpoint-at-end", action="store_true")
    t.add_argument("--local-dir", default=os.path.expanduser("~/rmm_results"))
    t.add_argument("--num-cpus", type=int, default=None)
    t.add_argument("--num-gpus", type=int, default=None)
    t.set_defaults(fn=cmd_train)
    e = sub.add_parser("evaluate", help="roll out a checkpointed policy")
    e.add_argument("checkpoint")
    e.add_argument("--run", required=True)
    e.add_argument("--env", required=True)
    e.add_argument("--config", default=None)
    e.add_argument("--episodes", type=int, default=5)
    e.add_argument("--max-steps", type=int, default=100000)
    e.add_argument("--out", default=None, help="write the rollouts as JSON lines")
    e.add_argument("--num-cpus", type=int, default=None)
    e.set_defaults(fn=cmd_evaluate)
    a = p.parse_args(argv)
    return a.fn(a)
