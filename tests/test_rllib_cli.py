"""`rllib train` / `rllib evaluate` (reference rllib/tests/test_rllib_train_and_evaluate.py):
train PG on CartPole through Tune with a checkpoint at the end, then evaluate the checkpoint."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rllib(*args, timeout=300):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, "-m", "ray_memory_management_amd.rllib", *args], capture_output=True,
                          text=True, env=e, timeout=timeout)


def test_train_then_evaluate(tmp_path):
    r = _rllib("train", "--run", "PG", "--env", "CartPole-v1", "--num-cpus", "2", "--local-dir", str(tmp_path),
               "--config", json.dumps({"num_workers": 0, "train_batch_size": 200, "rollout_fragment_length": 200,
                                       "model": {"fcnet_hiddens": [16]}}),
               "--stop", json.dumps({"training_iteration": 2}), "--checkpoint-at-end")
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert rows and rows[-1]["training_iteration"] == 2 and rows[-1]["checkpoint"], r.stdout
    out = tmp_path / "rollouts.jsonl"
    r = _rllib("evaluate", rows[-1]["checkpoint"], "--run", "PG", "--env", "CartPole-v1", "--episodes", "2",
               "--num-cpus", "2", "--config", json.dumps({"model": {"fcnet_hiddens": [16]}}), "--out", str(out))
    assert r.returncode == 0, r.stdout + r.stderr
    summ = json.loads([ln for ln in r.stdout.splitlines() if "episode_reward_mean" in ln][-1])
    assert summ["episodes"] == 2 and summ["episode_reward_mean"] > 0
    assert out.exists() and len(out.read_text().splitlines()) > 2
