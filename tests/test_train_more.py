"""SklearnTrainer / SklearnPredictor, RLTrainer / RLPredictor, and util helpers
(register_serializer, inspect_serializability, log_once, accelerators, remote pdb). Mirrors
reference python/ray/train/tests/{test_sklearn_trainer,test_rl_trainer}.py and
python/ray/tests/{test_serialization,test_debug_tools}.py at small scale."""
import io
import socket
import threading

import numpy as np
import pandas as pd
import pytest


def _frames(n=200, seed=0):
    g = np.random.default_rng(seed)
    X = g.standard_normal((n, 4))
    y = (X[:, 0] + 0.5 * X[:, 1] > 0).astype(int)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = y
    return df


def test_sklearn_trainer_fit_cv_and_predictor(ray_shared):
    from sklearn.linear_model import LogisticRegression

    import ray_memory_management_amd.data as data
    from ray_memory_management_amd.train.sklearn import SklearnPredictor, SklearnTrainer

    train = data.from_pandas(_frames(300, 0))
    valid = data.from_pandas(_frames(100, 1))
    t = SklearnTrainer(estimator=LogisticRegression(), datasets={"train": train, "valid": valid}, label_column="y",
                       cv=3, scoring="accuracy", params={"C": 10.0})
    res = t.fit()
    assert res.error is None, res.error
    assert res.metrics["valid/score"] > 0.9 and res.metrics["cv/test_score_mean"] > 0.9
    assert len(res.metrics["cv"]["test_score"]) == 3
    pred = SklearnPredictor.from_checkpoint(res.checkpoint)
    assert pred.estimator.C == 10.0
    out = pred.predict(_frames(50, 2).drop(columns=["y"]))
    assert list(out.columns) == ["predictions"] and len(out) == 50
    with pytest.raises(ValueError):
        from ray_memory_management_amd.air.config import ScalingConfig

        SklearnTrainer(estimator=LogisticRegression(), datasets={"train": train}, label_column="y",
                       scaling_config=ScalingConfig(num_workers=2))


def test_rl_trainer_and_predictor(ray_shared):
    from ray_memory_management_amd.air.config import RunConfig
    from ray_memory_management_amd.train.rl import RLPredictor, RLTrainer

    t = RLTrainer("PG", config={"env": "CartPole-v1", "num_workers": 0, "train_batch_size": 200,
                                "rollout_fragment_length": 200, "model": {"fcnet_hiddens": [16]}, "seed": 0},
                  run_config=RunConfig(stop={"training_iteration": 3}))
    res = t.fit()
    assert res.error is None, res.error
    assert res.metrics["training_iteration"] == 3 and len(res.metrics_history) == 3
    p = RLPredictor.from_checkpoint(res.checkpoint)
    acts = p.predict(np.zeros((5, 4), np.float32))
    assert acts.shape == (5,) and set(np.unique(acts)) <= {0, 1}


class _Opaque:
    def __init__(self, v):
        self.v = v
        self.lock = threading.Lock()  # not picklable on its own


def test_register_serializer_roundtrip(ray_shared):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.util import deregister_serializer, register_serializer

    with pytest.raises(Exception):
        ray.put(_Opaque(1))
    register_serializer(_Opaque, serializer=lambda o: o.v, deserializer=lambda v: _Opaque(v * 10))
    try:
        assert ray.get(ray.put(_Opaque(4))).v == 40
    finally:
        deregister_serializer(_Opaque)


def test_inspect_serializability_finds_culprit():
    from ray_memory_management_amd.util import inspect_serializability

    lock = threading.Lock()

    def uses_lock():
        return lock

    ok, fails = inspect_serializability(uses_lock, name="uses_lock", print_file=io.StringIO())
    assert not ok and any(f.name == "lock" for f in fails)
    ok, fails = inspect_serializability(lambda x: x + 1)
    assert ok and not fails


def test_log_once_and_accelerators():
    from ray_memory_management_amd.util import accelerators, debug

    debug.reset_log_once()
    assert debug.log_once("k") and not debug.log_once("k") and debug.log_once("k2")
    assert accelerators.AMD_INSTINCT_MI355X == "AMD-Instinct-MI355X"


def test_remote_pdb_session(ray_shared):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.util import rpdb

    @ray.remote
    def debug_me():
        x = 41
        rpdb.set_trace(breakpoint_uuid="bp1", timeout=60)
        return x + 1

    ref = debug_me.remote()
    bps = []
    import time

    deadline = time.time() + 30
    while time.time() < deadline and not bps:
        bps = [b for b in rpdb.list_breakpoints() if b["uuid"] == "bp1"]
        time.sleep(0.1)
    assert bps, "breakpoint never registered"
    s = socket.create_connection((bps[0]["host"], bps[0]["port"]), timeout=30)
    f = s.makefile("rw")
    f.write("p x\n")
    f.flush()
    buf = ""
    while "41" not in buf:
        buf += f.readline()
    f.write("c\n")
    f.flush()
    assert ray.get(ref, timeout=30) == 42
    s.close()
