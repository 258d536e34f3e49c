"""More namespace parity: tune.logger, runtime_env.RuntimeEnv, data.datasource partitioning /
metadata / write-path providers / extra datasources, framework checkpoints, experimental exports.
Mirrors reference tests test_logger.py, test_runtime_env.py (validation), data test_partitioning.py."""
import os

import numpy as np
import pandas as pd
import pytest

import ray_memory_management_amd as ray


def test_tune_loggers(tmp_path):
    from ray_memory_management_amd.tune import logger as L

    class T:
        trial_id, config, logdir = "t1", {"lr": 0.1}, str(tmp_path / "trial")

    cb = L.LegacyLoggerCallback([L.JsonLogger, L.CSVLogger])
    cb.on_trial_start(0, [], T)
    for i in range(3):
        cb.on_trial_result(i, [], T, {"training_iteration": i + 1, "m": {"a": i}})
    cb.on_trial_complete(3, [], T)
    d = os.path.join(T.logdir, "legacy")
    assert len(open(os.path.join(d, "result.json")).read().splitlines()) == 3
    df = pd.read_csv(os.path.join(d, "progress.csv"))
    assert list(df["m/a"]) == [0, 1, 2]
    u = L.UnifiedLogger({"x": 1}, str(tmp_path / "u"))
    u.on_result({"a": 1})
    u.close()
    assert "a: 1" in L.pretty_print({"a": 1, "config": {"z": 2}})
    with pytest.raises(ImportError):
        L.TBXLogger({}, str(tmp_path / "tb"))


def test_runtime_env_class(ray_start):
    from ray_memory_management_amd.runtime_env import RuntimeEnv, RuntimeEnvConfig

    r = RuntimeEnv(env_vars={"RMM_T": "7"}, config=RuntimeEnvConfig(setup_timeout_seconds=30))
    assert RuntimeEnv.deserialize(r.serialize()) == r and r.env_vars() == {"RMM_T": "7"}
    with pytest.raises(ValueError):
        RuntimeEnv(bogus=1)
    with pytest.raises(TypeError):
        RuntimeEnv(env_vars={"A": 1})

    @ray.remote
    def f():
        return os.environ.get("RMM_T")

    assert ray.get(f.options(runtime_env=RuntimeEnv(env_vars={"RMM_T": "7"})).remote()) == "7"


def test_partitioning_filters_and_write_paths(ray_start, tmp_path):
    from ray_memory_management_amd.data import datasource as D

    enc = D.PathPartitionEncoder.of(field_names=["year", "country"], base_dir=str(tmp_path))
    for year, country in (("2021", "us"), ("2022", "us"), ("2022", "fr")):
        d = enc([year, country])
        os.makedirs(d)
        pd.DataFrame({"v": [int(year)]}).to_csv(os.path.join(d, "a.csv"), index=False)
    assert enc(["1", "x"]).endswith("year=1/country=x")
    parser = D.PathPartitionParser.of(base_dir=str(tmp_path))
    assert parser(str(tmp_path / "year=2022" / "country=fr" / "a.csv")) == {"year": "2022", "country": "fr"}
    dparser = D.PathPartitionParser.of(style=D.PartitionStyle.DIRECTORY, field_names=["y", "c"],
                                       base_dir=str(tmp_path))
    assert dparser(str(tmp_path / "2022" / "fr" / "f.csv")) == {"y": "2022", "c": "fr"}
    flt = D.PathPartitionFilter.of(lambda p: p["year"] == "2022", base_dir=str(tmp_path))
    ds = ray.data.read_csv(str(tmp_path), partition_filter=flt)
    assert sorted(r["v"] for r in ds.take_all()) == [2022, 2022]
    assert D.FileExtensionFilter("csv")("x/a.CSV") and not D.FileExtensionFilter(["json"])("a.csv")
    files, sizes = D.DefaultFileMetadataProvider().expand_paths(str(tmp_path))
    assert len(files) == 3 and all(s > 0 for s in sizes)
    assert D.FastFileMetadataProvider().expand_paths(str(tmp_path))[1] == [None] * 3

    class ByIndex(D.BlockWritePathProvider):
        def _get_write_path_for_block(self, base_path, *, block_index=None, file_format=None, **kw):
            return os.path.join(base_path, f"part{block_index}", f"data.{file_format}")

    out = tmp_path / "out"
    ray.data.range_table(10, parallelism=2).write_csv(str(out), block_path_provider=ByIndex())
    assert sorted(os.listdir(out)) == ["part0", "part1"]


def test_extra_datasources(ray_start):
    from ray_memory_management_amd.data import datasource as D

    ds = ray.data.read_datasource(D.RandomIntRowDatasource(), parallelism=2, n=10, num_columns=3)
    assert ds.count() == 10
    ds = ray.data.read_datasource(D.SimpleTorchDatasource(), parallelism=2, dataset_factory=lambda: list(range(7)))
    assert sorted(ds.take_all()) == list(range(7))


def test_framework_checkpoints_and_experimental(tmp_path):
    from sklearn.linear_model import LinearRegression

    from ray_memory_management_amd import experimental
    from ray_memory_management_amd.train.sklearn import SklearnCheckpoint, SklearnPredictor

    est = LinearRegression().fit(np.arange(6).reshape(-1, 1), np.arange(6) * 2.0)
    ck = SklearnCheckpoint.from_estimator(est)
    assert ck.get_estimator().coef_[0] == pytest.approx(2.0)
    pred = SklearnPredictor.from_checkpoint(ck)
    out = pred.predict(pd.DataFrame({"x": [10.0]}))
    assert float(np.asarray(out).ravel()[0]) == pytest.approx(20.0)
    assert callable(experimental.get_object_locations) and callable(experimental.set_resource)
    with pytest.raises(NotImplementedError):
        experimental.load_package("x.yaml")
    from ray_memory_management_amd.util.multiprocessing import JoinableQueue

    assert JoinableQueue is not None
