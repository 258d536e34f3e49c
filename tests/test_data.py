"""Data library: mirrors reference python/ray/data/tests/{test_dataset,test_sort,test_split,
test_dataset_formats,test_dataset_pipeline,test_preprocessors}.py at smaller scale."""
import os

import numpy as np
import pandas as pd
import pytest


@pytest.fixture(scope="module")
def ray_data(ray_shared):
    import ray_memory_management_amd.data as data

    return ray_shared, data


def test_basic_range_and_transforms(ray_data):
    ray, data = ray_data
    ds = data.range(100, parallelism=5)
    assert ds.count() == 100 and ds.num_blocks() == 5
    assert ds.take(3) == [0, 1, 2]
    assert ds.map(lambda x: x * 2).take(3) == [0, 2, 4]
    assert ds.filter(lambda x: x % 10 == 0).take_all() == list(range(0, 100, 10))
    assert ds.flat_map(lambda x: [x, x]).count() == 200
    assert sorted(ds.map_batches(lambda b: [x + 1 for x in b], batch_size=7).take_all()) == list(range(1, 101))
    assert ds.sum() == sum(range(100)) and ds.min() == 0 and ds.max() == 99
    assert ds.mean() == pytest.approx(49.5)
    assert ds.std() == pytest.approx(np.std(np.arange(100), ddof=1))
    with pytest.raises(TypeError):
        iter(ds)


def test_lazy_fusion_and_stats(ray_data):
    ray, data = ray_data
    ds = data.range(20, parallelism=4).lazy().map(lambda x: x + 1).map(lambda x: x * 3)
    assert not ds.is_fully_executed()
    assert ds.take_all() == [(i + 1) * 3 for i in range(20)]
    assert "map(<lambda>)->map(<lambda>)" in ds.stats()  # the two stages ran fused


def test_table_ops(ray_data):
    ray, data = ray_data
    ds = data.from_items([{"a": i, "b": i % 3, "c": float(i)} for i in range(30)], parallelism=3)
    assert ds.count() == 30 and ds.schema().names == ["a", "b", "c"]
    assert ds.sum("a") == sum(range(30))
    g = ds.groupby("b").count().take_all()
    assert g == [{"b": 0, "count()": 10}, {"b": 1, "count()": 10}, {"b": 2, "count()": 10}]
    s = ds.groupby("b").sum("a").take_all()
    assert [r["sum(a)"] for r in s] == [sum(range(0, 30, 3)), sum(range(1, 30, 3)), sum(range(2, 30, 3))]
    m = ds.groupby("b").aggregate(data.Mean("c"), data.Max("a")).take_all()
    assert m[2]["max(a)"] == 29 and m[0]["mean(c)"] == pytest.approx(np.mean(range(0, 30, 3)))
    mg = ds.groupby("b").map_groups(lambda df: df.head(1), batch_format="pandas").take_all()
    assert [r["a"] for r in mg] == [0, 1, 2]
    df = ds.add_column("d", lambda df: df["a"] * 2).drop_columns(["c"]).to_pandas()
    assert list(df.columns) == ["a", "b", "d"] and (df["d"] == df["a"] * 2).all()
    pbatches = list(ds.iter_batches(batch_size=8, batch_format="pandas"))
    assert [len(b) for b in pbatches] == [8, 8, 8, 6] and isinstance(pbatches[0], pd.DataFrame)


def test_sort_shuffle_repartition(ray_data):
    ray, data = ray_data
    ds = data.range(200, parallelism=8).random_shuffle(seed=1)
    vals = ds.take_all()
    assert sorted(vals) == list(range(200)) and vals != list(range(200))
    assert ds.sort().take_all() == list(range(200))
    assert ds.sort(descending=True).take(3) == [199, 198, 197]
    t = data.from_items([{"k": (i * 37) % 101, "v": i} for i in range(101)], parallelism=4)
    assert [r["k"] for r in t.sort("k").take_all()] == list(range(101))
    r = data.range(100, parallelism=3).repartition(7)
    assert r.num_blocks() == 7 and r.take_all() == list(range(100))
    assert sorted(data.range(50, parallelism=2).repartition(4, shuffle=True).take_all()) == list(range(50))
    rb = data.range(40, parallelism=4).randomize_block_order(seed=0)
    assert sorted(rb.take_all()) == list(range(40))
    smp = data.range(1000, parallelism=4).random_sample(0.1, seed=3).count()
    assert 40 < smp < 180


def test_push_based_shuffle(ray_data):
    ray, data = ray_data
    ctx = data.DatasetContext.get_current()
    ctx.use_push_based_shuffle = True
    try:
        ds = data.range(300, parallelism=12).random_shuffle(seed=5)
        assert sorted(ds.take_all()) == list(range(300))
    finally:
        ctx.use_push_based_shuffle = False


def test_split_zip_union_limit(ray_data):
    ray, data = ray_data
    ds = data.range(20, parallelism=4)
    parts = ds.split(3)
    assert sum(p.count() for p in parts) == 20
    eq = ds.split(3, equal=True)
    assert [p.count() for p in eq] == [6, 6, 6]
    a, b, c = ds.split_at_indices([5, 12])
    assert a.take_all() == list(range(5)) and b.take_all() == list(range(5, 12)) and c.count() == 8
    tr, te = ds.train_test_split(0.25)
    assert tr.count() == 15 and te.count() == 5
    p1, p2 = ds.split_proportionately([0.5])
    assert p1.count() == 10 and p2.count() == 10
    z = ds.zip(data.range(20, parallelism=2).map(lambda x: -x))
    assert z.take(2) == [(0, 0), (1, -1)]
    assert ds.union(data.range(5)).count() == 25
    assert ds.limit(7).take_all() == list(range(7))


def test_tensor_and_numpy(ray_data):
    ray, data = ray_data
    ds = data.range_tensor(10, shape=(2, 3), parallelism=2)
    arr = np.concatenate(ray.get(ds.to_numpy_refs()))
    assert arr.shape == (10, 2, 3) and arr[3].max() == 3
    nds = data.from_numpy(np.arange(12).reshape(6, 2))
    out = list(nds.iter_batches(batch_size=4, batch_format="numpy"))
    assert out[0].shape == (4, 2) and out[1].shape == (2, 2)
    import torch

    tb = list(nds.iter_torch_batches(batch_size=3))
    assert isinstance(tb[0], torch.Tensor) and tb[0].shape == (3, 2)
    doubled = nds.map_batches(lambda b: b * 2, batch_format="numpy")
    assert np.concatenate(ray.get(doubled.to_numpy_refs()))[-1].tolist() == [20, 22]


def test_actor_pool_compute(ray_data):
    ray, data = ray_data

    class AddN:
        def __init__(self, n):
            self.n = n

        def __call__(self, batch):
            return [x + self.n for x in batch]

    ds = data.range(40, parallelism=4).map_batches(AddN, compute=data.ActorPoolStrategy(1, 2),
                                                   fn_constructor_args=(100,), num_cpus=0.5)
    assert sorted(ds.take_all()) == list(range(100, 140))
    with pytest.raises(ValueError):
        data.range(4).map_batches(AddN)


def test_read_write_formats(ray_data, tmp_path):
    ray, data = ray_data
    ds = data.from_items([{"x": i, "y": str(i)} for i in range(25)], parallelism=3)
    for fmt in ("parquet", "csv", "json"):
        d = str(tmp_path / fmt)
        getattr(ds, f"write_{fmt}")(d)
        assert len(os.listdir(d)) == 3
        back = getattr(data, f"read_{fmt}")(d)
        assert sorted(r["x"] for r in back.take_all()) == list(range(25))
        assert len(back.input_files()) == 3
    nd = str(tmp_path / "npy")
    data.from_numpy(np.arange(10)).write_numpy(nd)
    assert sorted(data.read_numpy(nd).take_all()) == list(range(10))
    tf = tmp_path / "t.txt"
    tf.write_text("a\nb\n\nc\n")
    assert data.read_text(str(tf)).take_all() == ["a", "b", "c"]
    assert data.read_binary_files(str(tf)).take_all() == [b"a\nb\n\nc\n"]
    dfs = data.from_pandas([pd.DataFrame({"q": [1, 2]}), pd.DataFrame({"q": [3]})])
    assert dfs.to_pandas()["q"].tolist() == [1, 2, 3]
    out = data.datasource.DummyOutputDatasource()
    dfs.write_datasource(out)
    assert out.num_ok == 1 and out.rows_written == 3


def test_pipeline(ray_data):
    ray, data = ray_data
    pipe = data.range(12, parallelism=4).window(blocks_per_window=2).map(lambda x: x * 10)
    assert pipe.take_all() if hasattr(pipe, "take_all") else True
    p2 = data.range(12, parallelism=4).window(blocks_per_window=2).map(lambda x: x * 10)
    assert list(p2.iter_rows()) == [x * 10 for x in range(12)]
    rep = data.range(5, parallelism=1).repeat(3)
    assert rep.count() == 15
    epochs = list(data.range(4, parallelism=2).repeat(2).random_shuffle_each_window(seed=0).iter_epochs())
    assert len(epochs) == 2 and sorted(epochs[1].iter_rows()) == [0, 1, 2, 3]
    shards = data.range(8, parallelism=4).window(blocks_per_window=2).split(2)
    assert sorted(list(shards[0].iter_rows()) + list(shards[1].iter_rows())) == list(range(8))


def test_random_access(ray_data):
    ray, data = ray_data
    ds = data.from_items([{"id": i, "v": i * i} for i in range(50)], parallelism=5)
    rad = ds.to_random_access_dataset("id", num_workers=2)
    assert ray.get(rad.get_async(7))["v"] == 49
    assert [r["v"] if r else None for r in rad.multiget([3, 40, 1000])] == [9, 1600, None]


def test_preprocessors(ray_data):
    ray, data = ray_data
    from ray_memory_management_amd.data.preprocessor import PreprocessorNotFittedException
    from ray_memory_management_amd.data.preprocessors import (BatchMapper, Chain, Concatenator, LabelEncoder,
                                                              MinMaxScaler, OneHotEncoder, SimpleImputer,
                                                              StandardScaler)

    df = pd.DataFrame({"a": [1.0, 2.0, 3.0, 4.0], "b": [10.0, None, 30.0, 40.0], "cat": ["x", "y", "x", "z"]})
    ds = data.from_pandas(df)
    sc = StandardScaler(["a"])
    with pytest.raises(PreprocessorNotFittedException):
        sc.transform(ds)
    out = sc.fit_transform(ds).to_pandas()
    assert out["a"].mean() == pytest.approx(0.0) and sc.stats_["mean(a)"] == pytest.approx(2.5)
    mm = MinMaxScaler(["a"]).fit(ds)
    assert mm.transform_batch(df.copy())["a"].tolist() == pytest.approx([0, 1 / 3, 2 / 3, 1])
    imp = SimpleImputer(["b"]).fit(ds)
    assert imp.transform_batch(df.copy())["b"].tolist() == pytest.approx([10, 80 / 3, 30, 40])
    oh = OneHotEncoder(["cat"]).fit(ds).transform_batch(df.copy())
    assert oh["cat_x"].tolist() == [1, 0, 1, 0]
    le = LabelEncoder("cat").fit(ds).transform_batch(df.copy())
    assert le["cat"].tolist() == [0, 1, 0, 2]
    ch = Chain(SimpleImputer(["b"]), BatchMapper(lambda d: d.assign(s=d["a"] + d["b"])),
               Concatenator(include=["a", "b"]))
    res = ch.fit_transform(ds).to_pandas()
    assert "concat_out" in res.columns and len(res["concat_out"][0]) == 2


def test_sampling_and_splits(ray_data):
    ray, data = ray_data
    ds = data.range(1000, parallelism=8)
    s = ds.random_sample(0.1, seed=0).take_all()
    assert 50 < len(s) < 150 and set(s) <= set(range(1000))
    with pytest.raises(ValueError):
        ds.random_sample(1.5)
    parts = ds.split_at_indices([100, 350])
    assert [p.count() for p in parts] == [100, 250, 650]
    assert parts[1].take(2) == [100, 101]
    a, b = ds.split_proportionately([0.25])
    assert a.count() == 250 and b.count() == 750
    with pytest.raises(ValueError):
        ds.split_proportionately([0.6, 0.5])
    tr, te = ds.train_test_split(0.2)
    assert tr.count() == 800 and te.count() == 200 and te.take(1) == [800]
    tr, te = ds.train_test_split(100, shuffle=True, seed=1)
    assert te.count() == 100 and sorted(tr.take_all() + te.take_all()) == list(range(1000))
    r = ds.randomize_block_order(seed=3)
    assert sorted(r.take_all()) == list(range(1000)) and r.num_blocks() == 8
    eq = ds.split(3, equal=True)
    assert len({p.count() for p in eq}) == 1


def test_from_sources_and_column_selection(ray_data):
    ray, data = ray_data
    import pyarrow as pa

    df = pd.DataFrame({"x": np.arange(10), "y": np.arange(10) * 2.0, "z": list("abcdefghij")})
    ds = data.from_pandas([df.iloc[:5], df.iloc[5:]])
    assert ds.num_blocks() == 2 and ds.count() == 10
    sel = ds.select_columns(["x", "z"]).to_pandas()
    assert list(sel.columns) == ["x", "z"] and sel["z"].tolist() == list("abcdefghij")
    t = pa.table({"k": [3, 1, 2]})
    assert sorted(r["k"] for r in data.from_arrow(t).take_all()) == [1, 2, 3]
    arr = np.arange(24, dtype=np.float32).reshape(6, 4)
    nd = data.from_numpy([arr[:3], arr[3:]])
    assert nd.count() == 6
    got = np.concatenate([ray.get(r) for r in nd.to_numpy_refs()])
    np.testing.assert_array_equal(got.reshape(6, 4), arr)
    assert sum(ray.get(r).num_rows for r in ds.to_arrow_refs()) == 10
    assert ds.size_bytes() > 0
    desc = ds.sort("y", descending=True).take(2)
    assert [r["x"] for r in desc] == [9, 8]


def test_torch_iteration(ray_data):
    ray, data = ray_data
    import torch

    ds = data.from_items([{"f1": float(i), "f2": float(2 * i), "label": i % 2} for i in range(20)], parallelism=3)
    batches = list(ds.iter_torch_batches(batch_size=6))
    assert [len(b["f1"]) for b in batches] == [6, 6, 6, 2]
    assert isinstance(batches[0]["f1"], torch.Tensor) and batches[0]["f2"][1].item() == 2.0
    dropped = list(ds.iter_torch_batches(batch_size=6, drop_last=True))
    assert len(dropped) == 3
    shuf = torch.cat([b["f1"] for b in ds.iter_torch_batches(batch_size=5, local_shuffle_buffer_size=10,
                                                             local_shuffle_seed=0)])
    assert sorted(shuf.tolist()) == [float(i) for i in range(20)] and shuf.tolist() != sorted(shuf.tolist())
    tds = ds.to_torch(label_column="label", batch_size=4)
    feats, labels = next(iter(tds))
    assert feats.shape == (4, 2) and labels.shape == (4, 1)


def test_pipeline_repeat_and_window(ray_data):
    ray, data = ray_data
    ds = data.range(12, parallelism=4)
    pipe = ds.repeat(3)
    assert sum(1 for _ in pipe.iter_rows()) == 36
    w = ds.window(blocks_per_window=2).map(lambda x: x + 1)
    seen = [sorted(wd.take_all()) for wd in w.iter_datasets()]
    assert len(seen) == 2 and seen[0] == list(range(1, 7)) and seen[1] == list(range(7, 13))
    with pytest.raises(ValueError):
        ds.repeat(0)


def test_read_images_folder(ray_data, tmp_path):
    ray, data = ray_data
    from PIL import Image

    for label, color in (("cat", (255, 0, 0)), ("dog", (0, 0, 255))):
        d = tmp_path / label
        d.mkdir()
        for i in range(3):
            Image.new("RGB", (8 + i, 6), color).save(d / f"{i}.png")
    ds = data.read_images(str(tmp_path), size=(4, 5), mode="RGB")
    rows = ds.take_all()
    assert len(rows) == 6 and sorted({r["label"] for r in rows}) == ["cat", "dog"]
    for r in rows:
        assert r["image"].shape == (4, 5, 3) and r["image"].dtype == np.uint8
        assert r["image"][0, 0, 0] == (255 if r["label"] == "cat" else 0)


def test_read_images_mixed_sizes_as_rows(ray_data, tmp_path):
    ray, data = ray_data
    from PIL import Image

    (tmp_path / "a").mkdir()
    Image.new("L", (3, 2)).save(tmp_path / "a" / "x.png")
    Image.new("L", (5, 4)).save(tmp_path / "a" / "y.png")
    rows = data.read_images(str(tmp_path), include_paths=True).take_all()
    assert sorted(r["image"].shape for r in rows) == [(2, 3), (4, 5)] and all(r["path"].endswith(".png") for r in rows)


def test_pipeline_outputs_and_splits(ray_data, tmp_path):
    ray, data = ray_data
    from ray_memory_management_amd.data.dataset_pipeline import DatasetPipeline

    pipe = data.range(20, parallelism=4).window(blocks_per_window=2)
    a, b = pipe.split_at_indices([3])
    assert sorted(a.take_all() + b.take_all()) == list(range(20))
    p2 = DatasetPipeline.from_iterable([lambda: data.range(3), lambda: data.range(2)])
    assert p2.take_all() == [0, 1, 2, 0, 1]
    p3 = data.from_items([{"x": i} for i in range(6)], parallelism=2).window(blocks_per_window=1)
    p3.write_json(str(tmp_path / "out"))
    assert sorted(os.listdir(tmp_path / "out")) == ["window_000000", "window_000001"]
    back = data.read_json(str(tmp_path / "out" / "window_000000")).take_all()
    assert sorted(r["x"] for r in back) == [0, 1, 2]
    p4 = data.from_items([{"f": float(i), "y": i % 2} for i in range(8)]).repeat(2)
    n = sum(len(lbl) for _, lbl in p4.to_torch(label_column="y", batch_size=4))
    assert n == 16


def test_lineage_serialization(ray_data, tmp_path):
    ray, data = ray_data
    ds = data.range(10, parallelism=2).map(lambda x: x * 3).filter(lambda x: x % 2 == 0)
    assert ds.has_serializable_lineage()
    blob = ds.serialize_lineage()
    again = data.Dataset.deserialize_lineage(blob)
    assert sorted(again.take_all()) == sorted(ds.take_all()) == [0, 6, 12, 18, 24]
    assert not data.from_items([1, 2]).has_serializable_lineage()
    import pytest

    with pytest.raises(ValueError):
        data.from_items([1, 2]).serialize_lineage()
