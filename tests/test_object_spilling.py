"""Object spilling, ported from the reference's python/ray/tests/test_object_spilling.py, test_object_spilling_2.py
and test_object_spilling_3.py (the fork's focus). Same workloads, same checks on results, spill files and
`memory_summary(stats_only=True)`, with these changes:
- spill files live directly in the configured directory (`rmm-spill-*.bin`), with no per-session prefix directory;
- multi-node variants, S3 / smart_open storage and the unstable / slow mock filesystems are not ported (no
  network, and spilling is native here, not a Python IO-worker class that can be mocked);
- sizes are scaled down where the reference writes several GiB, so the suite stays inside this container's
  disk and memory.
"""
import json
import os
import random
import re
import subprocess
import sys
import time

import numpy as np
import pytest

import ray_memory_management_amd as ray
from ray_memory_management_amd._private.internal_api import memory_summary

MB = 1 << 20
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(d):
    return json.dumps({"type": "filesystem", "params": {"directory_path": str(d)}})


def _spill_files(d):
    return [f for f in os.listdir(d) if f.startswith("rmm-spill")] if os.path.isdir(d) else []


def _dir_empty(d):
    return not _spill_files(d)


def _wait(cond, timeout=30.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if cond():
            return True
        time.sleep(0.1)
    raise AssertionError("condition not met in time")


def _stats():
    s = memory_summary(stats_only=True)
    sp = re.search(r"Spilled (\d+) MiB, (\d+) objects", s)
    rs = re.search(r"Restored (\d+) MiB, (\d+) objects", s)
    return s, (int(sp.group(2)) if sp else 0), (int(rs.group(2)) if rs else 0)


@pytest.fixture
def spill_dir(tmp_path):
    d = tmp_path / "spill"
    d.mkdir()
    yield d
    if ray.is_initialized():
        ray.shutdown()


def _init(d, store=75 * MB, **sys_cfg):
    cfg = {"max_io_workers": 4, "automatic_object_spilling_enabled": True, "object_store_full_delay_ms": 100,
           "object_spilling_config": _cfg(d), "min_spilling_size": 0}
    cfg.update(sys_cfg)
    return ray.init(num_cpus=1, object_store_memory=store, _system_config=cfg)


def test_invalid_config_raises_exception(tmp_path):
    """Reference test_object_spilling.py:94: raised by ray.init before anything starts."""
    with pytest.raises(ValueError):
        ray.init(_system_config={"object_spilling_config": json.dumps({"type": "abc"})})
    good = {"type": "filesystem", "params": {"directory_path": str(tmp_path)}}
    with pytest.raises(Exception):
        bad = json.loads(json.dumps(good))
        bad["params"]["random_arg"] = "abc"
        ray.init(_system_config={"object_spilling_config": json.dumps(bad)})
    with pytest.raises(Exception):
        bad = json.loads(json.dumps(good))
        bad["params"]["buffer_size"] = "abc"
        ray.init(_system_config={"object_spilling_config": json.dumps(bad)})
    with pytest.raises(ValueError):  # cloud targets need the network
        ray.init(_system_config={"object_spilling_config": json.dumps(
            {"type": "smart_open", "params": {"uri": "s3://bucket/x"}})})
    assert not ray.is_initialized()


def test_default_config_and_disabled_spilling(tmp_path):
    """Reference test_object_spilling.py:137: the basic workload succeeds with the default config, and with
    spilling disabled (then through fallback allocation)."""
    def run_basic_workload():
        arr = np.random.rand(5 * MB)  # 40 MB
        refs = [ray.put(arr) for _ in range(2)]
        assert np.array_equal(ray.get(ray.put(arr)), arr)
        return refs

    ray.init(num_cpus=0, object_store_memory=75 * MB)
    try:
        run_basic_workload()
    finally:
        ray.shutdown()
    ray.init(num_cpus=0, object_store_memory=75 * MB,
             _system_config={"automatic_object_spilling_enabled": False, "object_store_full_delay_ms": 100})
    try:
        run_basic_workload()
        assert _stats()[1] == 0  # nothing spilled
    finally:
        ray.shutdown()


def test_spilling_not_done_for_pinned_object(spill_dir):
    """Reference test_object_spilling.py:220: two 40 MB puts into a 75 MB store, the first one read back with
    get(); nothing is written to the spill directory."""
    _init(spill_dir)
    arr = np.random.rand(5 * MB)  # 40 MB
    ref = ray.get(ray.put(arr))  # noqa: F841
    ref2 = ray.put(arr)  # noqa: F841
    _wait(lambda: _dir_empty(spill_dir))


def test_spill_objects_automatically(spill_dir):
    """Reference test_object_spilling.py:289 (100 objects of 8-24 MB through a 75 MB store, 1000 random
    non-blocking gets), scaled to 40 objects / 300 gets."""
    _init(spill_dir)
    rng = random.Random(0)
    refs, sols = [], []
    for _ in range(40):
        arr = np.random.rand(rng.choice([1, 2, 3]) * MB)
        refs.append(ray.put(arr))
        sols.append(arr)
    assert _spill_files(spill_dir)
    for _ in range(300):
        i = rng.randrange(len(refs))
        assert np.array_equal(ray.get(refs[i], timeout=0), sols[i])
    s, spilled, restored = _stats()
    assert spilled > 0 and restored > 0, s


def test_spill_stats(spill_dir):
    """Reference test_object_spilling.py:405: four 50 MB task returns through a 100 MB store, read back
    newest first, then one more."""
    _init(spill_dir, store=100 * MB, max_io_workers=100, min_spilling_size=1)

    @ray.remote
    def f():
        return np.zeros(50 * MB, dtype=np.uint8)

    ids = [f.remote() for _ in range(4)]
    while ids:
        assert ray.get(ids.pop()).nbytes == 50 * MB
    x_id = f.remote()
    ray.get(x_id)
    s = memory_summary(stats_only=True)
    assert "Plasma memory usage 50 MiB, 1 objects, 50.0% full" in s, s
    _, spilled, restored = _stats()
    # the reference spills all four first returns (200 MiB) and restores three; here a read of the object that
    # is still resident needs no restore, so at least three of the four are spilled and restored
    assert spilled >= 3 and restored >= 3, s


@pytest.mark.parametrize("is_async", [False, True])
def test_spill_during_get(spill_dir, is_async):
    """Reference test_object_spilling.py:456: ten 80 MB returns through a 100 MB store with one IO worker,
    read back while later ones are still being created; must finish well inside 30 s."""
    _init(spill_dir, store=100 * MB, max_io_workers=1)
    if is_async:
        @ray.remote(num_cpus=0)
        class Actor:
            async def f(self):
                return np.zeros(10 * MB)

        a = Actor.remote()
        ids = [a.f.remote() for _ in range(10)]
    else:
        @ray.remote(num_cpus=0)
        def f():
            return np.zeros(10 * MB)

        ids = [f.remote() for _ in range(10)]
    t0 = time.time()
    for x in ids:
        obj = ray.get(x)
        assert obj.shape == (10 * MB,)
        del obj
    assert time.time() - t0 < 30


def test_spill_worker_failure(spill_dir):
    """Reference test_object_spilling.py:524: 50 MB returns through a 75 MB store with one IO worker."""
    _init(spill_dir, max_io_workers=1)

    @ray.remote
    def f():
        return np.zeros(50 * MB, dtype=np.uint8)

    ids = [f.remote() for _ in range(5)]
    for i in ids:
        assert ray.get(i).nbytes == 50 * MB


def test_delete_objects(spill_dir):
    """Reference test_object_spilling_2.py:15: spill files are deleted once every object in them is freed."""
    _init(spill_dir, max_io_workers=1)
    arr = np.random.rand(MB)  # 8 MB
    buf = [ray.put(arr) for _ in range(40)]
    assert _spill_files(spill_dir)
    del buf
    _wait(lambda: _dir_empty(spill_dir))


def test_delete_objects_delete_while_creating(spill_dir):
    """Reference test_object_spilling_2.py:46: refs dropped at random while creating, random reads, then all
    spill files go away."""
    _init(spill_dir)
    rng = random.Random(1)
    arr = np.random.rand(MB)
    buf = []
    for _ in range(60):
        buf.append(ray.put(arr))
        if rng.randint(0, 9) < 6:
            buf.pop()
    for _ in range(100):
        assert np.array_equal(ray.get(rng.choice(buf), timeout=0), arr)
    del buf
    _wait(lambda: _dir_empty(spill_dir))


def test_delete_objects_on_worker_failure(spill_dir):
    """Reference test_object_spilling_2.py:86: objects owned by an actor that is SIGKILLed are freed, spill files
    included."""
    _init(spill_dir)

    @ray.remote
    class Actor:
        def __init__(self):
            self.buf = []

        def get_pid(self):
            return os.getpid()

        def create_objects(self):
            rng = random.Random(2)
            arr = np.random.rand(MB)
            for _ in range(60):
                self.buf.append(ray.put(arr))
                if rng.randint(0, 9) < 6:
                    self.buf.pop()
            for _ in range(100):
                assert np.array_equal(ray.get(rng.choice(self.buf), timeout=0), arr)
            return len(self.buf)

    a = Actor.remote()
    pid = ray.get(a.get_pid.remote())
    assert ray.get(a.create_objects.remote()) > 0
    assert _spill_files(spill_dir)
    os.kill(pid, 9)

    def dead():
        try:
            ray.get(a.get_pid.remote(), timeout=10)
        except ray.exceptions.RayActorError:
            return True
        return False

    _wait(dead)
    _wait(lambda: _dir_empty(spill_dir))


def test_fusion_objects(spill_dir):
    """Reference test_object_spilling_2.py:219: with min_spilling_size = 10 MB, small objects are fused so at
    least one spill file reaches that size."""
    _init(spill_dir, max_io_workers=3, min_spilling_size=10 * MB)
    rng = random.Random(3)
    refs, sols = [], []
    for _ in range(40):
        arr = np.random.rand(rng.choice([1, 2, 3]) * MB // 4)  # 2-6 MB
        refs.append(ray.put(arr))
        sols.append(arr)
    for _ in range(200):
        i = rng.randrange(len(refs))
        assert np.array_equal(ray.get(refs[i], timeout=0), sols[i])
    sizes = [os.path.getsize(os.path.join(spill_dir, f)) for f in _spill_files(spill_dir)]
    assert sizes and max(sizes) >= 10 * MB, sizes


def test_release_resource(spill_dir):
    """Reference test_object_spilling_2.py:272 (ray issue 12912): a task reading a spilled argument keeps its
    CPU; another task must not be scheduled onto it."""
    _init(spill_dir, max_io_workers=1)
    plasma_obj = ray.put(np.ones(50 * MB, dtype=np.uint8))
    for _ in range(5):
        ray.put(np.ones(50 * MB, dtype=np.uint8))  # forces the first one out

    @ray.remote
    def canary_task():
        return "resources were released!"

    @ray.remote
    def f(dep):
        t0 = time.time()
        while time.time() - t0 < 4:
            try:
                ray.get(dep[0], timeout=0.001)
            except ray.exceptions.GetTimeoutError:
                pass
        return True

    done = f.remote([plasma_obj])
    canary = canary_task.remote()
    ready, _ = ray.wait([canary], timeout=2)
    assert not ready
    assert ray.get(done) and ray.get(canary, timeout=30)


def test_file_deleted_when_driver_exits(tmp_path):
    """Reference test_object_spilling_2.py:366: a driver that dies on SIGINT while holding spilled objects leaves
    no spill files behind."""
    d = tmp_path / "spill"
    d.mkdir()
    driver = f"""
import json, os, signal
import numpy as np
import ray_memory_management_amd as ray
ray.init(object_store_memory=75 * 1024 * 1024, _system_config={{
    "max_io_workers": 2, "min_spilling_size": 0, "automatic_object_spilling_enabled": True,
    "object_store_full_delay_ms": 100,
    "object_spilling_config": json.dumps({{"type": "filesystem", "params": {{"directory_path": {str(d)!r}}}}})}})
arr = np.random.rand(1024 * 1024)
buf = [ray.put(arr) for _ in range(30)]
assert any(f.startswith("rmm-spill") for f in os.listdir({str(d)!r}))
os.kill(os.getpid(), signal.SIGINT)
"""
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", driver], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "AssertionError" not in r.stderr, r.stderr
    _wait(lambda: _dir_empty(d))


def test_multiple_directories(tmp_path):
    """Reference test_object_spilling_3.py:21: spills are distributed over every directory, and the files go
    away when the objects do."""
    dirs = []
    for i in range(3):
        p = tmp_path / f"spill_{i}"
        p.mkdir()
        dirs.append(p)
    ray.init(object_store_memory=75 * MB, _system_config={
        "max_io_workers": 5, "object_store_full_delay_ms": 100, "min_spilling_size": 0,
        "object_spilling_config": json.dumps({"type": "filesystem",
                                              "params": {"directory_path": [str(p) for p in dirs]}})})
    try:
        arr = np.ones(30 * MB, dtype=np.uint8)
        refs = [ray.put(arr) for _ in range(16)]
        counts = [len(_spill_files(p)) for p in dirs]
        for r in refs:
            assert np.array_equal(ray.get(r), arr)
        assert all(c >= 2 for c in counts), counts
        del r
        refs = []
        ray.put(arr)
        for p in dirs:
            _wait(lambda p=p: _dir_empty(p))
    finally:
        ray.shutdown()
    for p in dirs:  # and nothing is left once the session is gone
        assert _dir_empty(p)


@pytest.mark.parametrize("thres,min_spilled,max_spilled", [(None, 1, 9), (1.0, 0, 0), (0.1, 8, 10)])
def test_object_spilling_threshold(thres, min_spilled, max_spilled):
    """Reference test_object_spilling_3.py:103-130 (ten 200 MB objects in a 2.2 GB store), scaled 1/10: with
    the default threshold (0.8) some objects are spilled, with 1.0 none, with 0.1 nearly all."""
    ray.init(object_store_memory=220 * MB, _system_config={"object_spilling_threshold": thres} if thres else {})
    try:
        objs = [ray.put(np.empty(20 * MB, dtype=np.uint8)) for _ in range(10)]
        deadline = time.time() + 20
        while True:
            _, spilled, _ = _stats()
            if spilled >= min_spilled or time.time() > deadline:
                break
            time.sleep(0.2)
        if max_spilled == 0:
            time.sleep(1.0)  # give a (wrong) threshold spill time to show up
        _, spilled, _ = _stats()
        assert min_spilled <= spilled <= max_spilled, (thres, spilled)
        del objs
    finally:
        ray.shutdown()
