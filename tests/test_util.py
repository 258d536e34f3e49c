"""util: ActorPool, Queue, multiprocessing.Pool, metrics, iter, annotations, timer.
Mirrors reference python/ray/tests/{test_actor_pool,test_queue,test_multiprocessing,test_metrics,
test_iter}.py at smaller scale."""
import asyncio
import time

import pytest


# ---------------------------------------------------------------------- ActorPool
def test_actor_pool_map_ordered_and_unordered(ray_shared):
    ray = ray_shared
    from ray_memory_management_amd.util import ActorPool

    @ray.remote
    class Doubler:
        def double(self, v):
            time.sleep(0.01 * (v % 3))
            return 2 * v

    pool = ActorPool([Doubler.remote() for _ in range(3)])
    assert list(pool.map(lambda a, v: a.double.remote(v), range(10))) == [2 * i for i in range(10)]
    assert sorted(pool.map_unordered(lambda a, v: a.double.remote(v), range(10))) == [2 * i for i in range(10)]
    # submit/get_next with more work than actors queues the overflow
    for i in range(7):
        pool.submit(lambda a, v: a.double.remote(v), i)
    assert [pool.get_next() for _ in range(7)] == [2 * i for i in range(7)]
    assert not pool.has_next()
    a = pool.pop_idle()
    assert a is not None and pool.has_free()
    pool.push(a)
    with pytest.raises(ValueError):
        pool.push(a)


def test_actor_pool_get_next_timeout(ray_shared):
    ray = ray_shared
    from ray_memory_management_amd.util import ActorPool

    @ray.remote
    class Slow:
        def f(self, v):
            time.sleep(2)
            return v

    pool = ActorPool([Slow.remote()])
    pool.submit(lambda a, v: a.f.remote(v), 1)
    with pytest.raises(TimeoutError):
        pool.get_next(timeout=0.05)
    assert pool.get_next() == 1


# ---------------------------------------------------------------------- Queue
def test_queue_basic(ray_shared):
    from ray_memory_management_amd.util.queue import Empty, Full, Queue

    q = Queue(maxsize=3)
    assert q.empty() and q.size() == 0
    q.put(1)
    q.put_nowait_batch([2, 3])
    assert q.full() and len(q) == 3
    with pytest.raises(Full):
        q.put(4, block=False)
    with pytest.raises(Full):
        q.put(4, timeout=0.05)
    assert q.get() == 1
    assert q.get_nowait_batch(2) == [2, 3]
    with pytest.raises(Empty):
        q.get(block=False)
    with pytest.raises(Empty):
        q.get(timeout=0.05)
    q.shutdown()


def test_queue_producer_consumer_across_tasks(ray_shared):
    ray = ray_shared
    from ray_memory_management_amd.util.queue import Queue

    q = Queue()

    @ray.remote
    def producer(q, n):
        for i in range(n):
            q.put(i)
        return n

    @ray.remote
    def consumer(q, n):
        return [q.get(timeout=20) for _ in range(n)]

    c = consumer.remote(q, 20)
    ray.get(producer.remote(q, 20))
    assert ray.get(c) == list(range(20))

    async def use_async():
        await q.put_async(5)
        return await q.get_async()

    assert asyncio.run(use_async()) == 5


# ---------------------------------------------------------------------- multiprocessing.Pool
def _sq(x):
    return x * x


def _add(a, b):
    return a + b


def _boom(x):
    if x == 3:
        raise ValueError("bad item")
    return x


_INIT = {}


def _init(v):
    _INIT["v"] = v


def _get_init(_):
    return _INIT.get("v")


def test_multiprocessing_pool(ray_shared):
    from ray_memory_management_amd.util.multiprocessing import Pool

    with Pool(processes=2, initializer=_init, initargs=(42,)) as pool:
        assert pool.map(_sq, range(20)) == [i * i for i in range(20)]
        assert pool.map(_sq, range(20), chunksize=7) == [i * i for i in range(20)]
        assert pool.starmap(_add, [(1, 2), (3, 4)]) == [3, 7]
        assert pool.apply(_add, (5, 6)) == 11
        r = pool.apply_async(_sq, (9,))
        assert r.get(timeout=30) == 81 and r.ready() and r.successful()
        assert list(pool.imap(_sq, range(6))) == [0, 1, 4, 9, 16, 25]
        assert sorted(pool.imap_unordered(_sq, range(6))) == [0, 1, 4, 9, 16, 25]
        assert set(pool.map(_get_init, range(4))) == {42}
        with pytest.raises(ValueError):
            pool.map(_boom, range(5))
        got = []
        pool.map_async(_sq, [2, 3], callback=got.append).wait(30)
        time.sleep(0.1)
        assert got == [[4, 9]]


def test_multiprocessing_pool_maxtasksperchild(ray_shared):
    import os

    from ray_memory_management_amd.util.multiprocessing import Pool

    pool = Pool(processes=1, maxtasksperchild=2)
    pids = pool.map(lambda _: os.getpid(), range(6), chunksize=1)
    assert len(set(pids)) >= 2  # the worker actor was replaced after 2 tasks
    pool.terminate()


# ---------------------------------------------------------------------- metrics
def test_metrics_validation():
    from ray_memory_management_amd.util.metrics import Counter, Gauge, Histogram

    with pytest.raises(ValueError):
        Counter("")
    with pytest.raises(TypeError):
        Counter("c1", tag_keys=["a"])
    c = Counter("c_valid", tag_keys=("route",))
    with pytest.raises(ValueError):
        c.inc(1.0)  # missing tag
    with pytest.raises(ValueError):
        c.inc(1.0, {"other": "x"})
    with pytest.raises(ValueError):
        Histogram("h_nob", boundaries=[])
    g = Gauge("g_valid")
    g.set(3.0)


def test_metrics_collect_across_processes(ray_shared):
    ray = ray_shared
    from ray_memory_management_amd.util import metrics

    @ray.remote
    def work(i):
        from ray_memory_management_amd.util.metrics import Counter, Histogram

        c = Counter("requests_total", "reqs", tag_keys=("kind",))
        c.inc(2.0, {"kind": "a"})
        h = Histogram("latency_s", "lat", boundaries=[0.1, 1.0])
        h.observe(0.5)
        from ray_memory_management_amd.util import metrics as m

        m.flush()
        return i

    ray.get([work.remote(i) for i in range(3)])
    c = metrics.Counter("requests_total", "reqs", tag_keys=("kind",))
    c.set_default_tags({"kind": "b"})
    c.inc(1.0)
    metrics.flush()
    got = metrics.collect()
    series = got["requests_total"]["series"]
    assert series[(("kind", "b"),)] == 1.0
    assert series[(("kind", "a"),)] >= 2.0  # summed over the worker processes that ran it
    text = metrics.prometheus_text()
    assert "# TYPE requests_total counter" in text and "latency_s_bucket" in text
    srv, port = metrics.start_http_exporter()
    import urllib.request

    body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=10).read().decode()
    assert "requests_total" in body
    srv.shutdown()


# ---------------------------------------------------------------------- iter
def test_parallel_iterator(ray_shared):
    from ray_memory_management_amd.util import iter as pi

    it = pi.from_range(12, num_shards=3)
    assert it.num_shards() == 3
    assert sorted(it.gather_sync()) == list(range(12))
    assert list(it.for_each(lambda x: x * 2).filter(lambda x: x % 4 == 0).gather_sync()) == \
        [0, 8, 16, 4, 12, 20]
    assert sorted(it.gather_async()) == list(range(12))
    b = list(it.batch(2).gather_sync())
    assert all(len(x) == 2 for x in b) and sorted(y for x in b for y in x) == list(range(12))
    assert sorted(it.batch(2).flatten().gather_sync()) == list(range(12))
    assert list(it.get_shard(1)) == [4, 5, 6, 7]
    assert list(it.batch_across_shards())[0] == [0, 4, 8]
    u = it.union(pi.from_items([100, 101], num_shards=1))
    assert u.num_shards() == 4 and sorted(u.gather_sync())[-2:] == [100, 101]
    assert sorted(it.repartition(2).gather_sync()) == list(range(12))
    assert it.take(3) == [0, 4, 8]
    rep = pi.from_items([1, 2], num_shards=1, repeat=True)
    assert rep.take(5) == [1, 2, 1, 2, 1]
    sh = sorted(it.local_shuffle(3, seed=0).gather_sync())
    assert sh == list(range(12))


def test_local_iterator_ops():
    from ray_memory_management_amd.util.iter import LocalIterator

    it = LocalIterator(lambda: iter(range(10)))
    assert it.for_each(lambda x: x + 1).filter(lambda x: x % 2).take(3) == [1, 3, 5]
    a, b = LocalIterator(lambda: iter(range(4))).duplicate(2)
    assert list(a) == [0, 1, 2, 3] and list(b) == [0, 1, 2, 3]
    u = LocalIterator(lambda: iter([1, 2, 3])).union(LocalIterator(lambda: iter([10, 20])))
    assert list(u) == [1, 10, 2, 20, 3]
    assert sorted(LocalIterator(lambda: iter(range(8))).shuffle(4, seed=1)) == list(range(8))
    assert list(LocalIterator(lambda: iter(range(5))).batch(2)) == [[0, 1], [2, 3], [4]]


# ---------------------------------------------------------------------- annotations / timer
def test_annotations_and_timer():
    import warnings

    from ray_memory_management_amd.util.annotations import Deprecated, DeveloperAPI, PublicAPI
    from ray_memory_management_amd.util.timer import _Timer

    @PublicAPI(stability="beta")
    def f():
        """doc"""
        return 1

    @DeveloperAPI
    class C:
        pass

    @Deprecated(message="use g")
    def old():
        return 2

    assert "PublicAPI (beta)" in f.__doc__ and f() == 1 and C._annotated == "DeveloperAPI"
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert old() == 2
        assert any(issubclass(x.category, DeprecationWarning) for x in w)
    t = _Timer()
    with t:
        time.sleep(0.01)
    t.push_units_processed(10)
    assert t.count == 1 and t.mean > 0.005 and t.mean_throughput > 0


def test_joblib_ray_backend(ray_shared):
    """Reference util/joblib tests: Parallel over the ray backend returns in order."""
    import joblib

    from ray_memory_management_amd.util.joblib import register_ray

    register_ray()
    with joblib.parallel_backend("ray"):
        out = joblib.Parallel(n_jobs=2)(joblib.delayed(pow)(i, 2) for i in range(20))
    assert out == [i * i for i in range(20)]


def test_actor_group(ray_shared):
    """Reference util/tests/test_actor_group.py: group method calls, execute, execute_single."""
    from ray_memory_management_amd.util.actor_group import ActorGroup

    class Counter:
        def __init__(self, start):
            self.v = start

        def inc(self, k=1):
            self.v += k
            return self.v

    g = ActorGroup(Counter, num_actors=3, num_cpus_per_actor=0.1, init_args=(10,))
    assert len(g) == 3
    assert ray_shared.get(g.inc.remote(5)) == [15, 15, 15]
    assert g.execute(lambda a, m: a.v * m, 2) == [30, 30, 30]
    assert g.execute_single(1, lambda a: a.inc()) == 16
    assert ray_shared.get(g[1].inc.remote()) == 17
    with pytest.raises(AttributeError):
        g.nope
    g.shutdown()
    assert len(g) == 0


def test_state_get_by_id_logs_and_runtime_envs(ray_start):
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.util import state

    @ray.remote
    class A:
        def hello(self):
            print("hello-from-actor", flush=True)
            return 1

    a = A.options(runtime_env={"env_vars": {"X": "1"}}).remote()
    assert ray.get(a.hello.remote()) == 1
    aid = a._actor_id.hex()
    assert state.get_actor(aid)["actor_id"] == aid
    nodes = state.list_nodes()
    assert state.get_node(nodes[0]["NodeID"]) is not None
    w = [x for x in state.list_workers() if x["actor_id"] == aid][0]
    assert state.get_worker(w["worker_id"])["pid"] == w["pid"]
    logs = state.list_logs()
    assert any(f.startswith("worker-") for fs in logs.values() for f in fs)
    import time

    deadline = time.time() + 10
    found = False
    while time.time() < deadline and not found:
        found = any("hello-from-actor" in line for line in state.get_log(actor_id=aid))
        time.sleep(0.1)
    assert found
    envs = state.list_runtime_envs()
    assert any(e["runtime_env"].get("env_vars") == {"X": "1"} for e in envs)
    with state.warnings_on_slow_request(address="", endpoint="x", timeout=10, explain=True):
        pass
