"""Scalability envelope of the runtime on ONE node.

Parity: reference release/benchmarks/single_node/test_single_node.py:29-127 (10k task args, 3k
returns, 10k gets, 1M queued tasks, a 100 GB object) and release/benchmarks/distributed/
test_many_{actors,pgs,tasks}.py (actors / placement groups / concurrently running tasks per second).
Reference numbers: release/release_logs/2.0.0/scalability/single_node.json and
release_logs/2.0.0/benchmarks/many_{actors,pgs,tasks}.json (the distributed ones ran on a
multi-node cluster; here every count is scaled to one node and the scale is printed).

    python benchmarks/scalability.py [--queued 1000000] [--large-gb 16] [--actors 500] [--pgs 1000]

Prints one JSON object: per test the count, seconds, rate and the reference's value.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF_SINGLE_NODE = {"10000_args_time": 17.83, "3000_returns_time": 6.27, "10000_get_time": 26.83,
                   "1000000_queued_time": 178.33, "107374182400_large_object_time": 257.34}
REF_DISTRIBUTED = {"actors_per_second": 509.9, "pgs_per_second": 16.87, "tasks_per_second_10000": 27.6}


def _t(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def many_args(ray, n):
    @ray.remote
    def sum_args(*args):
        return sum(sum(a) for a in args)

    args = [[1] * 10000 for _ in range(n)]
    assert ray.get(sum_args.remote(*args)) == n * 10000


def many_returns(ray, n):
    @ray.remote(num_returns=n)
    def f():
        return tuple(list(range(10000)) for _ in range(n))

    refs = f.remote()
    assert len(refs) == n
    expected = list(range(10000))
    for r in refs:
        assert ray.get(r) == expected


def get_args(ray, n):
    import numpy as np

    refs = [ray.put(list(range(10000))) for _ in range(n)]
    res = ray.get(refs)
    assert len(res) == n and res[-1] == list(range(10000))
    refs = [ray.put(np.arange(10000)) for _ in range(n)]
    res = ray.get(refs)
    assert len(res) == n and (res[-1] == np.arange(10000)).all()


def many_queued(ray, n):
    from ray_memory_management_amd.util.queue import Queue  # noqa: F401  (API parity import)

    @ray.remote
    class Sema:
        def __init__(self):
            self.v = 0

        def release(self):
            self.v += 1

        def acquire(self):
            return self.v

    sema = Sema.remote()

    @ray.remote(num_cpus=1)
    def block(s):
        while ray.get(s.acquire.remote()) == 0:
            time.sleep(0.01)

    @ray.remote(num_cpus=1)
    def f():
        return None

    cpus = int(ray.cluster_resources()["CPU"])
    blocked = [block.remote(sema) for _ in range(cpus)]
    t0 = time.perf_counter()
    pending = [f.remote() for _ in range(n)]
    submit = time.perf_counter() - t0
    sema.release.remote()
    ray.get(blocked)
    chunk = 100000
    for i in range(0, n, chunk):
        assert all(x is None for x in ray.get(pending[i:i + chunk]))
    return submit


def large_object(ray, nbytes):
    import numpy as np

    obj = np.zeros(nbytes, dtype=np.int8)
    ref = ray.put(obj)
    del obj
    big = ray.get(ref)
    assert big[0] == 0 and big[-1] == 0
    del big, ref


def many_actors(ray, n):
    @ray.remote(num_cpus=0.01)
    class A:
        def foo(self):
            return None

    actors = [A.remote() for _ in range(n)]
    assert all(x is None for x in ray.get([a.foo.remote() for a in actors]))
    for a in actors:
        ray.kill(a)


def many_pgs(ray, n):
    from ray_memory_management_amd.util.placement_group import placement_group, remove_placement_group

    @ray.remote(num_cpus=0)
    class C:
        def ping(self):
            return "pong"

    pgs = [placement_group([{"CPU": 0.001}, {"CPU": 0.001}, {"CPU": 0.001}]) for _ in range(n)]
    for pg in pgs:
        ray.get(pg.ready())
    for pg in pgs:
        remove_placement_group(pg)


def many_running_tasks(ray, n, sleep_s):
    """Reference release/benchmarks/distributed/test_many_tasks.py: n sleeping tasks that must all run
    at once (one worker process each), rate = n / (wall time - sleep). The reference uses 0.25-CPU
    tasks on a 2,500-CPU cluster; on one node the tasks are 0-CPU so that n >> CPUs can run together.
    Peak concurrency comes from the tasks' own start / end times."""

    @ray.remote(num_cpus=0)
    def task():
        t0 = time.time()
        time.sleep(sleep_s)
        return t0, time.time()

    t0 = time.time()
    refs = [task.remote() for _ in range(n)]
    spans = ray.get(refs)
    wall = time.time() - t0
    edges = sorted([(a, 1) for a, _ in spans] + [(b, -1) for _, b in spans])
    cur = peak = 0
    for _, d in edges:
        cur += d
        peak = max(peak, cur)
    last_start = max(a for a, _ in spans) - t0
    return wall, {"peak_concurrent": peak, "all_started_after_s": round(last_start, 3), "sleep_s": sleep_s}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--args", type=int, default=10000)
    ap.add_argument("--returns", type=int, default=3000)
    ap.add_argument("--gets", type=int, default=10000)
    ap.add_argument("--queued", type=int, default=1_000_000)
    ap.add_argument("--large-gb", type=float, default=8.0)
    ap.add_argument("--actors", type=int, default=200)
    ap.add_argument("--pgs", type=int, default=1000)
    ap.add_argument("--tasks", type=int, default=1000, help="concurrently running 0-CPU sleep tasks")
    ap.add_argument("--task-sleep", type=float, default=20.0)
    ap.add_argument("--num-cpus", type=int, default=0)
    ap.add_argument("--only", default="")
    a = ap.parse_args()

    import ray_memory_management_amd as ray

    cpus = a.num_cpus or (os.cpu_count() or 8)
    store = int(max(a.large_gb * 1.2, 4.0) * (1 << 30))
    # one worker process per running task: raise the worker cap above the concurrent-task count
    ray.init(num_cpus=cpus, object_store_memory=store, _system_config={"max_workers": a.tasks + 64})
    only = set(a.only.split(",")) if a.only else None
    out = {"cpus": cpus, "object_store_bytes": store}

    def run(name, fn, count, ref=None, rate_unit=None):
        if only is not None and name not in only:
            return
        try:
            dt = fn()
            d = {"count": count, "seconds": round(dt, 3)}
            if rate_unit:
                d[rate_unit] = round(count / dt, 1)
            if ref is not None:
                d["reference"] = ref
        except Exception as e:  # noqa: BLE001 - report and keep going
            d = {"count": count, "error": repr(e)[:400]}
        out[name] = d
        print(f"[scalability] {name}: {d}", file=sys.stderr, flush=True)

    run("many_args", lambda: _t(lambda: many_args(ray, a.args)), a.args, REF_SINGLE_NODE["10000_args_time"])
    run("many_returns", lambda: _t(lambda: many_returns(ray, a.returns)), a.returns, REF_SINGLE_NODE["3000_returns_time"])
    run("ray_get_args", lambda: _t(lambda: get_args(ray, a.gets)), a.gets, REF_SINGLE_NODE["10000_get_time"])
    qs = {}

    def queued():
        t0 = time.perf_counter()
        qs["submit"] = many_queued(ray, a.queued)
        return time.perf_counter() - t0

    run("many_queued_tasks", queued, a.queued, REF_SINGLE_NODE["1000000_queued_time"], "tasks_per_s")
    if "many_queued_tasks" in out and "submit" in qs:
        out["many_queued_tasks"]["submit_seconds"] = round(qs["submit"], 3)
    nb = int(a.large_gb * (1 << 30))
    run("large_object", lambda: _t(lambda: large_object(ray, nb)), nb,
        {"bytes": 107374182400, "seconds": REF_SINGLE_NODE["107374182400_large_object_time"]})
    def fresh():
        # the reference runs each distributed benchmark (release/benchmarks/distributed/*) on its own
        # cluster; here a fresh head, so the single-node tests' cleanup (e.g. the ref-delta backlog of
        # a million finished tasks) does not run underneath
        ray.shutdown()
        ray.init(num_cpus=cpus, object_store_memory=1 << 30, _system_config={"max_workers": a.tasks + 64})

    fresh()
    run("many_actors", lambda: _t(lambda: many_actors(ray, a.actors)), a.actors, REF_DISTRIBUTED["actors_per_second"],
        "actors_per_s")
    fresh()
    run("many_pgs", lambda: _t(lambda: many_pgs(ray, a.pgs)), a.pgs, REF_DISTRIBUTED["pgs_per_second"], "pgs_per_s")
    fresh()
    nt = a.tasks
    extra = {}

    def running():
        wall, info = many_running_tasks(ray, nt, a.task_sleep)
        extra.update(info)
        return wall - a.task_sleep

    run("many_running_tasks", running, nt, REF_DISTRIBUTED["tasks_per_second_10000"], "tasks_per_s")
    if "many_running_tasks" in out:
        out["many_running_tasks"].update(extra)
    ray.shutdown()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
