"""Core microbenchmarks (`rmm microbenchmark`). Parity: reference python/ray/_private/ray_perf.py
(same metric names as release_logs/*/microbenchmark.json so results compare line by line with
BASELINE.md). Each metric runs for ~`duration` seconds after a warm-up and reports ops/s (or
GB/s for the *_gigabytes rows)."""
from __future__ import annotations

import json
import os
import time
from typing import Callable, Dict, List

import numpy as np

import ray_memory_management_amd as ray

BASELINE = {  # reference release_logs/2.0.0/microbenchmark.json (other hardware)
    "single_client_get_calls_Plasma_Store": 5403, "single_client_put_calls_Plasma_Store": 5390,
    "multi_client_put_calls_Plasma_Store": 10955, "single_client_put_gigabytes": 19.67,
    "single_client_tasks_and_get_batch": 10.4, "multi_client_put_gigabytes": 34.63,
    "single_client_get_object_containing_10k_refs": 12.87, "single_client_tasks_sync": 1424,
    "single_client_tasks_async": 13150, "multi_client_tasks_async": 35467, "1_1_actor_calls_sync": 2490,
    "1_1_actor_calls_async": 6146, "1_1_actor_calls_concurrent": 5324, "1_n_actor_calls_async": 11848,
    "n_n_actor_calls_async": 34777, "n_n_actor_calls_with_arg_async": 3346, "1_1_async_actor_calls_sync": 1516,
    "1_1_async_actor_calls_async": 3497, "1_1_async_actor_calls_with_args_async": 2422,
    "1_n_async_actor_calls_async": 10478, "n_n_async_actor_calls_async": 28553,
    "placement_group_create/removal": 1243,
}


def timeit(name: str, fn: Callable[[], None], multiplier: float = 1, duration: float = 2.0,
           warmup: float = 0.3) -> Dict[str, float]:
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warmup:
        fn()
    n = 0
    t0 = time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= duration:
            break
    rate = n * multiplier / dt
    key = name.replace(" ", "_").replace(":", "_").replace("(", "").replace(")", "").replace("-", "_")
    key = {"single_client_get_calls_Plasma_Store": "single_client_get_calls_Plasma_Store"}.get(key, key)
    return {"name": key, "value": rate, "baseline": BASELINE.get(key),
            "ratio": (rate / BASELINE[key]) if key in BASELINE else None}


@ray.remote
def _do_put():
    for _ in range(10):
        ray.put(np.zeros(10 * 1024 * 1024, dtype=np.int64))


@ray.remote
def _small_value():
    return b"ok"


@ray.remote
def _small_value_arg(x):
    return b"ok"


@ray.remote
def _small_value_batch(n):
    ray.get([_small_value.remote() for _ in range(n)])
    return 0


@ray.remote
class _Actor:
    def small_value(self):
        return b"ok"

    def small_value_arg(self, x):
        return b"ok"

    def small_value_batch(self, n):
        ray.get([_small_value.remote() for _ in range(n)])


@ray.remote
class _AsyncActor:
    async def small_value(self):
        return b"ok"

    async def small_value_with_arg(self, x):
        return b"ok"


@ray.remote
class _Client:
    def __init__(self, servers):
        self.servers = servers if isinstance(servers, list) else [servers]

    def small_value_batch(self, n):
        results = []
        for s in self.servers:
            results.extend([s.small_value.remote() for _ in range(n)])
        ray.get(results)

    def small_value_batch_arg(self, n):
        x = ray.put(0)
        results = []
        for s in self.servers:
            results.extend([s.small_value_arg.remote(x) for _ in range(n)])
        ray.get(results)

    def put_many(self, n, size):
        for _ in range(n):
            ray.put(np.zeros(size, dtype=np.uint8) if size else 0)

    def put_large(self, n, nbytes):
        arr = np.zeros(nbytes, dtype=np.int64)
        for _ in range(n):
            ray.put(arr)


def run(duration: float = 2.0, filter_pattern: str = "") -> List[dict]:
    if not ray.is_initialized():
        ray.init()
    res: List[dict] = []
    n_cpu = max(int(ray.cluster_resources().get("CPU", 4)), 2)

    def want(name):
        return filter_pattern in name

    def add(name, fn, mult=1):
        if want(name.replace(" ", "_")):
            r = timeit(name, fn, mult, duration)
            res.append(r)
            print(json.dumps(r), flush=True)

    value = ray.put(0)
    add("single client get calls (Plasma Store)", lambda: ray.get(value))
    add("single client put calls (Plasma Store)", lambda: ray.put(0))
    clients = [_Client.remote([]) for _ in range(min(4, n_cpu))]
    add("multi client put calls (Plasma Store)", lambda: ray.get([c.put_many.remote(1000, 0) for c in clients]),
        1000 * len(clients))
    arr = np.zeros(100 * 1024 * 1024, dtype=np.int64)  # 800 MB per put (reference: 8 x 0.1 GB)
    add("single client put gigabytes", lambda: ray.put(arr), 8 * 0.1)
    # reference ray_perf.py:139-146: 10 tasks x 10 puts of a fresh 80 MB np.zeros each
    add("multi client put gigabytes", lambda: ray.get([_do_put.remote() for _ in range(10)]), 10 * 8 * 0.1)
    add("single client tasks and get batch", lambda: ray.get([_small_value.remote() for _ in range(1000)]))
    add("single client tasks sync", lambda: ray.get(_small_value.remote()))
    add("single client tasks async", lambda: ray.get([_small_value.remote() for _ in range(1000)]), 1000)
    add("multi client tasks async", lambda: ray.get([_small_value_batch.remote(250) for _ in range(4)]), 1000)
    a = _Actor.remote()
    add("1:1 actor calls sync", lambda: ray.get(a.small_value.remote()))
    add("1:1 actor calls async", lambda: ray.get([a.small_value.remote() for _ in range(1000)]), 1000)
    ac = _Actor.options(max_concurrency=16).remote()
    add("1:1 actor calls concurrent", lambda: ray.get([ac.small_value.remote() for _ in range(1000)]), 1000)
    actors = [_Actor.remote() for _ in range(min(4, n_cpu))]
    add("1:n actor calls async", lambda: ray.get([x.small_value.remote() for x in actors for _ in range(250)]),
        250 * len(actors))
    servers = [_Actor.remote() for _ in range(min(2, n_cpu // 2))]
    cl = [_Client.remote(servers) for _ in range(min(2, n_cpu // 2))]
    add("n:n actor calls async", lambda: ray.get([c.small_value_batch.remote(250) for c in cl]),
        250 * len(servers) * len(cl))
    add("n:n actor calls with arg async", lambda: ray.get([c.small_value_batch_arg.remote(100) for c in cl]),
        100 * len(servers) * len(cl))
    aa = _AsyncActor.remote()
    add("1:1 async-actor calls sync", lambda: ray.get(aa.small_value.remote()))
    add("1:1 async-actor calls async", lambda: ray.get([aa.small_value.remote() for _ in range(1000)]), 1000)
    add("1:1 async-actor calls with args async",
        lambda: ray.get([aa.small_value_with_arg.remote(i) for i in range(1000)]), 1000)

    from ray_memory_management_amd.util.placement_group import placement_group, remove_placement_group

    def pg_cycle():
        pgs = [placement_group([{"CPU": 0.001}]) for _ in range(20)]
        for p in pgs:
            p.wait(10)
        for p in pgs:
            remove_placement_group(p)

    add("placement group create/removal", pg_cycle, 20)
    return res


def main(argv=None):
    import argparse

    p = argparse.ArgumentParser(prog="rmm microbenchmark")
    p.add_argument("--duration", type=float, default=2.0)
    p.add_argument("--filter", default="")
    p.add_argument("--out", default=None)
    a = p.parse_args(argv)
    res = run(a.duration, a.filter)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    main()
