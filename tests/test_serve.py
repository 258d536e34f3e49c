"""Serve: mirrors reference python/ray/serve/tests/{test_api,test_deploy,test_batching,
test_autoscaling_policy,test_http_routes,test_fastapi}.py at small scale."""
import asyncio
import time

import pytest
import requests


@pytest.fixture(scope="module")
def serve_inst(ray_shared):
    from ray_memory_management_amd import serve

    serve.start(http_options={"host": "127.0.0.1", "port": 0})
    yield ray_shared, serve
    serve.shutdown()


@pytest.fixture(autouse=True)
def _cleanup(serve_inst):
    """Replicas hold 1 CPU each: free them between tests (the shared cluster has 4 CPUs)."""
    yield
    ray, serve = serve_inst
    for name in list(serve.list_deployments()):
        serve.delete(name)


def test_function_and_class_deployments_via_handle(serve_inst):
    ray, serve = serve_inst

    @serve.deployment
    def hello(name):
        return f"hello {name}"

    @serve.deployment(num_replicas=2)
    class Counter:
        def __init__(self, start):
            self.n = start

        def __call__(self, x):
            self.n += x
            return self.n

        def ping(self):
            return serve.get_replica_context().deployment

    hello.deploy()
    h = hello.get_handle()
    assert ray.get(h.remote("x")) == "hello x"
    Counter.deploy(100)
    hc = Counter.get_handle()
    outs = ray.get([hc.remote(1) for _ in range(10)])
    assert all(o > 100 for o in outs)
    assert ray.get(hc.ping.remote()) == "Counter"
    assert set(serve.list_deployments()) >= {"hello", "Counter"}
    assert serve.status()["Counter"]["num_replicas"] == 2
    serve.delete("hello")
    assert "hello" not in serve.list_deployments()


def test_http_routes_and_requests(serve_inst):
    ray, serve = serve_inst
    port = serve.http_port()

    @serve.deployment(route_prefix="/echo")
    class Echo:
        async def __call__(self, request):
            body = await request.body()
            return {"path": request.url.path, "q": request.query_params.get("a"), "body": body.decode()}

    Echo.deploy()
    r = requests.post(f"http://127.0.0.1:{port}/echo/sub?a=7", data=b"payload", timeout=30)
    assert r.status_code == 200
    j = r.json()
    assert j["q"] == "7" and j["body"] == "payload" and j["path"].endswith("/sub")
    assert requests.get(f"http://127.0.0.1:{port}/nope", timeout=30).status_code == 404


def test_fastapi_ingress(serve_inst):
    ray, serve = serve_inst
    from fastapi import FastAPI

    app = FastAPI()

    @serve.deployment(route_prefix="/api")
    @serve.ingress(app)
    class Api:
        def __init__(self):
            self.k = 3

        @app.get("/mul/{x}")
        def mul(self, x: int):
            return {"y": x * self.k}

    Api.deploy()
    port = serve.http_port()
    r = requests.get(f"http://127.0.0.1:{port}/api/mul/5", timeout=30)
    assert r.status_code == 200 and r.json() == {"y": 15}


def test_batching(serve_inst):
    ray, serve = serve_inst

    @serve.deployment
    class Batcher:
        def __init__(self):
            self.sizes = []

        @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.2)
        async def handle(self, xs):
            self.sizes.append(len(xs))
            return [x * 2 for x in xs]

        async def __call__(self, x):
            return await self.handle(x)

        def sizes_seen(self):
            return self.sizes

    Batcher.deploy()
    h = Batcher.get_handle()
    assert sorted(ray.get([h.remote(i) for i in range(16)])) == [2 * i for i in range(16)]
    assert max(ray.get(h.sizes_seen.remote())) > 1


def test_user_config_and_versioned_redeploy(serve_inst):
    ray, serve = serve_inst

    @serve.deployment(user_config={"v": 1}, version="1")
    class Conf:
        def reconfigure(self, cfg):
            self.v = cfg["v"]

        def __call__(self):
            return self.v

    Conf.deploy()
    h = Conf.get_handle()
    assert ray.get(h.remote()) == 1
    Conf.options(user_config={"v": 2}).deploy()   # same version: reconfigure in place
    assert ray.get(h.remote()) == 2
    Conf.options(user_config={"v": 3}, version="2").deploy()  # new version: replicas replaced
    deadline = time.time() + 20
    while ray.get(h.remote()) != 3 and time.time() < deadline:
        time.sleep(0.1)
    assert ray.get(h.remote()) == 3


def test_deployment_graph_composition(serve_inst):
    ray, serve = serve_inst

    @serve.deployment
    class Adder:
        def __init__(self, inc):
            self.inc = inc

        def __call__(self, x):
            return x + self.inc

    @serve.deployment
    class Driver:
        def __init__(self, a, b):
            self.a, self.b = a, b

        async def __call__(self, x):
            y = await self.a.remote(x)
            return await self.b.remote(y)

    h = serve.run(Driver.bind(Adder.options(name="A1").bind(1), Adder.options(name="A2").bind(10)),
                  route_prefix=None)
    assert ray.get(h.remote(5)) == 16


def test_autoscaling_up_and_down(serve_inst):
    ray, serve = serve_inst

    @serve.deployment(autoscaling_config={"min_replicas": 1, "max_replicas": 3,
                                          "target_num_ongoing_requests_per_replica": 1, "upscale_delay_s": 0.2,
                                          "downscale_delay_s": 0.5, "look_back_period_s": 1.0},
                      max_concurrent_queries=10)
    class Slow:
        async def __call__(self):
            await asyncio.sleep(1.0)
            return 1

    Slow.deploy()
    h = Slow.get_handle()
    refs = [h.remote() for _ in range(12)]
    peak = 0
    deadline = time.time() + 20
    while time.time() < deadline:
        peak = max(peak, serve.status()["Slow"]["num_replicas"])
        if peak >= 2:
            break
        refs += [h.remote() for _ in range(4)]
        time.sleep(0.2)
    ray.get(refs)
    assert peak >= 2
    deadline = time.time() + 30
    while serve.status()["Slow"]["num_replicas"] > 1 and time.time() < deadline:
        time.sleep(0.2)
    assert serve.status()["Slow"]["num_replicas"] == 1


def test_route_prefix_validation_and_options():
    from ray_memory_management_amd import serve

    with pytest.raises(ValueError, match="start with"):
        serve.deployment(route_prefix="bad")(lambda x: x)
    with pytest.raises(ValueError, match="end with"):
        serve.deployment(route_prefix="/bad/")(lambda x: x)

    @serve.deployment(num_replicas=1)
    def f(x):
        return x

    g = f.options(name="g", num_replicas=3, route_prefix="/gg", ray_actor_options={"num_cpus": 0})
    assert g.name == "g" and g.num_replicas == 3 and g.route_prefix == "/gg" and f.num_replicas == 1
    assert g.ray_actor_options == {"num_cpus": 0}


def test_errors_propagate_and_replica_restart_after_crash(serve_inst):
    ray, serve = serve_inst
    import os

    @serve.deployment(ray_actor_options={"num_cpus": 0}, health_check_period_s=0.2, health_check_timeout_s=2)
    class Fragile:
        def __call__(self, x):
            if x == "boom":
                raise ValueError("bad input")
            return os.getpid()

        def die(self):
            os._exit(1)

    Fragile.deploy()
    h = Fragile.get_handle()
    pid0 = ray.get(h.remote(1))
    with pytest.raises(Exception, match="bad input"):
        ray.get(h.remote("boom"))
    assert ray.get(h.remote(2)) == pid0  # a user exception does not kill the replica
    h.die.remote()
    deadline = time.time() + 30
    pid1 = None
    while time.time() < deadline:
        try:
            pid1 = ray.get(h.remote(3), timeout=5)
            if pid1 != pid0:
                break
        except Exception:
            time.sleep(0.2)
    assert pid1 is not None and pid1 != pid0  # the controller replaced the dead replica
    assert serve.status()["Fragile"]["num_replicas"] == 1


def test_handle_method_options_and_async_methods(serve_inst):
    ray, serve = serve_inst

    @serve.deployment(ray_actor_options={"num_cpus": 0})
    class Model:
        def __init__(self):
            self.calls = 0

        async def predict(self, x):
            await asyncio.sleep(0.01)
            self.calls += 1
            return x * 2

        def count(self):
            return self.calls

    Model.deploy()
    h = Model.get_handle()
    hp = h.options(method_name="predict")
    assert ray.get([hp.remote(i) for i in range(8)]) == [i * 2 for i in range(8)]
    assert ray.get(h.count.remote()) == 8
    assert serve.get_deployment("Model").name == "Model"


def test_dag_driver_routes_and_adapters(serve_inst):
    ray, serve = serve_inst
    from ray_memory_management_amd.serve.drivers import DAGDriver
    from ray_memory_management_amd.serve.http_adapters import json_request, json_to_ndarray

    @serve.deployment(ray_actor_options={"num_cpus": 0})
    class Scale:
        def __init__(self, k):
            self.k = k

        def __call__(self, x):
            import numpy as np

            return (np.asarray(x) * self.k).tolist()

    app = DAGDriver.options(ray_actor_options={"num_cpus": 0}).bind(
        {"/double": Scale.options(name="S2").bind(2), "/triple": Scale.options(name="S3").bind(3)},
        http_adapter=json_request)
    h = serve.run(app, route_prefix="/dag")
    port = serve.http_port()
    r = requests.post(f"http://127.0.0.1:{port}/dag/double", json=[1, 2], timeout=30)
    assert r.status_code == 200 and r.json() == [2, 4]
    r = requests.post(f"http://127.0.0.1:{port}/dag/triple", json=[1], timeout=30)
    assert r.json() == [3]
    assert ray.get(h.predict_with_route.remote("/triple", [2])) == [6]
    serve.delete("DAGDriver")
    app2 = DAGDriver.options(name="D2", ray_actor_options={"num_cpus": 0}).bind(Scale.options(name="S4").bind(4),
                                                                                http_adapter=json_to_ndarray)
    serve.run(app2, route_prefix="/nd")
    r = requests.post(f"http://127.0.0.1:{port}/nd", json={"array": [1, 2, 3, 4], "shape": [2, 2]}, timeout=30)
    assert r.json() == [[4, 8], [12, 16]]


def test_predictor_deployment_serves_a_checkpoint(serve_inst):
    ray, serve = serve_inst
    import numpy as np
    import torch

    from ray_memory_management_amd.air.checkpoint import Checkpoint
    from ray_memory_management_amd.serve.air_integrations import PredictorDeployment
    from ray_memory_management_amd.train.predictor import TorchPredictor

    m = torch.nn.Linear(2, 1, bias=False)
    with torch.no_grad():
        m.weight.copy_(torch.tensor([[1.0, 2.0]]))
    ck = Checkpoint.from_dict({"model": m})
    app = PredictorDeployment.options(name="Lin", ray_actor_options={"num_cpus": 0}).bind(
        TorchPredictor, ck, batching_params={"max_batch_size": 4, "batch_wait_timeout_s": 0.05})
    serve.run(app, route_prefix="/lin")
    port = serve.http_port()
    r = requests.post(f"http://127.0.0.1:{port}/lin", json={"array": [[1.0, 1.0], [2.0, 0.5]]}, timeout=30)
    assert r.status_code == 200, r.text
    assert np.allclose(np.asarray(r.json()).reshape(-1), [3.0, 3.0])
