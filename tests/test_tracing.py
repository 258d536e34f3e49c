"""Distributed tracing (reference python/ray/tests/test_tracing.py): with a startup hook, task and
actor submissions produce PRODUCER spans in the driver and CONSUMER spans in the workers, linked by
trace id / parent span id; nested submissions stay in the same trace."""
import glob
import json
import os

import pytest

import ray_memory_management_amd as ray

HOOK = "ray_memory_management_amd.util.tracing.setup_local_tmp_tracing:setup_tracing"


@pytest.fixture
def span_dir(tmp_path, monkeypatch):
    d = str(tmp_path / "spans")
    monkeypatch.setenv("RMM_SPAN_DIR", d)
    import importlib

    import ray_memory_management_amd.util.tracing.setup_local_tmp_tracing as m

    importlib.reload(m)
    yield d
    ray.shutdown()


def _short(s):
    return s["name"].split(" ")[0].rsplit(".", 1)[-1]


def _spans(d):
    out = []
    for f in glob.glob(os.path.join(d, "*.json")):
        with open(f) as fh:
            out += [json.loads(l) for l in fh if l.strip()]
    return out


def test_task_and_actor_spans(span_dir):
    ray.init(num_cpus=2, _tracing_startup_hook=HOOK)

    @ray.remote
    def child(x):
        return x + 1

    @ray.remote
    def parent(x):
        return ray.get(child.remote(x)) * 2

    @ray.remote
    class Counter:
        def __init__(self):
            self.n = 0

        def inc(self):
            self.n += 1
            return self.n

    assert ray.get(parent.remote(1)) == 4
    c = Counter.remote()
    assert ray.get(c.inc.remote()) == 1
    ray.shutdown()

    spans = _spans(span_dir)
    by_id = {s["context"]["span_id"]: s for s in spans}
    prod = [s for s in spans if s["kind"] == "PRODUCER"]
    cons = [s for s in spans if s["kind"] == "CONSUMER"]
    names = {s["name"] for s in spans}
    assert any(".parent ray.remote" in n for n in names) and any(".parent ray.remote_worker" in n for n in names)
    assert any("inc" in n and n.endswith("ray.remote_worker") for n in names)
    for c_ in cons:  # every execution span hangs off its submission span, same trace
        p = by_id[c_["parent_id"]]
        assert p["kind"] == "PRODUCER" and p["context"]["trace_id"] == c_["context"]["trace_id"]
    # the nested child() submission is inside parent's execution span: one trace for both
    pc = next(s for s in cons if _short(s) == "parent")
    cp = next(s for s in prod if _short(s) == "child")
    assert cp["parent_id"] == pc["context"]["span_id"]
    assert cp["context"]["trace_id"] == pc["context"]["trace_id"]
    # spans come from more than one process (driver + workers)
    assert len({s["resource"]["process.pid"] for s in spans}) >= 2


def test_tracing_off_by_default(span_dir):
    ray.init(num_cpus=1)

    @ray.remote
    def f():
        return 1

    assert ray.get(f.remote()) == 1
    ray.shutdown()
    assert _spans(span_dir) == []
