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


class _Collector:
    """A local OTLP/HTTP endpoint (what Tempo serves on :4318) recording every ExportTraceServiceRequest."""

    def __init__(self):
        import http.server
        import threading

        got = self.requests = []

        class H(http.server.BaseHTTPRequestHandler):
            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                got.append((self.path, self.headers.get("Content-Type"), json.loads(self.rfile.read(n))))
                self.send_response(200)
                self.end_headers()
                self.wfile.write(b"{}")

            def log_message(self, *a):
                pass

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}/v1/traces"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def spans(self):
        return [sp for _, _, req in self.requests for rs in req["resourceSpans"] for ss in rs["scopeSpans"]
                for sp in ss["spans"]]

    def close(self):
        self.srv.shutdown()


def test_tempo_exporter_posts_otlp_json(monkeypatch):
    """setup_tempo_tracing: spans leave as OTLP/HTTP JSON (trace / span ids in hex, kinds and status as
    the proto enums, int64 times as strings), batched by a background thread."""
    from ray_memory_management_amd.util.tracing import setup_tempo_tracing as tempo
    from ray_memory_management_amd.util.tracing import tracing_helper as th

    col = _Collector()
    monkeypatch.setenv("RMM_OTLP_ENDPOINT", col.url)
    monkeypatch.setenv("RMM_OTLP_CONSOLE", "0")
    try:
        tempo.setup_tracing()
        spec = {}
        th.inject(spec, "f", {"k": 3})
        with th.execution_span(spec, "f", {"ok": True}):
            pass
        tempo._installed.flush()
        spans = col.spans()
        assert col.requests[0][0] == "/v1/traces" and col.requests[0][1] == "application/json"
        res = col.requests[0][2]["resourceSpans"][0]["resource"]["attributes"]
        assert {"key": "service.name", "value": {"stringValue": "ray_memory_management_amd"}} in res
        prod = next(s for s in spans if s["kind"] == 4)
        cons = next(s for s in spans if s["kind"] == 5)
        assert cons["parentSpanId"] == prod["spanId"] and cons["traceId"] == prod["traceId"]
        assert len(prod["traceId"]) == 32 and len(prod["spanId"]) == 16
        assert int(cons["endTimeUnixNano"]) >= int(cons["startTimeUnixNano"]) > 0
        assert cons["status"] == {"code": 1}
        assert {"key": "k", "value": {"intValue": "3"}} in prod["attributes"]
        assert tempo._installed.sent == 2 and tempo._installed.dropped == 0
    finally:
        th.set_exporter(None)
        if tempo._installed is not None:
            tempo._installed.shutdown()
        col.close()


def test_tempo_exporter_across_processes(monkeypatch):
    """The tempo hook in a cluster: driver and worker processes post to the collector, and the worker's
    execution span hangs off the driver's submission span."""
    col = _Collector()
    monkeypatch.setenv("RMM_OTLP_ENDPOINT", col.url)
    monkeypatch.setenv("RMM_OTLP_CONSOLE", "0")
    monkeypatch.setenv("RMM_OTLP_FLUSH_S", "0.1")
    try:
        ray.init(num_cpus=1, _tracing_startup_hook="ray_memory_management_amd.util.tracing.setup_tempo_tracing:"
                                                   "setup_tracing")

        @ray.remote
        def g(x):
            return x * 3

        assert ray.get(g.remote(2)) == 6
        import time

        deadline = time.time() + 20
        while time.time() < deadline and not any(s["kind"] == 5 for s in col.spans()):
            time.sleep(0.1)
        ray.shutdown()
        from ray_memory_management_amd.util.tracing import setup_tempo_tracing as tempo

        if tempo._installed is not None:
            tempo._installed.flush()
        spans = col.spans()
        prod = [s for s in spans if s["kind"] == 4 and ".g ray.remote" in s["name"]]
        cons = [s for s in spans if s["kind"] == 5 and ".g ray.remote_worker" in s["name"]]
        assert prod and cons, [s["name"] for s in spans]
        assert cons[0]["parentSpanId"] == prod[0]["spanId"]
        pids = {a["value"]["intValue"] for _, _, req in col.requests for rs in req["resourceSpans"]
                for a in rs["resource"]["attributes"] if a["key"] == "process.pid"}
        assert len(pids) >= 2
    finally:
        ray.shutdown()
        from ray_memory_management_amd.util.tracing import tracing_helper as th

        th.set_exporter(None)
        col.close()
