"""Dashboard head: a small HTTP server in front of the cluster's state, metrics, memory and job
APIs.

Parity: reference dashboard/head.py + dashboard/modules/{state (state_head.py: /api/v0/{actors,
tasks,objects,nodes,workers,jobs,placement_groups} + summaries), node (/nodes),
reporter (/api/cluster_status, Prometheus metrics, per-GPU utilization / HBM and GPU object-store
occupancy + spill state: /api/gpus, dashboard/gpu_reporter.py), job (job_head.py: REST job submission
/api/jobs/ — submit / list / info / logs / stop / delete), log (/api/v0/logs),
healthz (/api/gcs_healthz), event (/events), snapshot (/api/snapshot, /api/actors/kill), actor
(/logical/actors, /logical/actor_groups, /logical/kill_actor), serve (/api/serve/deployments/) and
tune (/tune/info) — the last five in dashboard/modules.py}. The reference dashboard also ships a React UI; this one serves JSON
and Prometheus text only.

It runs as its own process that connects to the cluster as a client driver (like the reference's
dashboard process talks to GCS), so slow HTTP clients never stall the head's event loop. Request
handling is a thread per request (ThreadingHTTPServer); every handler is a read of the head's
state tables over the normal worker connection.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlparse

API_VERSION = "1"


def _filters(q: Dict[str, List[str]]):
    """?filter_keys=state&filter_predicates==&filter_values=ALIVE (reference state_head) or the
    shorthand ?state=ALIVE."""
    out = []
    keys, preds, vals = q.get("filter_keys", []), q.get("filter_predicates", []), q.get("filter_values", [])
    for i, k in enumerate(keys):
        out.append((k, preds[i] if i < len(preds) else "=", vals[i] if i < len(vals) else ""))
    for k, v in q.items():
        if k not in ("filter_keys", "filter_predicates", "filter_values", "limit", "detail", "timeout"):
            out.append((k, "=", v[0]))
    return out


class _Routes:
    def __init__(self):
        self.table: List[Tuple[str, "re.Pattern", Callable]] = []

    def add(self, method: str, pattern: str, fn: Callable):
        self.table.append((method, re.compile("^" + pattern + "$"), fn))

    def match(self, method: str, path: str):
        for m, rx, fn in self.table:
            if m == method:
                g = rx.match(path)
                if g:
                    return fn, g.groupdict()
        return None, None


class DashboardHead:
    def __init__(self, host: str = "127.0.0.1", port: int = 8265, session_dir: Optional[str] = None):
        self.host, self.port = host, port
        self.session_dir = session_dir
        self.started = time.time()
        self.routes = _Routes()
        self._jobs = None
        self._jobs_lock = threading.Lock()
        self._register()
        self.server: Optional[ThreadingHTTPServer] = None

    # ------------------------------------------------------------------ modules
    def _register(self):
        r = self.routes.add
        r("GET", r"/api/version", lambda q, b: {"version": API_VERSION, "ray_version": _version(),
                                                "session_dir": self.session_dir})
        r("GET", r"/api/gcs_healthz", lambda q, b: "success")
        r("GET", r"/api/cluster_status", self._cluster_status)
        r("GET", r"/nodes", lambda q, b: {"result": True, "data": {"summary": _w().nodes()}})
        # state module
        for kind in ("actors", "tasks", "objects", "nodes", "workers", "jobs", "placement_groups"):
            r("GET", rf"/api/v0/{kind}", self._lister(kind))
        r("GET", r"/api/v0/tasks/summarize", lambda q, b: _state().summarize_tasks())
        r("GET", r"/api/v0/actors/summarize", lambda q, b: _state().summarize_actors())
        r("GET", r"/api/v0/objects/summarize", lambda q, b: _state().summarize_objects())
        r("GET", r"/api/v0/timeline", lambda q, b: _w().timeline())
        # memory module (this fork's focus): store, pressure, GPU store
        r("GET", r"/api/memory/summary", lambda q, b: {"summary": _internal().memory_summary(
            stats_only=q.get("stats_only", ["0"])[0] in ("1", "true"))})
        r("GET", r"/api/memory/store", lambda q, b: _state().object_store_stats())
        r("GET", r"/api/memory/pressure", lambda q, b: _internal().memory_pressure_stats())
        r("GET", r"/api/memory/node", lambda q, b: _w()._state("memory"))
        # logs
        r("GET", r"/api/v0/logs", self._list_logs)
        r("GET", r"/api/v0/logs/file", self._log_file)
        # job module (REST; reference dashboard/modules/job/job_head.py)
        r("GET", r"/api/jobs/", lambda q, b: [self._job_json(i) for i in self._job_client().list_jobs()])
        r("POST", r"/api/jobs/", self._submit_job)
        r("GET", r"/api/jobs/(?P<sid>[^/]+)", lambda q, b, sid: self._job_json(self._job_client().get_job_info(sid)))
        r("GET", r"/api/jobs/(?P<sid>[^/]+)/logs", lambda q, b, sid: {"logs": self._job_client().get_job_logs(
            sid, int(q.get("offset", ["0"])[0]))})
        r("POST", r"/api/jobs/(?P<sid>[^/]+)/stop", lambda q, b, sid: {"stopped": self._job_client().stop_job(sid)})
        r("DELETE", r"/api/jobs/(?P<sid>[^/]+)", lambda q, b, sid: {"deleted": self._job_client().delete_job(sid)})
        # GPUs (reference reporter_agent.py _get_gpu_usage) + GPU object stores
        r("GET", r"/api/gpus", lambda q, b: {"gpus": _gpu().gpu_devices(),
                                             "gpu_object_stores": _gpu().gpu_object_stores()})
        # metrics (Prometheus text)
        r("GET", r"/metrics", self._metrics)
        # event / snapshot / actor / serve / tune modules (dashboard/modules.py)
        from ray_memory_management_amd.dashboard.modules import MODULES

        self.modules = [m(self) for m in MODULES]
        for m in self.modules:
            m.register(r)

    def _lister(self, kind):
        def fn(q, b):
            limit = int(q.get("limit", ["10000"])[0])
            rows = getattr(_state(), f"list_{kind}")(filters=_filters(q), limit=limit)
            return {"result": rows, "total": len(rows)}
        return fn

    def _cluster_status(self, q, b):
        w = _w()
        return {"cluster_resources": w.cluster_resources(), "available_resources": w.available_resources(),
                "summary": w._state("summary"), "uptime_s": time.time() - self.started,
                "gpus": _gpu().gpu_devices(),
                "gpu_object_stores": [s for s in _gpu().gpu_object_stores() if s.get("alive")]}

    def _list_logs(self, q, b):
        d = os.path.join(self.session_dir or "", "logs")
        out = []
        for root, _, files in os.walk(d):
            for f in files:
                p = os.path.join(root, f)
                out.append({"filename": os.path.relpath(p, d), "size": os.path.getsize(p)})
        return {"result": sorted(out, key=lambda x: x["filename"])}

    def _log_file(self, q, b):
        d = os.path.realpath(os.path.join(self.session_dir or "", "logs"))
        name = q.get("filename", [""])[0]
        p = os.path.realpath(os.path.join(d, name))
        if not p.startswith(d + os.sep) or not os.path.isfile(p):
            raise _HTTPError(404, f"no log file {name!r}")
        tail = int(q.get("lines", ["0"])[0])
        with open(p, "rb") as f:
            data = f.read().decode(errors="replace")
        if tail > 0:
            data = "\n".join(data.splitlines()[-tail:])
        return _Text(data)

    def _job_client(self):
        with self._jobs_lock:
            if self._jobs is None:
                from ray_memory_management_amd.job_submission import JobSubmissionClient

                self._jobs = JobSubmissionClient()
            return self._jobs

    @staticmethod
    def _job_json(info) -> Dict[str, Any]:
        return {"submission_id": info.submission_id, "job_id": info.submission_id, "status": str(info.status.value),
                "entrypoint": info.entrypoint, "message": info.message, "start_time": info.start_time,
                "end_time": info.end_time, "metadata": info.metadata, "runtime_env": info.runtime_env,
                "driver_exit_code": info.driver_exit_code}

    def _submit_job(self, q, body):
        req = json.loads(body or b"{}")
        if not req.get("entrypoint"):
            raise _HTTPError(400, "entrypoint is required")
        sid = self._job_client().submit_job(entrypoint=req["entrypoint"],
                                            submission_id=req.get("submission_id") or req.get("job_id"),
                                            runtime_env=req.get("runtime_env"), metadata=req.get("metadata"))
        return {"submission_id": sid, "job_id": sid}

    def _metrics(self, q, b):
        from ray_memory_management_amd.util import metrics

        lines = [_builtin_metrics(), _gpu().prometheus_lines(), metrics.prometheus_text()]
        return _Text("".join(lines), "text/plain; version=0.0.4")

    # ------------------------------------------------------------------ server
    def start(self) -> int:
        head = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def _do(self, method):
                u = urlparse(self.path)
                fn, kw = None, None
                for cand in (u.path, u.path.rstrip("/") or "/", u.path.rstrip("/") + "/"):
                    fn, kw = head.routes.match(method, cand)
                    if fn is not None:
                        break
                body = b""
                n = int(self.headers.get("Content-Length") or 0)
                if n:
                    body = self.rfile.read(n)
                if fn is None:
                    return self._send(404, {"error": f"no route {method} {u.path}"})
                try:
                    out = fn(parse_qs(u.query), body, **kw)
                    self._send(200, out)
                except _HTTPError as e:
                    self._send(e.code, {"error": e.msg})
                except (ValueError, RuntimeError, KeyError) as e:
                    self._send(400 if isinstance(e, ValueError) else 404 if isinstance(e, KeyError) else 500,
                               {"error": f"{type(e).__name__}: {e}"})
                except Exception as e:  # noqa: BLE001 - a handler bug answers 500, never drops the socket
                    self._send(500, {"error": f"{type(e).__name__}: {e}"})

            def _send(self, code, out):
                if isinstance(out, _Text):
                    data, ctype = out.text.encode(), out.ctype
                else:
                    data, ctype = json.dumps(out, default=_json_default).encode(), "application/json"
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_DELETE(self):
                self._do("DELETE")

            def do_PUT(self):
                self._do("PUT")

            def log_message(self, *a):
                pass

        self.server = ThreadingHTTPServer((self.host, self.port), Handler)
        self.server.daemon_threads = True
        self.port = self.server.server_address[1]
        threading.Thread(target=self.server.serve_forever, daemon=True, name="dashboard-http").start()
        return self.port

    def stop(self):
        if self.server is not None:
            self.server.shutdown()
            self.server.server_close()
            self.server = None


class _HTTPError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code, self.msg = code, msg


class _Text:
    def __init__(self, text, ctype="text/plain; charset=utf-8"):
        self.text, self.ctype = text, ctype


def _json_default(o):
    if isinstance(o, bytes):
        return o.hex()
    if hasattr(o, "item"):
        return o.item()
    if isinstance(o, (set, tuple)):
        return list(o)
    return str(o)


def _w():
    from ray_memory_management_amd._private import worker

    return worker


def _state():
    from ray_memory_management_amd.util import state

    return state


def _gpu():
    from ray_memory_management_amd.dashboard import gpu_reporter

    return gpu_reporter


def _internal():
    from ray_memory_management_amd import internal

    return internal


def _version():
    try:
        import ray_memory_management_amd as r

        return getattr(r, "__version__", "0")
    except Exception:
        return "0"


def _builtin_metrics() -> str:
    """Cluster gauges the reference's reporter module exports (resources, object store, tasks,
    actors, memory pressure), in Prometheus text format."""
    w = _w()
    lines = []

    def g(name, help_, series):
        lines.append(f"# HELP {name} {help_}\n# TYPE {name} gauge\n")
        for labels, v in series:
            lab = "{" + ",".join(f'{k}="{x}"' for k, x in labels.items()) + "}" if labels else ""
            lines.append(f"{name}{lab} {float(v)}\n")

    tot, avail = w.cluster_resources(), w.available_resources()
    g("rmm_resources_total", "Total logical resources", [({"resource": k}, v) for k, v in sorted(tot.items())])
    g("rmm_resources_available", "Available logical resources",
      [({"resource": k}, avail.get(k, 0.0)) for k in sorted(tot)])
    st = _state().object_store_stats() or {}
    g("rmm_object_store_stats", "Shared-memory object store counters",
      [({"stat": k}, v) for k, v in sorted(st.items()) if isinstance(v, (int, float))])
    counts: Dict[str, int] = {}
    for t in _state().list_tasks():
        counts[t["state"]] = counts.get(t["state"], 0) + 1
    g("rmm_tasks", "Tasks by state", [({"state": k}, v) for k, v in sorted(counts.items())])
    counts = {}
    for a in _state().list_actors():
        counts[a["state"]] = counts.get(a["state"], 0) + 1
    g("rmm_actors", "Actors by state", [({"state": k}, v) for k, v in sorted(counts.items())])
    mp = _internal().memory_pressure_stats() or {}
    g("rmm_memory_pressure", "Memory-pressure machinery counters",
      [({"stat": k}, v) for k, v in sorted(mp.items()) if isinstance(v, (int, float)) and not isinstance(v, bool)])
    return "".join(lines)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8265)
    ap.add_argument("--ready-file", default=None)
    a = ap.parse_args(argv)
    import ray_memory_management_amd as ray

    ray.init(address=a.address, namespace="_rmm_dashboard")
    sess = a.address[len("rmm://"):] if a.address.startswith("rmm://") else _w()._session_dir
    head = DashboardHead(a.host, a.port, sess)
    port = head.start()
    url = f"http://{a.host}:{port}"
    if a.ready_file:
        tmp = a.ready_file + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"url": url, "pid": os.getpid()}, f)
        os.replace(tmp, a.ready_file)
    # exit with the cluster: the head's pid is in session.json
    try:
        head_pid = json.load(open(os.path.join(sess, "session.json"))).get("head_pid")
    except (OSError, ValueError):
        head_pid = None
    while True:
        time.sleep(1.0)
        if head_pid:
            try:
                os.kill(head_pid, 0)
            except ProcessLookupError:
                break
    head.stop()


if __name__ == "__main__":
    main()
