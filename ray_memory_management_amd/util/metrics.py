"""Application metrics: Counter / Gauge / Histogram with tags.

Parity: reference python/ray/util/metrics.py (Metric(name, description, tag_keys),
set_default_tags, Counter.inc, Gauge.set, Histogram(boundaries).observe; tag validation).

Design: every process keeps its metric series in a local registry; a daemon thread flushes
changed series to the head's internal KV (namespace ``__metrics__``, one key per metric and
process) at most every ``FLUSH_INTERVAL_S``. ``collect()`` merges all processes' series (sum for
counters and histograms, last-writer for gauges) and ``prometheus_text()`` renders them in the
Prometheus exposition format (``start_http_exporter`` serves it).
"""
from __future__ import annotations

import json
import os
import re
import threading
import time
from typing import Dict, List, Optional, Tuple

FLUSH_INTERVAL_S = 0.5
_NS = "__metrics__"
_NAME_RE = re.compile(r"^[a-zA-Z_:][a-zA-Z0-9_:]*$")

_registry: Dict[str, "Metric"] = {}
_dirty = threading.Event()
_flusher: Optional[threading.Thread] = None
_lock = threading.Lock()


def _proc_key() -> str:
    return f"{os.getpid()}-{id(_registry)}"


def _ensure_flusher():
    global _flusher
    if _flusher is None or not _flusher.is_alive():
        _flusher = threading.Thread(target=_flush_loop, daemon=True, name="rmm-metrics")
        _flusher.start()


def _flush_loop():
    while True:
        _dirty.wait()
        time.sleep(FLUSH_INTERVAL_S)
        _dirty.clear()
        try:
            flush()
        except Exception:
            pass


def flush():
    """Push this process' series to the head now."""
    from ray_memory_management_amd import internal
    from ray_memory_management_amd._private import worker as _w

    if _w.global_worker is None:
        return
    with _lock:
        payload = {n: m._snapshot() for n, m in _registry.items()}
    for name, snap in payload.items():
        internal._internal_kv_put(f"{name}|{_proc_key()}", json.dumps(snap), True, _NS)


class Metric:
    _type = "untyped"

    def __init__(self, name: str, description: str = "", tag_keys: Optional[Tuple[str, ...]] = None):
        if not name:
            raise ValueError("Empty name is not allowed. Please provide a metric name.")
        if not _NAME_RE.match(name):
            raise ValueError(f"Invalid metric name {name!r}")
        if tag_keys is None:
            tag_keys = tuple()
        if not isinstance(tag_keys, tuple):
            raise TypeError(f"tag_keys should be a tuple type, got: {type(tag_keys)}")
        for k in tag_keys:
            if not isinstance(k, str):
                raise TypeError(f"Tag keys must be str, got {type(k)}.")
        self._name, self._description, self._tag_keys = name, description, tag_keys
        self._default_tags: Dict[str, str] = {}
        self._series: Dict[Tuple[Tuple[str, str], ...], object] = {}
        with _lock:
            _registry[name] = self

    @property
    def info(self) -> dict:
        return {"name": self._name, "description": self._description, "tag_keys": self._tag_keys,
                "default_tags": self._default_tags}

    def set_default_tags(self, default_tags: Dict[str, str]):
        for k, v in default_tags.items():
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
            if not isinstance(v, str):
                raise TypeError(f"Tag values must be str, got {type(v)}.")
        self._default_tags = dict(default_tags)
        return self

    def _tags(self, tags: Optional[Dict[str, str]]):
        final = dict(self._default_tags)
        for k, v in (tags or {}).items():
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
            if not isinstance(v, str):
                raise TypeError(f"Tag values must be str, got {type(v)}.")
            final[k] = v
        missing = [k for k in self._tag_keys if k not in final]
        if missing:
            raise ValueError(f"Missing value for tag key(s): {','.join(missing)}.")
        return tuple(sorted(final.items()))

    def _touch(self):
        _dirty.set()
        _ensure_flusher()

    def _snapshot(self) -> dict:
        return {"type": self._type, "description": self._description,
                "series": [[list(map(list, k)), v] for k, v in self._series.items()]}


class Counter(Metric):
    """Monotonically increasing cumulative value."""
    _type = "counter"

    def inc(self, value: float = 1.0, tags: Optional[Dict[str, str]] = None):
        if value <= 0:
            raise ValueError(f"value must be >0, got {value}")
        k = self._tags(tags)
        with _lock:
            self._series[k] = self._series.get(k, 0.0) + float(value)
        self._touch()


class Gauge(Metric):
    """Current value that can go up and down."""
    _type = "gauge"

    def set(self, value: float, tags: Optional[Dict[str, str]] = None):
        if value is None:
            return
        k = self._tags(tags)
        with _lock:
            self._series[k] = float(value)
        self._touch()


class Histogram(Metric):
    """Distribution over fixed bucket boundaries."""
    _type = "histogram"

    def __init__(self, name: str, description: str = "", boundaries: Optional[List[float]] = None,
                 tag_keys: Optional[Tuple[str, ...]] = None):
        if not boundaries:
            raise ValueError("boundaries argument should be provided when using the Histogram class. "
                             "e.g., Histogram(boundaries=[1.0, 2.0])")
        for b in boundaries:
            if b <= 0:
                raise ValueError("Invalid `boundaries` argument: boundaries must be > 0")
        self.boundaries = sorted(float(b) for b in boundaries)
        super().__init__(name, description, tag_keys)

    def observe(self, value: float, tags: Optional[Dict[str, str]] = None):
        k = self._tags(tags)
        with _lock:
            s = self._series.get(k)
            if s is None:
                s = self._series[k] = {"buckets": [0] * (len(self.boundaries) + 1), "sum": 0.0, "count": 0}
            i = 0
            while i < len(self.boundaries) and value > self.boundaries[i]:
                i += 1
            s["buckets"][i] += 1
            s["sum"] += float(value)
            s["count"] += 1
        self._touch()

    def _snapshot(self) -> dict:
        d = super()._snapshot()
        d["boundaries"] = self.boundaries
        return d

    @property
    def info(self):
        d = super().info
        d["boundaries"] = self.boundaries
        return d


def collect() -> Dict[str, dict]:
    """Cluster-wide view: {name: {"type", "description", "series": {tags_tuple: value}}}."""
    from ray_memory_management_amd import internal

    out: Dict[str, dict] = {}
    for key in internal._internal_kv_list("", namespace=_NS):
        raw = internal._internal_kv_get(key, namespace=_NS)
        if raw is None:
            continue
        name = key.decode().split("|", 1)[0]
        snap = json.loads(raw)
        m = out.setdefault(name, {"type": snap["type"], "description": snap["description"], "series": {},
                                  "boundaries": snap.get("boundaries")})
        for tags, v in snap["series"]:
            k = tuple(tuple(t) for t in tags)
            if snap["type"] == "gauge" or k not in m["series"]:
                m["series"][k] = v
            elif snap["type"] == "counter":
                m["series"][k] += v
            else:
                cur = m["series"][k]
                m["series"][k] = {"buckets": [a + b for a, b in zip(cur["buckets"], v["buckets"])],
                                  "sum": cur["sum"] + v["sum"], "count": cur["count"] + v["count"]}
    return out


def prometheus_text() -> str:
    lines = []

    def lab(tags, extra=()):
        items = list(tags) + list(extra)
        return "{" + ",".join(f'{k}="{v}"' for k, v in items) + "}" if items else ""

    for name, m in sorted(collect().items()):
        lines.append(f"# HELP {name} {m['description']}")
        lines.append(f"# TYPE {name} {m['type']}")
        for tags, v in m["series"].items():
            if m["type"] == "histogram":
                cum = 0
                for b, c in zip(m["boundaries"] + ["+Inf"], v["buckets"]):
                    cum += c
                    lines.append(f"{name}_bucket{lab(tags, [('le', b)])} {cum}")
                lines.append(f"{name}_sum{lab(tags)} {v['sum']}")
                lines.append(f"{name}_count{lab(tags)} {v['count']}")
            else:
                lines.append(f"{name}{lab(tags)} {v}")
    return "\n".join(lines) + "\n"


def start_http_exporter(port: int = 0, host: str = "127.0.0.1"):
    """Serve prometheus_text() at http://host:port/metrics; returns (server, port)."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            body = prometheus_text().encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; version=0.0.4")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer((host, port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, srv.server_address[1]
