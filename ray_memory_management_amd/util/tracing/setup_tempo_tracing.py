"""Tracing startup hook that ships spans to an OTLP collector such as Grafana Tempo, and prints each span
to the console (reference python/ray/util/tracing/setup_tempo_tracing.py: an OTLP/gRPC exporter to
localhost:4317 plus a ConsoleSpanExporter).

The OpenTelemetry SDK is not installed in this stack, so the exporter speaks OTLP/HTTP with the JSON
encoding itself (``POST <endpoint>`` with ``ExportTraceServiceRequest`` JSON; Tempo, the OpenTelemetry
Collector and Jaeger accept it on port 4318 at ``/v1/traces``). Spans are batched by one background
thread per process (flushed every ``RMM_OTLP_FLUSH_S`` seconds, at 512 spans, and at exit); a collector
that is down costs dropped spans, never a failed task. Use as
``ray.init(_tracing_startup_hook="ray_memory_management_amd.util.tracing.setup_tempo_tracing:setup_tracing")``.

Environment: ``RMM_OTLP_ENDPOINT`` (default ``http://localhost:4318/v1/traces``), ``RMM_OTLP_SERVICE``
(``service.name``, default ``ray_memory_management_amd``), ``RMM_OTLP_CONSOLE=0`` (no console copy).
"""
from __future__ import annotations

import atexit
import json
import os
import sys
import threading
import urllib.request
from typing import Any, Dict, List, Optional

from ray_memory_management_amd.util.tracing.tracing_helper import set_exporter

# OTLP SpanKind / StatusCode enum values (opentelemetry-proto trace.proto)
_KIND = {"INTERNAL": 1, "SERVER": 2, "CLIENT": 3, "PRODUCER": 4, "CONSUMER": 5}
_STATUS = {"UNSET": 0, "OK": 1, "ERROR": 2}


def _any_value(v: Any) -> Dict:
    if isinstance(v, bool):
        return {"boolValue": v}
    if isinstance(v, int):
        return {"intValue": str(v)}  # int64 travels as a string in OTLP JSON
    if isinstance(v, float):
        return {"doubleValue": v}
    return {"stringValue": str(v)}


def _attrs(d: Dict[str, Any]) -> List[Dict]:
    return [{"key": str(k), "value": _any_value(v)} for k, v in d.items()]


def otlp_span(span: Dict) -> Dict:
    """One tracing_helper span record as an OTLP JSON Span."""
    ctx = span["context"]
    out = {"traceId": ctx["trace_id"], "spanId": ctx["span_id"], "name": span["name"],
           "kind": _KIND.get(span.get("kind", "INTERNAL"), 1),
           "startTimeUnixNano": str(int(span["start_time"] * 1e9)),
           "endTimeUnixNano": str(int(span["end_time"] * 1e9)),
           "attributes": _attrs(span.get("attributes", {})),
           "status": {"code": _STATUS.get(span.get("status", {}).get("status_code", "UNSET"), 0)}}
    if span.get("parent_id"):
        out["parentSpanId"] = span["parent_id"]
    return out


def export_request(spans: List[Dict], service: str) -> Dict:
    """ExportTraceServiceRequest JSON for spans of one process (one resource)."""
    res = {"service.name": service}
    if spans:
        res.update({k: v for k, v in spans[0].get("resource", {}).items()})
    return {"resourceSpans": [{"resource": {"attributes": _attrs(res)},
                               "scopeSpans": [{"scope": {"name": "ray_memory_management_amd.util.tracing"},
                                               "spans": [otlp_span(s) for s in spans]}]}]}


class OTLPHttpExporter:
    """Batching OTLP/HTTP JSON span exporter (callable: the tracing_helper exporter contract)."""

    def __init__(self, endpoint: str, service: str, flush_s: float = 1.0, max_batch: int = 512,
                 timeout_s: float = 5.0, console=None):
        self.endpoint, self.service = endpoint, service
        self.flush_s, self.max_batch, self.timeout_s = flush_s, max_batch, timeout_s
        self.console = console
        self._buf: List[Dict] = []
        self._cv = threading.Condition()
        self._stop = False
        self.sent = self.dropped = self.requests = 0
        self.last_error: Optional[str] = None
        self._th = threading.Thread(target=self._run, name="rmm-otlp-exporter", daemon=True)
        self._th.start()

    def __call__(self, span: Dict) -> None:
        if self.console is not None:
            self.console.write(json.dumps(span) + "\n")
        with self._cv:
            self._buf.append(span)
            if len(self._buf) >= self.max_batch:
                self._cv.notify()

    def _post(self, batch: List[Dict]) -> None:
        body = json.dumps(export_request(batch, self.service)).encode()
        req = urllib.request.Request(self.endpoint, data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s) as r:
                r.read()
            self.sent += len(batch)
        except Exception as e:  # noqa: BLE001 — a collector that is down drops spans, nothing else
            self.dropped += len(batch)
            self.last_error = repr(e)
        self.requests += 1

    def _run(self) -> None:
        while True:
            with self._cv:
                if not self._buf and not self._stop:
                    self._cv.wait(self.flush_s)
                batch, self._buf = self._buf, []
                stop = self._stop
            for i in range(0, len(batch), self.max_batch):
                self._post(batch[i:i + self.max_batch])
            if stop:
                return

    def flush(self) -> None:
        """Send everything queued so far (blocking)."""
        with self._cv:
            batch, self._buf = self._buf, []
        for i in range(0, len(batch), self.max_batch):
            self._post(batch[i:i + self.max_batch])

    def shutdown(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._th.join(timeout=self.timeout_s + 1)


_installed: Optional[OTLPHttpExporter] = None


def setup_tracing() -> None:
    global _installed
    endpoint = os.environ.get("RMM_OTLP_ENDPOINT", "http://localhost:4318/v1/traces")
    service = os.environ.get("RMM_OTLP_SERVICE", "ray_memory_management_amd")
    console = None if os.environ.get("RMM_OTLP_CONSOLE", "1") == "0" else sys.stdout
    if _installed is not None:
        _installed.shutdown()
    _installed = OTLPHttpExporter(endpoint, service, flush_s=float(os.environ.get("RMM_OTLP_FLUSH_S", "1.0")),
                                  console=console)
    set_exporter(_installed)
    atexit.register(_installed.shutdown)
