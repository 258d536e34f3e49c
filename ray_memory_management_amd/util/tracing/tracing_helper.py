"""Distributed tracing of tasks and actor calls.

Parity: reference python/ray/util/tracing/tracing_helper.py. ``ray.init(_tracing_startup_hook=
"module:function")`` names a function every process of the job (driver and workers) calls at
startup to install a span exporter. Tracing then records, with trace-context propagation through
the task spec:

* a PRODUCER span per submission (``<fn> ray.remote`` / ``<Class>.<method> ray.remote``) in the
  submitting process, and
* a CONSUMER span per execution (``<fn> ray.remote_worker``) in the executing process, whose
  parent is the producer span — so a trace follows a call tree across processes.

OpenTelemetry is not installed in this stack, so spans are this module's own records
(OpenTelemetry's JSON field names: name, context.trace_id / span_id, parent_id, kind, start_time,
end_time, attributes, status) handed to the installed exporter; ``setup_local_tmp_tracing`` writes
one JSON line per span to ``/tmp/spans/<pid>.json`` like the reference's console exporter.
"""
from __future__ import annotations

import contextvars
import importlib
import os
import threading
import time
from typing import Any, Callable, Dict, Optional

_exporter: Optional[Callable[[Dict], None]] = None
_lock = threading.Lock()
_current: contextvars.ContextVar = contextvars.ContextVar("rmm_trace_ctx", default=None)


def _is_tracing_enabled() -> bool:
    return _exporter is not None


def set_exporter(fn: Optional[Callable[[Dict], None]]) -> None:
    """Install the span sink (a callable taking one span dict); None disables tracing."""
    global _exporter
    _exporter = fn


def _import_from_string(import_str: str):
    if ":" in import_str:
        mod, _, attr = import_str.partition(":")
    else:
        mod, _, attr = import_str.rpartition(".")
    return getattr(importlib.import_module(mod), attr)


def _setup_tracing(hook: Optional[str]) -> None:
    """Run the job's tracing startup hook in this process (idempotent per hook)."""
    if not hook or getattr(_setup_tracing, "_done", None) == hook:
        return
    _import_from_string(hook)()
    _setup_tracing._done = hook


def _new_id(nbytes: int) -> str:
    return os.urandom(nbytes).hex()


def _emit(span: Dict) -> None:
    ex = _exporter
    if ex is None:
        return
    try:
        with _lock:
            ex(span)
    except Exception:  # a broken exporter must never fail the task
        pass


def _span(name: str, kind: str, trace_id: str, parent_id: Optional[str], start: float, end: float,
          attributes: Dict[str, Any], status: str = "OK", span_id: Optional[str] = None) -> Dict:
    return {"name": name, "context": {"trace_id": trace_id, "span_id": span_id or _new_id(8)}, "parent_id": parent_id,
            "kind": kind, "start_time": start, "end_time": end, "attributes": attributes,
            "status": {"status_code": status}, "resource": {"process.pid": os.getpid()}}


def inject(spec: Dict, name: str, attributes: Optional[Dict] = None) -> None:
    """Submission side: record the producer span and put its context into the task spec."""
    if _exporter is None:
        return
    parent = _current.get()
    trace_id = parent["trace_id"] if parent else _new_id(16)
    span_id = _new_id(8)
    now = time.time()
    spec["_trace_ctx"] = {"trace_id": trace_id, "parent_span_id": span_id}
    _emit(_span(f"{name} ray.remote", "PRODUCER", trace_id, parent["span_id"] if parent else None, now, now,
                dict(attributes or {}, **{"ray.function": name}), span_id=span_id))


class execution_span:
    """Execution side: ``with execution_span(spec, name): run`` records the consumer span; nested
    submissions inside it become its children."""

    def __init__(self, spec: Dict, name: str, attributes: Optional[Dict] = None):
        self.ctx = spec.get("_trace_ctx") if _exporter is not None else None
        self.name, self.attributes = name, dict(attributes or {})
        self.status = "OK"

    def __enter__(self):
        if self.ctx is None:
            return self
        self.span_id = _new_id(8)
        self.t0 = time.time()
        self.token = _current.set({"trace_id": self.ctx["trace_id"], "span_id": self.span_id})
        return self

    def __exit__(self, et, ev, tb):
        if self.ctx is None:
            return False
        _current.reset(self.token)
        if et is not None:
            self.status = "ERROR"
        _emit(_span(f"{self.name} ray.remote_worker", "CONSUMER", self.ctx["trace_id"], self.ctx["parent_span_id"],
                    self.t0, time.time(), dict(self.attributes, **{"ray.function": self.name}), self.status,
                    span_id=self.span_id))
        return False

    def set_status(self, status: str):
        self.status = status
