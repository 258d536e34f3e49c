"""Cluster events: structured, severity-tagged records of what the runtime did to the user's work
(a worker died, the memory monitor killed a task, an actor restarted, a node left, the spill disk
filled up, a job changed state), appended as JSON lines under ``<session>/logs/events/``.

Parity: reference src/ray/util/event.h (RAY_EVENT: source_type, severity, label, message,
custom_fields; written by the GCS / raylet as ``event_<SOURCE>.log`` files) and
dashboard/modules/event/event_head.py (monitors that directory, serves ``/events`` grouped by job).
One line per event:

  {"event_id": hex, "source_type": "RAYLET", "source_hostname": ..., "source_pid": ..., "severity":
   "ERROR", "label": "WORKER_DIED", "message": ..., "timestamp": unix_s, "custom_fields": {...}}

The head writes through one EventLogger per source type; appends are line-buffered and guarded by
a lock (the head's event loop and its IO threads both report), and a logger that cannot write
(read-only or vanished session dir) drops events rather than failing the runtime.
"""
from __future__ import annotations

import glob
import json
import os
import socket
import threading
import time
from typing import Dict, List, Optional

SEVERITIES = ("DEBUG", "INFO", "WARNING", "ERROR", "FATAL")
SOURCE_TYPES = ("COMMON", "CORE_WORKER", "GCS", "RAYLET", "CLUSTER_LIFECYCLE", "AUTOSCALER", "JOBS", "SERVE")


def events_dir(session_dir: str) -> str:
    return os.path.join(session_dir, "logs", "events")


class EventLogger:
    def __init__(self, session_dir: str, source_type: str):
        if source_type not in SOURCE_TYPES:
            raise ValueError(f"unknown event source type {source_type!r}")
        self.source_type = source_type
        self.path = os.path.join(events_dir(session_dir), f"event_{source_type}.log")
        self.host = socket.gethostname()
        self.pid = os.getpid()
        self.lock = threading.Lock()
        self.f = None
        self.dropped = 0
        self.written = 0

    def emit(self, severity: str, label: str, message: str, **custom_fields) -> Optional[str]:
        if severity not in SEVERITIES:
            raise ValueError(f"unknown severity {severity!r}")
        eid = os.urandom(18).hex()
        rec = {"event_id": eid, "source_type": self.source_type, "source_hostname": self.host,
               "source_pid": self.pid, "severity": severity, "label": label, "message": str(message),
               "timestamp": time.time(),
               "custom_fields": {k: (v.hex() if isinstance(v, bytes) else v) for k, v in custom_fields.items()}}
        line = json.dumps(rec, default=str) + "\n"
        with self.lock:
            try:
                if self.f is None:
                    os.makedirs(os.path.dirname(self.path), exist_ok=True)
                    self.f = open(self.path, "a", buffering=1)
                self.f.write(line)
                self.written += 1
            except OSError:
                self.dropped += 1
                return None
        return eid

    def close(self):
        with self.lock:
            if self.f is not None:
                try:
                    self.f.close()
                except OSError:
                    pass
                self.f = None


def read_events(session_dir: str, job_id: Optional[str] = None, severity: Optional[str] = None,
                limit: int = 10000) -> List[Dict]:
    """Every event under the session (newest last), optionally of one job / at least `severity`."""
    out: List[Dict] = []
    floor = SEVERITIES.index(severity) if severity in SEVERITIES else 0
    for p in sorted(glob.glob(os.path.join(events_dir(session_dir), "event_*.log"))):
        try:
            with open(p) as f:
                for line in f:
                    try:
                        e = json.loads(line)
                    except ValueError:
                        continue  # a line being appended right now
                    if job_id is not None and e.get("custom_fields", {}).get("job_id") != job_id:
                        continue
                    if SEVERITIES.index(e.get("severity", "INFO")) < floor:
                        continue
                    out.append(e)
        except OSError:
            continue
    out.sort(key=lambda e: e.get("timestamp", 0.0))
    return out[-limit:]


def events_by_job(session_dir: str) -> Dict[str, List[Dict]]:
    """The reference /events shape: {job_id: [events]} (events without a job under "global")."""
    out: Dict[str, List[Dict]] = {}
    for e in read_events(session_dir):
        out.setdefault(e.get("custom_fields", {}).get("job_id") or "global", []).append(e)
    return out
