"""State API. Parity: reference python/ray/experimental/state/api.py (list_* / summarize_*)."""
from __future__ import annotations

from typing import List, Optional

from ray_memory_management_amd._private import worker as _w


def _q(what, arg=None):
    return _w._state(what, arg)


def _filter(rows, filters):
    if not filters:
        return rows
    out = []
    for r in rows:
        ok = True
        for key, op, val in filters:
            v = r.get(key)
            if op in ("=", "==") and str(v) != str(val):
                ok = False
            elif op == "!=" and str(v) == str(val):
                ok = False
        if ok:
            out.append(r)
    return out


def list_actors(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("actors"), filters)[:limit]


def list_tasks(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("tasks"), filters)[:limit]


def list_objects(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("objects"), filters)[:limit]


def list_nodes(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("nodes"), filters)[:limit]


def list_workers(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("workers"), filters)[:limit]


def list_jobs(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(_q("jobs"), filters)[:limit]


def list_placement_groups(filters: Optional[list] = None, limit: int = 10000, detail: bool = False) -> List[dict]:
    return _filter(list(_q("placement_groups").values()), filters)[:limit]


def summarize_tasks() -> dict:
    out = {}
    for t in list_tasks():
        s = out.setdefault(t["func_or_class_name"] or "task", {})
        s[t["state"]] = s.get(t["state"], 0) + 1
    return {"cluster": {"summary": out, "total_tasks": sum(sum(v.values()) for v in out.values())}}


def summarize_actors() -> dict:
    out = {}
    for a in list_actors():
        s = out.setdefault(a["class_name"], {})
        s[a["state"]] = s.get(a["state"], 0) + 1
    return {"cluster": {"summary": out}}


def summarize_objects() -> dict:
    objs = list_objects()
    return {"cluster": {"total_objects": len(objs), "total_size_bytes": sum(o["size"] for o in objs),
                        "spilled": sum(1 for o in objs if o["state"] == "SPILLED")}}


def object_store_stats() -> dict:
    return _q("store_stats")


# ---------------------------------------------------------------------------- get_* by id
def _get_one(rows, key, value):
    for r in rows:
        if str(r.get(key)) == str(value):
            return r
    return None


def get_actor(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    return _get_one(list_actors(), "actor_id", id)


def get_task(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    return _get_one(list_tasks(), "task_id", id)


def get_node(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    return _get_one(list_nodes(), "NodeID", id)


def get_worker(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    return _get_one(list_workers(), "worker_id", id)


def get_job(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    for j in list_jobs():
        if id in (str(j.get("job_id")), str(j.get("submission_id")), str(j.get("job_id_hex"))):
            return j
    return None


def get_placement_group(id: str, address=None, timeout: int = 30, _explain: bool = False) -> Optional[dict]:
    pgs = _q("placement_groups")
    return pgs.get(id) if isinstance(pgs, dict) else _get_one(pgs, "placement_group_id", id)


def get_objects(id: str, address=None, timeout: int = 30, _explain: bool = False) -> List[dict]:
    """All copies of one object (here: at most one, the node's store entry)."""
    return [o for o in list_objects() if o.get("object_id") == id]


def list_runtime_envs(address=None, filters: Optional[list] = None, limit: int = 10000, timeout: int = 30,
                      detail: bool = False, raise_on_missing_output: bool = True,
                      _explain: bool = False) -> List[dict]:
    return _filter(_q("runtime_envs"), filters)[:limit]


# ---------------------------------------------------------------------------- logs
def _log_dir() -> str:
    import os

    return os.path.join(_q("session_dir"), "logs")


def list_logs(address=None, node_id: Optional[str] = None, node_ip: Optional[str] = None,
              glob_filter: Optional[str] = None, timeout: int = 30) -> dict:
    """{category: [file names]} of the session's log files (worker-*, head, dashboard, ...)."""
    import fnmatch
    import os

    d = _log_dir()
    files = sorted(f for f in os.listdir(d) if os.path.isfile(os.path.join(d, f))) if os.path.isdir(d) else []
    if glob_filter:
        files = [f for f in files if fnmatch.fnmatch(f, glob_filter)]
    out: dict = {}
    for f in files:
        cat = "worker_out" if f.startswith("worker-") else f.split(".")[0].split("-")[0]
        out.setdefault(cat, []).append(f)
    return out


def get_log(address=None, node_id: Optional[str] = None, node_ip: Optional[str] = None,
            filename: Optional[str] = None, actor_id: Optional[str] = None, task_id: Optional[str] = None,
            pid: Optional[int] = None, follow: bool = False, tail: int = 1000, timeout: int = 30,
            _interval: Optional[float] = None):
    """Yield the last `tail` lines of a log file, chosen by name, actor id, task id or worker pid
    (``follow=True`` keeps yielding appended lines)."""
    import os
    import time

    if filename is None:
        wid = None
        if actor_id is not None:
            w = _get_one(list_workers(), "actor_id", actor_id)
            wid = w and w["worker_id"]
        elif pid is not None:
            w = _get_one(list_workers(), "pid", pid)
            wid = w and w["worker_id"]
        elif task_id is not None:
            t = get_task(task_id)
            w = _get_one(list_workers(), "pid", t.get("worker_pid")) if t else None
            wid = w and w["worker_id"]
        if not wid:
            raise ValueError("no log file found for the given actor_id / task_id / pid; pass filename=")
        filename = f"worker-{wid[:12]}.log"
    path = os.path.join(_log_dir(), os.path.basename(filename))
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    with open(path, "r", errors="replace") as f:
        lines = f.readlines()
        for line in (lines[-tail:] if tail and tail > 0 else lines):
            yield line.rstrip("\n")
        while follow:
            line = f.readline()
            if line:
                yield line.rstrip("\n")
            else:
                time.sleep(_interval or 0.2)


def warnings_on_slow_request(*, address: str = "", endpoint: str = "", timeout: float = 30.0, explain: bool = False):
    """Context manager printing a warning when a state request is slow (reference helper)."""
    import contextlib
    import threading

    @contextlib.contextmanager
    def _cm():
        if not explain:
            yield
            return
        timers = [threading.Timer(timeout / k, lambda k=k: print(f"(explain) request to {endpoint} is slow: "
                                                                  f"{timeout / k:.1f}s elapsed")) for k in (2, 4, 8)]
        for t in timers:
            t.start()
        try:
            yield
        finally:
            for t in timers:
                t.cancel()

    return _cm()
