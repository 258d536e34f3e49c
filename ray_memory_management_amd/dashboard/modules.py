"""Dashboard head modules beyond state / jobs / logs / metrics: events, snapshot, actors, Serve and
Tune. Each registers its routes on the DashboardHead route table and answers with the reference's
``rest_response`` envelope ({"result": bool, "msg": str, "data": {...}}).

Parity (reference dashboard/modules/):
  event/event_head.py:64       GET /events[?job_id=]            cluster events grouped by job
                                                                (_private/event_log.py writes them)
  snapshot/snapshot_head.py:93 GET /api/actors/kill?actor_id=&force_kill=&no_restart=
  snapshot/snapshot_head.py:118 GET /api/snapshot                jobs, job submissions, actors,
                                                                Serve deployments, session, version
  actor/actor_head.py:216-236  GET /logical/actor_groups, /logical/actors, /logical/kill_actor
  serve/serve_agent.py:48-113  GET/PUT/DELETE /api/serve/deployments/, GET .../status
  tune/tune_head.py:44-69      GET /tune/info, /tune/availability, /tune/set_experiment
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional


def rest(success: bool = True, message: str = "", **data) -> Dict[str, Any]:
    return {"result": bool(success), "msg": message, "data": data}


def _w():
    from ray_memory_management_amd._private import worker

    return worker


def _state():
    from ray_memory_management_amd.util import state

    return state


def _kill_by_id(actor_id_hex: str, no_restart: bool = True) -> None:
    from ray_memory_management_amd._private import protocol as P

    try:
        aid = bytes.fromhex(actor_id_hex)
    except ValueError:
        raise ValueError(f"actor_id {actor_id_hex!r} is not hex")
    if not any(a.get("actor_id") == actor_id_hex for a in _state().list_actors()):
        raise KeyError(f"no actor {actor_id_hex}")
    _w()._require_worker().send((P.KILL_ACTOR, aid, bool(no_restart)))


def _flag(q, name, default=False) -> bool:
    v = q.get(name, [None])[0]
    return default if v is None else v in ("1", "true", "True")


class EventModule:
    def __init__(self, head):
        self.head = head

    def register(self, r):
        r("GET", r"/events", self.get_events)

    def get_events(self, q, b):
        from ray_memory_management_amd._private.event_log import events_by_job, read_events

        sess = self.head.session_dir or ""
        job_id = q.get("job_id", [None])[0]
        if job_id is None:
            return rest(True, "All events fetched.", events=events_by_job(sess))
        return rest(True, "Job events fetched.", job_id=job_id,
                    events=read_events(sess, job_id=job_id, severity=q.get("severity", [None])[0]))


class SnapshotModule:
    def __init__(self, head):
        self.head = head

    def register(self, r):
        r("GET", r"/api/snapshot", self.snapshot)
        r("GET", r"/api/actors/kill", self.kill_actor)

    def kill_actor(self, q, b):
        aid = q.get("actor_id", [""])[0]
        if not aid:
            return rest(False, "actor_id is required.")
        # the kill is always immediate here (the head SIGKILLs the actor's worker); no_restart=false
        # lets an actor with max_restarts come back, as in the reference
        _kill_by_id(aid, no_restart=_flag(q, "no_restart", False))
        force = _flag(q, "force_kill", False)
        return rest(True, f"Force killed actor with id {aid}" if force else
                    f"Requested actor with id {aid} to terminate. It will exit once running tasks complete")

    def snapshot(self, q, b):
        limit = int(q.get("actor_limit", ["1000"])[0])
        st = _state()
        jobs = {}
        for j in st.list_jobs():
            k = j.get("job_id")
            jobs[k.hex() if isinstance(k, (bytes, bytearray)) else str(k)] = j
        actors = {a["actor_id"]: a for a in st.list_actors(limit=limit)}
        try:
            subs = [self.head._job_json(i) for i in self.head._job_client().list_jobs()]
        except Exception:  # noqa: BLE001 - no job manager yet
            subs = []
        snap = {"jobs": jobs, "job_submission": subs, "actors": actors, "deployments": ServeModule.deployments(),
                "session_name": os.path.basename((self.head.session_dir or "").rstrip("/")),
                "ray_version": _version(), "ray_commit": None}
        return rest(True, "hello", snapshot=snap)


class ActorModule:
    def __init__(self, head):
        self.head = head

    def register(self, r):
        r("GET", r"/logical/actors", self.actors)
        r("GET", r"/logical/actor_groups", self.actor_groups)
        r("GET", r"/logical/kill_actor", self.kill)

    def actors(self, q, b):
        return rest(True, "All actors fetched.", actors={a["actor_id"]: a for a in _state().list_actors()})

    def actor_groups(self, q, b):
        groups: Dict[str, Dict[str, Any]] = {}
        for a in _state().list_actors():
            g = groups.setdefault(a.get("class_name") or "?", {"entries": [], "summary": {"stateToCount": {}}})
            g["entries"].append(a)
            sc = g["summary"]["stateToCount"]
            sc[a["state"]] = sc.get(a["state"], 0) + 1
        return rest(True, "Fetched actor groups.", actor_groups=groups)

    def kill(self, q, b):
        aid = q.get("actorId", q.get("actor_id", [""]))[0]
        if not aid:
            return rest(False, "actorId is required.")
        _kill_by_id(aid, no_restart=True)
        return rest(True, "Killed actor with id " + aid)


class ServeModule:
    def __init__(self, head):
        self.head = head

    def register(self, r):
        r("GET", r"/api/serve/deployments/", self.get)
        r("GET", r"/api/serve/deployments/status", self.status)
        r("PUT", r"/api/serve/deployments/", self.put)
        r("DELETE", r"/api/serve/deployments/", self.delete)

    @staticmethod
    def deployments() -> Dict[str, Dict[str, Any]]:
        """Every running deployment's options (empty when Serve is not running)."""
        from ray_memory_management_amd import serve

        try:
            ds = serve.list_deployments()
        except Exception:  # noqa: BLE001 - Serve not started
            return {}
        out = {}
        for name, d in ds.items():
            out[name] = {"name": name, "version": d.version, "num_replicas": d.num_replicas,
                         "route_prefix": d.route_prefix, "max_concurrent_queries": d.max_concurrent_queries,
                         "user_config": d.user_config, "ray_actor_options": d.ray_actor_options}
        return out

    def get(self, q, b):
        return {"deployments": list(self.deployments().values())}

    def status(self, q, b):
        from ray_memory_management_amd import serve

        try:
            st = serve.status()
        except Exception as e:  # noqa: BLE001
            return {"app_status": {"status": "NOT_STARTED", "message": repr(e)}, "deployment_statuses": []}
        return {"app_status": {"status": "RUNNING", "message": "", "deployment_timestamp": time.time()},
                "deployment_statuses": [{"name": k, **(v if isinstance(v, dict) else {"status": str(v)})}
                                        for k, v in st.items()]}

    def put(self, q, body):
        """Deploy a ServeApplicationSchema-shaped body: {"import_path": "mod:app", "runtime_env":
        {"working_dir": ...}, "deployments": [per-deployment overrides], "host", "port"}."""
        import sys

        from ray_memory_management_amd import serve
        from ray_memory_management_amd.serve.scripts import _apply_overrides, import_attr

        cfg = json.loads(body or b"{}")
        if not cfg.get("import_path"):
            raise ValueError("import_path is required")
        wd = (cfg.get("runtime_env") or {}).get("working_dir")
        if wd and wd not in sys.path:
            sys.path.insert(0, wd)
        app = _apply_overrides(import_attr(cfg["import_path"]), cfg.get("deployments"))
        http = {"host": cfg.get("host", "127.0.0.1"), "port": int(cfg.get("port", 8000))}
        serve.start(detached=True, http_options=http)
        serve.run(app, host=http["host"], port=http["port"], route_prefix=cfg.get("route_prefix", "/"))
        return {"deployed": sorted(serve.list_deployments()), "http_port": serve.http_port()}

    def delete(self, q, b):
        from ray_memory_management_amd import serve

        serve.shutdown()
        return {"deleted": True}


class TuneModule:
    """Trials of the experiment directory being watched (reference tune_head.py: the dashboard
    follows one Tune experiment's logdir, TUNE_RESULT_DIR or ~/ray_results by default)."""

    def __init__(self, head):
        self.head = head
        self.experiment: Optional[str] = None

    def register(self, r):
        r("GET", r"/tune/info", self.info)
        r("GET", r"/tune/availability", self.availability)
        r("GET", r"/tune/set_experiment", self.set_experiment)

    def _dir(self) -> str:
        return self.experiment or os.environ.get("TUNE_RESULT_DIR") or os.path.expanduser("~/ray_results")

    def availability(self, q, b):
        d = self._dir()
        return rest(True, "Fetched tune availability", result={"available": os.path.isdir(d), "trials_available":
                                                                 bool(self._trial_dirs(d))})

    @staticmethod
    def _trial_dirs(d):
        out = []
        if not os.path.isdir(d):
            return out
        for root, dirs, files in os.walk(d):
            if "params.json" in files:
                out.append(root)
                dirs[:] = []
        return sorted(out)

    def set_experiment(self, q, b):
        exp = q.get("experiment", [""])[0]
        if not exp or not os.path.isdir(os.path.expanduser(exp)):
            return rest(False, f"Not a valid experiment directory: {exp!r}")
        self.experiment = os.path.expanduser(exp)
        return rest(True, "Successfully set experiment", experiment=self.experiment)

    def info(self, q, b):
        from ray_memory_management_amd.tune.result_grid import _LoadedTrial

        trials = {}
        for d in self._trial_dirs(self._dir()):
            try:
                t = _LoadedTrial(d)
            except (OSError, ValueError):
                continue
            last = {k: v for k, v in t.last_result.items() if isinstance(v, (int, float, str, bool))}
            trials[t.trial_id] = {"trial_id": t.trial_id, "job_id": os.path.basename(os.path.dirname(d)),
                                  "logdir": d, "status": t.status, "params": t.config, "metrics": last,
                                  "num_results": len(t.results), "checkpoints": len(t.saved_checkpoints)}
        return rest(True, "Fetched tune info", result={"trial_records": trials, "experiment_dir": self._dir()})


MODULES = (EventModule, SnapshotModule, ActorModule, ServeModule, TuneModule)


def _version():
    try:
        import ray_memory_management_amd as r

        return getattr(r, "__version__", "0")
    except Exception:  # noqa: BLE001
        return "0"
