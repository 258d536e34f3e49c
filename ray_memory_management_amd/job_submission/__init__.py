"""Job submission. Parity: reference python/ray/job_submission/__init__.py +
dashboard/modules/job/{sdk.py (JobSubmissionClient), common.py (JobStatus, JobInfo),
job_manager.py (JobManager / JobSupervisor actors running the entrypoint as a subprocess with
logs captured, stop = SIGTERM then SIGKILL)}.

The client talks to a detached JobManager actor in the cluster (no HTTP hop); each job gets a
supervisor actor that runs `entrypoint` in a shell with RMM_ADDRESS pointing at the cluster, so
`ray.init()` inside the job connects to it."""
from __future__ import annotations

import dataclasses
import enum
import os
import signal
import subprocess
import threading
import time
import uuid
from typing import Any, Dict, Iterator, List, Optional

import ray_memory_management_amd as ray

_MANAGER = "_rmm_job_manager"
_NS = "_rmm_jobs"


class JobStatus(str, enum.Enum):
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    STOPPED = "STOPPED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"

    def is_terminal(self) -> bool:
        return self in (JobStatus.STOPPED, JobStatus.SUCCEEDED, JobStatus.FAILED)


@dataclasses.dataclass
class JobInfo:
    status: JobStatus
    entrypoint: str
    submission_id: str
    message: Optional[str] = None
    error_type: Optional[str] = None
    start_time: Optional[float] = None
    end_time: Optional[float] = None
    metadata: Optional[Dict[str, str]] = None
    runtime_env: Optional[Dict[str, Any]] = None
    driver_exit_code: Optional[int] = None

    @property
    def job_id(self):
        return self.submission_id


class _JobManager:
    def __init__(self, session_dir: str):
        self.session_dir = session_dir
        self.jobs: Dict[str, dict] = {}
        self.lock = threading.Lock()
        os.makedirs(os.path.join(session_dir, "logs", "jobs"), exist_ok=True)

    def _log_path(self, sid):
        return os.path.join(self.session_dir, "logs", "jobs", f"job-driver-{sid}.log")

    def submit(self, entrypoint: str, submission_id: Optional[str], runtime_env: Optional[dict],
               metadata: Optional[dict]) -> str:
        sid = submission_id or f"rmmsubmit_{uuid.uuid4().hex[:12]}"
        with self.lock:
            if sid in self.jobs:
                raise ValueError(f"Job with submission_id {sid} already exists. Please use a different submission_id.")
            self.jobs[sid] = {"status": JobStatus.PENDING, "entrypoint": entrypoint, "metadata": metadata or {},
                              "runtime_env": runtime_env or {}, "start_time": time.time(), "end_time": None,
                              "message": "Job is pending", "proc": None, "exit": None}
        threading.Thread(target=self._run, args=(sid,), daemon=True).start()
        return sid

    def _run(self, sid):
        j = self.jobs[sid]
        env = dict(os.environ)
        env["RMM_ADDRESS"] = f"rmm://{self.session_dir}"
        env["RMM_JOB_SUBMISSION_ID"] = sid
        for k, v in (j["runtime_env"].get("env_vars") or {}).items():
            env[k] = str(v)
        cwd = j["runtime_env"].get("working_dir") or None
        with open(self._log_path(sid), "ab") as log:
            try:
                p = subprocess.Popen(j["entrypoint"], shell=True, stdout=log, stderr=subprocess.STDOUT, env=env,
                                     cwd=cwd, start_new_session=True)
            except OSError as e:
                j.update(status=JobStatus.FAILED, message=f"failed to start: {e}", end_time=time.time())
                return
            with self.lock:
                j["proc"] = p
                if j["status"] == JobStatus.PENDING:
                    j["status"] = JobStatus.RUNNING
                    j["message"] = "Job is currently running."
            rc = p.wait()
        with self.lock:
            j["exit"] = rc
            j["end_time"] = time.time()
            if j["status"] == JobStatus.STOPPED:
                j["message"] = "Job was intentionally stopped."
            elif rc == 0:
                j["status"] = JobStatus.SUCCEEDED
                j["message"] = "Job finished successfully."
            else:
                j["status"] = JobStatus.FAILED
                j["message"] = f"Job entrypoint command failed with exit code {rc}"

    def info(self, sid) -> Optional[dict]:
        with self.lock:
            j = self.jobs.get(sid)
            if j is None:
                return None
            return {k: v for k, v in j.items() if k != "proc"}

    def list(self) -> Dict[str, dict]:
        with self.lock:
            return {s: {k: v for k, v in j.items() if k != "proc"} for s, j in self.jobs.items()}

    def logs(self, sid, offset: int = 0) -> str:
        try:
            with open(self._log_path(sid), "rb") as f:
                f.seek(offset)
                return f.read().decode(errors="replace")
        except OSError:
            return ""

    def stop(self, sid) -> bool:
        with self.lock:
            j = self.jobs.get(sid)
            if j is None:
                raise ValueError(f"Job {sid} does not exist")
            if j["status"].is_terminal() if isinstance(j["status"], JobStatus) else False:
                return False
            j["status"] = JobStatus.STOPPED
            p = j["proc"]
        if p is not None and p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)   # the job's own process group
                try:
                    p.wait(timeout=3)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        return True

    def delete(self, sid) -> bool:
        with self.lock:
            j = self.jobs.get(sid)
            if j is None:
                raise ValueError(f"Job {sid} does not exist")
            if not j["status"].is_terminal():
                raise RuntimeError(f"Job {sid} is still running; stop it first")
            del self.jobs[sid]
        return True


def _to_info(sid, d) -> JobInfo:
    return JobInfo(status=JobStatus(d["status"]), entrypoint=d["entrypoint"], submission_id=sid,
                   message=d.get("message"), start_time=d.get("start_time"), end_time=d.get("end_time"),
                   metadata=d.get("metadata"), runtime_env=d.get("runtime_env"), driver_exit_code=d.get("exit"))


class _HttpJobClient:
    """REST client for the dashboard's job module (reference dashboard/modules/job/sdk.py talks
    HTTP to /api/jobs/)."""

    def __init__(self, url: str):
        self.url = url.rstrip("/")

    def _call(self, method, path, body=None):
        import json
        import urllib.error
        import urllib.request

        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(self.url + path, data=data, method=method,
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=60) as r:
                return json.loads(r.read())
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")
            raise RuntimeError(f"{method} {path} -> {e.code}: {msg}") from None

    def submit(self, entrypoint, sid, runtime_env, metadata):
        return self._call("POST", "/api/jobs/", {"entrypoint": entrypoint, "submission_id": sid,
                                                  "runtime_env": runtime_env, "metadata": metadata})["submission_id"]

    def stop(self, sid):
        return self._call("POST", f"/api/jobs/{sid}/stop")["stopped"]

    def delete(self, sid):
        return self._call("DELETE", f"/api/jobs/{sid}")["deleted"]

    def info(self, sid):
        try:
            d = self._call("GET", f"/api/jobs/{sid}")
        except RuntimeError:
            return None
        d["exit"] = d.pop("driver_exit_code", None)
        return d

    def list(self):
        out = {}
        for d in self._call("GET", "/api/jobs/"):
            d["exit"] = d.pop("driver_exit_code", None)
            out[d["submission_id"]] = d
        return out

    def logs(self, sid, offset=0):
        return self._call("GET", f"/api/jobs/{sid}/logs?offset={int(offset)}")["logs"]


class JobSubmissionClient:
    def __init__(self, address: Optional[str] = None, create_cluster_if_needed: bool = False, **kw):
        if address and address.startswith(("http://", "https://")):
            self._http = _HttpJobClient(address)
            return
        self._http = None
        if not ray.is_initialized():
            ray.init(address=address or "auto") if not create_cluster_if_needed else ray.init(address=address)
        from ray_memory_management_amd._private import worker as _w

        try:
            self._m = ray.get_actor(_MANAGER, namespace=_NS)
        except ValueError:
            self._m = ray.remote(_JobManager).options(name=_MANAGER, namespace=_NS, lifetime="detached", num_cpus=0,
                                                      max_concurrency=64, get_if_exists=True).remote(_w._session_dir)

    def _do(self, name, *args):
        if self._http is not None:
            return getattr(self._http, name)(*args)
        return ray.get(getattr(self._m, name).remote(*args))

    def submit_job(self, *, entrypoint: str, job_id: Optional[str] = None, submission_id: Optional[str] = None,
                   runtime_env: Optional[Dict[str, Any]] = None, metadata: Optional[Dict[str, str]] = None,
                   **kw) -> str:
        return self._do("submit", entrypoint, submission_id or job_id, runtime_env, metadata)

    def stop_job(self, job_id: str) -> bool:
        return self._do("stop", job_id)

    def delete_job(self, job_id: str) -> bool:
        return self._do("delete", job_id)

    def get_job_info(self, job_id: str) -> JobInfo:
        d = self._do("info", job_id)
        if d is None:
            raise RuntimeError(f"Job {job_id} does not exist")
        return _to_info(job_id, d)

    def list_jobs(self) -> List[JobInfo]:
        return [_to_info(s, d) for s, d in self._do("list").items()]

    def get_job_status(self, job_id: str) -> JobStatus:
        return self.get_job_info(job_id).status

    def get_job_logs(self, job_id: str, offset: int = 0) -> str:
        return self._do("logs", job_id, offset)

    def tail_job_logs(self, job_id: str, poll_s: float = 0.2) -> Iterator[str]:
        off = 0
        while True:
            chunk = self._do("logs", job_id, off)
            if chunk:
                off += len(chunk.encode())
                yield chunk
            if self.get_job_status(job_id).is_terminal():
                rest = self._do("logs", job_id, off)
                if rest:
                    yield rest
                return
            time.sleep(poll_s)


__all__ = ["JobSubmissionClient", "JobStatus", "JobInfo"]
