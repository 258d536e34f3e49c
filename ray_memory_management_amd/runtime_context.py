"""Runtime context. Parity: reference python/ray/runtime_context.py."""
from __future__ import annotations

from ray_memory_management_amd._private import worker as _w
from ray_memory_management_amd._private.ids import ActorID, JobID, NodeID, TaskID, WorkerID


class RuntimeContext:
    def __init__(self, worker):
        self.worker = worker

    def get(self):
        return {"job_id": self.get_job_id(), "node_id": self.get_node_id(), "namespace": self.namespace,
                "task_id": self.get_task_id(), "actor_id": self.get_actor_id()}

    @property
    def job_id(self):
        return JobID(self.worker.job_id)

    def get_job_id(self) -> str:
        return self.worker.job_id.hex()

    @property
    def node_id(self):
        return self.worker.node_id

    def get_node_id(self):
        return self.worker.node_id

    def _task_id_bytes(self):
        if self.worker.current_actor_id is not None:
            return _w.actor_task_id.get()
        return self.worker.current_task_id

    @property
    def task_id(self):
        t = self._task_id_bytes()
        return TaskID(t) if t else None

    def get_task_id(self):
        t = self._task_id_bytes()
        return t.hex() if t else None

    @property
    def actor_id(self):
        a = self.worker.current_actor_id
        return ActorID(a) if a else None

    def get_actor_id(self):
        a = self.worker.current_actor_id
        return a.hex() if a else None

    def get_worker_id(self):
        return self.worker.worker_id.hex()

    @property
    def namespace(self):
        return self.worker.namespace

    @property
    def was_current_actor_reconstructed(self):
        return bool(getattr(self.worker, "actor_restart_count", 0))

    @property
    def current_actor(self):
        h = self.worker.actor_handle_for_self
        if h is None:
            raise RuntimeError("This method is only available in an actor.")
        return h

    @property
    def should_capture_child_tasks_in_placement_group(self):
        return self.worker.placement_group_capture is not None

    @property
    def current_placement_group_id(self):
        pg = self.worker.placement_group_capture
        return pg.id if pg else None

    def get_placement_group_id(self):
        pg = self.worker.placement_group_capture
        return pg.id.hex() if pg else None

    def get_assigned_resources(self):
        """Resources reserved for the running task / actor (its scheduling request), e.g. {"CPU": 1.0}."""
        res = dict(getattr(self.worker, "assigned_resources", None) or {})
        if self.worker.gpu_ids and "GPU" not in res:
            res["GPU"] = float(len(self.worker.gpu_ids))
        return res

    @property
    def gcs_address(self):
        return self.worker.head_socket

    def get_runtime_env_string(self):
        import json

        return json.dumps(getattr(self.worker, "job_runtime_env", None) or {})


def get_runtime_context() -> RuntimeContext:
    if _w._local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return RuntimeContext(lm.fake_worker())
    return RuntimeContext(_w._require_worker())
