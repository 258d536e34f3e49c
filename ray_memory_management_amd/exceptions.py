"""Exception types. Parity: reference python/ray/exceptions.py."""
from __future__ import annotations

import traceback


class RayError(Exception):
    """Base class for all framework errors."""


class RaySystemError(RayError):
    def __init__(self, client_exc=None, traceback_str=None):
        self.client_exc = client_exc
        self.traceback_str = traceback_str
        super().__init__(str(client_exc))


class RayTaskError(RayError):
    """A task raised an exception. ``cause`` is the original exception.

    ``as_instanceof_cause()`` returns an exception that is BOTH a RayTaskError and an instance of
    the cause's class (reference behaviour), so ``except ValueError`` still works on ``get``."""

    def __init__(self, function_name="", traceback_str="", cause=None, proctitle=None, pid=None, ip=None):
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause
        self.pid = pid
        self.ip = ip
        self.proctitle = proctitle or f"ray::{function_name}"
        super().__init__(self._msg())

    def _msg(self):
        cname = type(self.cause).__name__ if self.cause is not None else "Exception"
        return f"{cname} in {self.function_name} (pid={self.pid}):\n{self.traceback_str}"

    def __str__(self):
        return self._msg()

    def as_instanceof_cause(self):
        cause_cls = type(self.cause) if self.cause is not None else None
        if cause_cls is None or issubclass(RayTaskError, cause_cls) or isinstance(self.cause, RayTaskError):
            return self
        try:
            name = f"RayTaskError({cause_cls.__name__})"
            err = self

            class cls(RayTaskError, cause_cls):  # type: ignore[misc, valid-type]
                def __init__(self, *a, **k):
                    pass

                def __str__(self_inner):
                    return str(err)

                def __getattr__(self_inner, item):
                    return getattr(err.cause, item)

            cls.__name__ = name
            cls.__qualname__ = name
            inst = cls.__new__(cls)
            inst.__dict__.update(self.__dict__)
            inst.args = getattr(self.cause, "args", ())
            return inst
        except TypeError:
            return self

    def __reduce__(self):
        return (RayTaskError, (self.function_name, self.traceback_str, self.cause, self.proctitle, self.pid, self.ip))

    @staticmethod
    def from_exception(e: BaseException, function_name: str, pid=None):
        tb = "".join(traceback.format_exception(type(e), e, e.__traceback__))
        try:
            import pickle

            pickle.dumps(e)
            cause = e
        except Exception:
            cause = RuntimeError(f"{type(e).__name__}: {e} (original exception was not picklable)")
        return RayTaskError(function_name, tb, cause, pid=pid)


class WorkerCrashedError(RayError):
    def __init__(self, message: str = None):
        self.message = message
        super().__init__(*([message] if message else []))

    def __str__(self):
        return self.message or "The worker died unexpectedly while executing this task."

    def __reduce__(self):
        return (type(self), (self.message,))


class RayActorError(RayError):
    def __init__(self, actor_id=None, error_msg="The actor died unexpectedly before finishing this task."):
        self.actor_id = actor_id
        self.error_msg = error_msg
        super().__init__(error_msg)

    def __str__(self):
        return self.error_msg

    def __reduce__(self):
        return (type(self), (self.actor_id, self.error_msg))


class ActorDiedError(RayActorError):
    pass


class ActorUnschedulableError(RayError):
    pass


class LocalRayletDiedError(RayError):
    def __str__(self):
        return "The node manager (head) died."


class TaskCancelledError(RayError):
    def __init__(self, task_id=None):
        self.task_id = task_id
        super().__init__(f"Task {task_id} was cancelled")

    def __reduce__(self):
        return (type(self), (self.task_id,))


class GetTimeoutError(RayError, TimeoutError):
    pass


class ObjectLostError(RayError):
    def __init__(self, object_ref_hex="", owner_address="", call_site="", message=None):
        self.object_ref_hex = object_ref_hex
        self.message = message
        super().__init__(message or f"Object {object_ref_hex} is lost.")

    def __reduce__(self):
        return (type(self), (self.object_ref_hex, "", "", self.message))


class ObjectFetchTimedOutError(ObjectLostError):
    pass


class ReferenceCountingAssertionError(ObjectLostError):
    pass


class OwnerDiedError(ObjectLostError):
    pass


class ObjectReconstructionFailedError(ObjectLostError):
    pass


class ObjectStoreFullError(RayError):
    pass


class OutOfDiskError(RayError):
    pass


class OutOfMemoryError(WorkerCrashedError):
    """The worker running the task was killed by the node's memory monitor (reference node_manager.cc:2902
    memory-pressure eviction). A WorkerCrashedError, as the reference of this era raises for it; the message
    is the eviction's exit detail ("System memory low at node with IP ...")."""

    def __str__(self):
        return self.message or "The worker was killed because the node ran low on memory."


class NodeDiedError(RayError):
    pass


class RuntimeEnvSetupError(RayError):
    pass


class TaskPlacementGroupRemoved(RayError):
    pass


class ActorPlacementGroupRemoved(RayError):
    pass


class PendingCallsLimitExceeded(RayError):
    pass


class TaskUnschedulableError(RayError):
    pass


class AsyncioActorExit(RayError):
    pass


class CrossLanguageError(RayError):
    pass


class RaySystemErrorWrapper(RayError):
    pass


RAY_EXCEPTION_TYPES = [
    RayError, RayTaskError, WorkerCrashedError, RayActorError, ObjectStoreFullError, ObjectLostError,
    GetTimeoutError, TaskCancelledError, OutOfMemoryError, NodeDiedError,
]
