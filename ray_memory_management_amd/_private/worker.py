"""Core worker (one per process: driver or worker) and the public core API.

Parity: reference python/ray/_private/worker.py (init/get/put/wait/remote/kill/cancel/shutdown,
get_gpu_ids) and src/ray/core_worker/core_worker.cc (task submission, reference counting,
direct actor transport, dependency handling for `get`).
"""
from __future__ import annotations

import atexit
import collections
import contextvars
import ctypes
import hashlib
import json
import logging
import os
import queue
import socket
import subprocess
import sys
import tempfile
import threading
import time
import traceback
import uuid
from typing import Any, Dict, List, Optional, Sequence

import cloudpickle

from ray_memory_management_amd import exceptions as exc
from ray_memory_management_amd._native import store_ext
from ray_memory_management_amd._private import ids as _ids
from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import serialization as ser
from ray_memory_management_amd.object_ref import ObjectRef, _set_worker

logger = logging.getLogger("ray_memory_management_amd")

SCRIPT_MODE = 0
WORKER_MODE = 1
LOCAL_MODE = 2
SPILL_WORKER_MODE = 3
RESTORE_WORKER_MODE = 4

global_worker: Optional["CoreWorker"] = None
_init_lock = threading.RLock()


class _Pending:
    __slots__ = ("ev", "value", "cb")

    def __init__(self, cb=None):
        self.ev = threading.Event()
        self.value = None
        self.cb = cb


# id of the actor task running in this thread / asyncio task (actors run calls on several threads or
# coroutines at once, so one worker attribute would be wrong): read by RuntimeContext.get_task_id
actor_task_id: "contextvars.ContextVar[Optional[bytes]]" = contextvars.ContextVar("rmm_actor_task_id", default=None)


class _ActorCallPin:
    """A reference to an actor (its scope key) held by one submitted call's keep-alive list until the call
    is done; used for actor handles nested inside a call's inline arguments. Released by __del__ when the
    call's in-flight / queued entry is dropped, whichever path drops it."""

    __slots__ = ("worker", "key")

    def __init__(self, worker, key: bytes):
        self.worker, self.key = worker, key
        worker.add_local_ref(key)

    def __del__(self):
        try:
            self.worker.remove_local_ref(self.key)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class ActorConn:
    """Direct caller→actor connection with in-flight tracking (direct actor transport).

    Submission never blocks on the actor's state (reference direct_actor_task_submitter.cc queues calls
    until the actor is alive): while there is no connection, calls wait in `queued` in submission order and
    one background thread asks the head for the actor's address (WAIT_ACTOR answers once the actor is
    alive or dead), connects, and sends them in order."""

    def __init__(self, worker: "CoreWorker", actor_id: bytes, max_task_retries: int):
        self.worker = worker
        self.actor_id = actor_id
        self.max_task_retries = max_task_retries
        self.lock = threading.Lock()
        self.sock: Optional[socket.socket] = None
        self.seq = 0
        self.inflight: Dict[int, tuple] = {}
        self.queued: list = []  # (spec, keep_alive, tries) waiting for a connection, in order
        self.dead_error: Optional[BaseException] = None
        self.epoch = -1
        self.connected = threading.Event()
        self.connecting = False
        # While any call is queued or in flight the caller holds one reference to the actor, so dropping the
        # last handle right after a call, as in ``ray.get(Actor.remote().method.remote())``, terminates the
        # actor only once that call has run (reference python/ray/tests/test_actor.py:797
        # test_actor_method_deletion). One ref per busy period, not per call: the submit path stays cheap.
        self.pinned = False
        from ray_memory_management_amd.actor import _actor_ref_key

        self.scope_key = _actor_ref_key(actor_id)

    def _unpin_if_idle_locked(self):
        if self.pinned and not self.inflight and not self.queued:
            self.pinned = False
            self.worker.remove_local_ref(self.scope_key)

    def _connect(self):
        """Blocking: the head's WAIT_ACTOR answer -> a connected socket, or None (dead_error set)."""
        # The head may briefly still advertise the address of a process that just died; retry
        # until it reports the restarted address or the death.
        for attempt in range(200):
            status = self.worker.request(lambda rid: (P.WAIT_ACTOR, rid, self.actor_id))
            if status[0] != "alive" or status[2] != self.epoch or self.epoch < 0:
                try:
                    return self._connect_once(status)
                except (ConnectionRefusedError, FileNotFoundError):
                    pass
            time.sleep(0.05)
        self.dead_error = exc.RayActorError(self.actor_id.hex(), "could not connect to the actor")
        return None

    def _connect_once(self, status):
        kind, addr, restarts = status
        if kind == "dead":
            cause = addr
            if isinstance(cause, (bytes, bytearray)):
                try:
                    cause = ser.loads_inline(cause)
                except Exception:
                    cause = None
            if isinstance(cause, BaseException):
                self.dead_error = exc.RayActorError(self.actor_id.hex(),
                                                    f"The actor died because of an error raised in its creation task: {cause}")
                self.dead_error.__cause__ = cause
            else:
                self.dead_error = exc.RayActorError(self.actor_id.hex(), f"The actor is dead: {cause}")
            return None
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.connect(addr)
            P.send(s, (P.ACTOR_HELLO, os.getpid()))
        except OSError:
            s.close()
            raise ConnectionRefusedError(addr)
        self.epoch = restarts
        return s

    def _start_connect_locked(self):
        if not self.connecting:
            self.connecting = True
            threading.Thread(target=self._connect_and_flush, daemon=True, name="rmm-actor-connect").start()

    def _connect_and_flush(self):
        try:
            s = self._connect()
        except Exception as e:  # noqa: BLE001 - head gone / shutdown
            s = None
            if self.dead_error is None:
                self.dead_error = exc.RayActorError(self.actor_id.hex(), f"could not reach the actor: {e!r}")
        with self.lock:
            self.connecting = False
            items, self.queued = self.queued, []
            if s is None:
                for spec, keep, tries in items:
                    self.worker._store_errors(spec["return_ids"], self.dead_error)
                self._unpin_if_idle_locked()
                return
            self.sock = s
            self.connected.set()
            threading.Thread(target=self._reader, args=(s,), daemon=True).start()
            for spec, keep, tries in items:
                self._send_locked(spec, keep, tries)

    def _send_locked(self, spec, keep_alive, tries):
        self.seq += 1
        spec["seq"] = self.seq
        self.inflight[self.seq] = (spec, keep_alive, tries)
        try:
            P.send(self.sock, (P.ACTOR_TASK, spec))
        except OSError:
            pass  # the reader thread observes the failure and handles in-flight tasks

    def submit(self, spec, keep_alive):
        with self.lock:
            if self.dead_error is not None:
                self.worker._store_errors(spec["return_ids"], self.dead_error)
                return
            if not self.pinned:
                self.pinned = True
                self.worker.add_local_ref(self.scope_key)
            if self.sock is None or self.queued:
                self.queued.append((spec, keep_alive, 0))
                self._start_connect_locked()
                return
            self._send_locked(spec, keep_alive, 0)

    def _reader(self, s: socket.socket):
        try:
            while True:
                m = P.recv(s)
                if m[0] == P.REPLY:  # ack batch: list of seq
                    with self.lock:
                        for sq in m[2]:
                            self.inflight.pop(sq, None)
                        if not self.inflight:
                            self._unpin_if_idle_locked()
        except (ConnectionError, OSError, EOFError):
            pass
        self._on_disconnect(s)

    def _on_disconnect(self, s):
        with self.lock:
            if self.sock is not s:
                return
            self.sock = None
            self.connected.clear()
            pending = sorted(self.inflight.items())
            self.inflight.clear()
            retry, failed = [], []
            for sq, (spec, keep, tries) in pending:
                if self.max_task_retries != 0 and (self.max_task_retries < 0 or tries < self.max_task_retries):
                    retry.append((spec, keep, tries + 1))
                else:
                    failed.append((spec, keep))
            if failed:
                self._fail_inflight(failed)
            if retry:  # resent, in their original order, once the restarted actor is reachable
                self.queued[:0] = retry
            if self.queued:
                self._start_connect_locked()
            else:
                self._unpin_if_idle_locked()

    def _fail_inflight(self, failed):
        """In-flight calls of an actor whose process died: RayActorError, with the head's exit detail when
        it killed the actor (memory monitor: "System memory low ...", reference node_manager.cc:2962)."""
        aid = self.actor_id

        def done(reply):
            msg = "The actor died unexpectedly before finishing this task."
            if isinstance(reply, str) and reply:
                msg += " " + reply
            err = exc.RayActorError(aid.hex(), msg)
            w = self.worker
            for spec, _keep in failed:
                # a call that completed but whose ack was lost with the process has nothing to report, and a
                # return nobody references any more (its result was read and dropped) must not be re-created
                # as an error object no one would ever free
                rids = [o for o in spec["return_ids"] if o in w.local_refs and not w.store.contains(o)]
                if rids:
                    w._store_errors(rids, err)

        try:
            self.worker.request_async(lambda rid: (P.EXIT_DETAIL, rid, aid), done)
        except Exception:  # noqa: BLE001 - no head: plain actor death
            done(None)

    def close(self):
        with self.lock:
            if self.sock is not None:
                try:
                    self.sock.close()
                except OSError:
                    pass


class CoreWorker:
    def __init__(self, mode, head_socket, store_name, session_dir, job_id=None, namespace=None,
                 worker_id=None, node_id=1):
        self.mode = mode
        self.session_dir = session_dir
        self.head_socket = head_socket
        self.store_name = store_name
        self.store = store_ext().ObjectStore.attach(store_name)
        self.worker_id = worker_id or os.urandom(16)
        self.job_id = job_id or os.urandom(4)
        self._namespace = namespace
        self.node_id = node_id
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.connect(head_socket)
        self.send_lock = threading.Lock()
        self.req_lock = threading.Lock()
        self.reqs: Dict[int, _Pending] = {}
        self.req_counter = 0
        self.task_queue: "queue.Queue" = queue.Queue()
        self.ref_lock = threading.Lock()
        # removals from __del__ (GC can run them inside a ref_lock critical section of the same
        # thread): queued lock-free, applied by whoever next holds ref_lock
        self._deferred_removes: "collections.deque" = collections.deque()
        # GPU objects put by this process whose ref never left it (never pickled, never a task
        # arg): the owner frees their HBM as soon as its last local ref dies, without the head
        # round trip (the reference's owner-side free when no borrower exists)
        self._gpu_unescaped: set = set()
        self._eager_gpu_free: List[bytes] = []
        self.local_refs: Dict[bytes, int] = {}
        self.deltas: Dict[bytes, int] = {}
        self.exported = set()
        self.actor_conns: Dict[bytes, ActorConn] = {}
        self.connected = True
        self.current_task_id: Optional[bytes] = None
        self.current_actor_id: Optional[bytes] = None
        self.current_task_name = None
        self.gpu_ids: List[int] = [int(x) for x in os.environ.get("RMM_GPU_IDS", "").split(",") if x != ""]
        self.blocked = False
        self.events: List[dict] = []
        self.events_lock = threading.Lock()
        self.gpu_store = None
        self.config: Dict[str, Any] = json.loads(os.environ.get("RMM_CONFIG", "{}") or "{}")
        self.placement_group_capture = None  # (pg, capture_child_tasks)
        self.actor_handle_for_self = None
        self.direct = None  # DirectTaskSubmitter (worker leases), created on first eligible task
        self.multi_node = False  # head-pushed: direct submission only on single-node clusters
        self.pushed_errors = collections.deque(maxlen=100)  # head-pushed warnings (PUSH_ERROR) for this job
        self._reader_t = threading.Thread(target=self._reader, daemon=True, name="rmm-reader")
        self._reader_t.start()
        self._flusher_stop = threading.Event()
        self._flusher = threading.Thread(target=self._flush_loop, daemon=True, name="rmm-flusher")
        self._flusher.start()

    # ------------------------------------------------------------------ head connection
    def _reader(self):
        try:
            while True:
                m = P.recv(self.sock)
                t = m[0]
                if t == P.REPLY:
                    p = self.reqs.pop(m[1], None)
                    if p is not None:
                        if p.cb is not None:
                            try:
                                p.cb(m[2])
                            except Exception as e:  # pragma: no cover
                                logger.warning("async reply handler failed: %r", e)
                            # drop the callback (and whatever its closure keeps alive: a failed call's
                            # argument refs) now, not when the next message from the head rebinds `p`
                            p = m = None
                            continue
                        p.value = m[2]
                        p.ev.set()
                elif t == P.NODES_CHANGED:
                    self.multi_node = bool(m[1])
                elif t == P.TRIGGER_GC:
                    threading.Thread(target=_collect_garbage, daemon=True).start()
                elif t == P.PUSH_ERROR:  # scheduler warning for this job (infeasible task, resource deadlock)
                    self.pushed_errors.append({"type": m[1], "message": m[2], "time": time.time()})
                    if self.mode == SCRIPT_MODE:
                        print(f"(raylet) [{m[1]}] {m[2]}", file=sys.stderr, flush=True)
                elif t in (P.CANCEL_TASK, P.FREE_GPU):
                    try:  # a failing side-channel handler must never take the reader thread down
                        if t == P.CANCEL_TASK:
                            self._cancel_current(m[1])
                        else:
                            self._free_gpu(m[1])
                    except Exception as e:  # pragma: no cover
                        logger.warning("handler for message %s failed: %r", t, e)
                else:
                    self.task_queue.put(m)
        except (ConnectionError, OSError, EOFError):
            pass
        self.connected = False
        for p in list(self.reqs.values()):
            p.value = exc.LocalRayletDiedError()
            p.ev.set()
            if p.cb is not None:
                try:
                    p.cb(p.value)
                except Exception:
                    pass
        self.task_queue.put((P.EXIT,))

    def _flush_loop(self):
        while not self._flusher_stop.wait(0.01):
            if self.direct is not None and self.direct.done_buf:
                self.direct.flush()
            if self._eager_gpu_free:
                self._run_eager_frees()
            if getattr(self, "_gpu_deferred_free", None):
                try:  # GPU objects whose descriptors were still pinned by readers at FREE time
                    from ray_memory_management_amd._private import gpu_object_store as gos

                    gos.retry_deferred(self)
                except Exception:
                    pass
            # queued removals count too: a __del__ that lost the try-lock race (or ran inside a
            # ref_lock critical section) is drained here, under ref_lock, by _take_deltas
            if self.deltas or self._deferred_removes:
                try:
                    self.send(None)
                except Exception:
                    pass

    def _take_deltas(self):
        with self.ref_lock:
            self._drain_removes()
            if not self.deltas:
                return None
            # A ref created and dropped between two flushes nets to 0 but must still reach the head:
            # (oid, 0) with no local ref left lets the head free an object nobody else references.
            d = [(k, v) for k, v in self.deltas.items() if v or k not in self.local_refs]
            self.deltas = {}
        return d

    def send(self, msg):
        if not self.connected:
            if msg is None:
                return
            raise exc.LocalRayletDiedError()
        with self.send_lock:
            d = self._take_deltas()
            try:
                if d:
                    P.send(self.sock, (P.REF_DELTAS, d))
                if msg is not None:
                    P.send(self.sock, msg)
            except OSError:
                self.connected = False
                if msg is not None:
                    raise exc.LocalRayletDiedError()

    def request_async(self, build, cb):
        """Send a request; `cb(reply)` runs on the reader thread when the head answers."""
        p = _Pending(cb)
        with self.req_lock:
            self.req_counter += 1
            rid = self.req_counter
            self.reqs[rid] = p
        self.send(build(rid))

    def request(self, build, timeout=None):
        p = _Pending()
        with self.req_lock:
            self.req_counter += 1
            rid = self.req_counter
            self.reqs[rid] = p
        self.send(build(rid))
        if not p.ev.wait(timeout):
            self.reqs.pop(rid, None)
            raise exc.GetTimeoutError("request to the head timed out")
        if isinstance(p.value, exc.LocalRayletDiedError):
            raise p.value
        return p.value

    # ------------------------------------------------------------------ reference counting
    def add_local_ref(self, oid: bytes):
        with self.ref_lock:
            self._drain_removes()
            n = self.local_refs.get(oid, 0)
            self.local_refs[oid] = n + 1
            if n == 0:
                self.deltas[oid] = self.deltas.get(oid, 0) + 1

    def remove_local_ref(self, oid: bytes):
        """Called from ObjectRef/ActorHandle __del__, i.e. possibly from a GC pass that runs while
        this very thread holds ref_lock: never block on it."""
        self._deferred_removes.append(oid)
        if self.ref_lock.acquire(blocking=False):
            try:
                self._drain_removes()
            finally:
                self.ref_lock.release()
            if self._eager_gpu_free:
                self._run_eager_frees()

    def pending_borrows(self) -> bool:
        """True when this process took references (0 -> 1) the head has not been told about yet."""
        with self.ref_lock:
            self._drain_removes()
            return any(v > 0 for v in self.deltas.values())

    def flush_refs_sync(self):
        """Make the head apply this process's new references before returning. An actor calls it before it
        acknowledges a call to its caller: the ack lets the caller drop the refs it kept for the call, and the
        head must see the actor's borrow of those refs first (both reach the head over different
        connections)."""
        if self.pending_borrows():
            self.request(lambda rid: (P.STATE, rid, "session_dir", None))

    def pin_out_of_band(self, oid: bytes):
        """One permanent local reference per object pickled out of band (dropped with this process)."""
        pins = self.__dict__.setdefault("_oob_pins", set())
        if oid in pins:
            return
        pins.add(oid)
        self.add_local_ref(oid)

    def note_escaped(self, oid: bytes):
        """The ref is being serialized or handed to a task: another process may now borrow it."""
        self._gpu_unescaped.discard(oid)

    def _run_eager_frees(self):
        from ray_memory_management_amd._private import gpu_object_store as gos

        while self._eager_gpu_free:
            try:
                oid = self._eager_gpu_free.pop()
            except IndexError:
                return
            try:
                gos.free_unescaped(self, oid)
            except Exception:
                pass  # the head's FREE_GPU still frees it

    def _drain_removes(self):  # caller holds ref_lock
        q = self._deferred_removes
        while q:
            oid = q.popleft()
            n = self.local_refs.get(oid, 0) - 1
            if n <= 0:
                self.local_refs.pop(oid, None)
                self.deltas[oid] = self.deltas.get(oid, 0) - 1
                if oid in self._gpu_unescaped:
                    self._gpu_unescaped.discard(oid)
                    self._eager_gpu_free.append(oid)
            else:
                self.local_refs[oid] = n

    # ------------------------------------------------------------------ objects
    def put_object(self, value, oid: Optional[bytes] = None, _owner=None) -> ObjectRef:
        if isinstance(value, ObjectRef):
            raise TypeError("Calling 'put' on an ObjectRef is not allowed. If you really want to do this, "
                            "you can wrap the ObjectRef in a list and call 'put' on it.")
        oid = oid or _ids.new_put_id()
        ref = None
        if _is_cuda_tensor(value) and self.config.get("gpu_object_store", True):
            from ray_memory_management_amd._private import gpu_object_store as gos

            ref = ObjectRef(oid)
            gos.put_tensor(self, oid, value)
            self.send((P.GPU_OBJECT, oid))
            if _owner is None:
                self._gpu_unescaped.add(oid)
            return ref
        with self.gpu_sink():
            data, bufs, contained = ser.serialize(value)
        return self._put_serialized(oid, data, bufs, contained)

    def _put_serialized(self, oid: bytes, data, bufs, contained) -> ObjectRef:
        """Store an already-serialized value (`ser.serialize` output) under `oid`."""
        ref = ObjectRef(oid)
        if contained:
            self.send((P.CONTAINED, oid, contained))
        try:
            self.store.put_serialized(oid, data, bufs, ser.TAG_PICKLE, False)
        except RuntimeError as e:
            if "OutOfDiskError" in str(e):
                raise exc.OutOfDiskError(str(e)) from None
            if "ObjectStoreFullError" in str(e):
                raise exc.ObjectStoreFullError(str(e)) from None
            raise
        return ref

    def gpu_sink(self):
        """Serializer context that keeps nested CUDA tensors in the HBM object store."""
        import contextlib

        if not self.config.get("gpu_object_store", True) or not self.config.get("gpu_nested_tensors", True):
            return contextlib.nullcontext()
        return ser.gpu_sink(self._gpu_sink_put)

    def _gpu_sink_put(self, t) -> bytes:
        from ray_memory_management_amd._private import gpu_object_store as gos

        oid = _ids.new_put_id()
        gos.put_tensor(self, oid, t)
        self.send((P.GPU_OBJECT, oid))
        return oid

    def get_gpu_object(self, oid: bytes):
        from ray_memory_management_amd._private import gpu_object_store as gos

        return gos.get_tensor(self, oid)

    def _store_errors(self, return_ids, error):
        data, bufs, _ = ser.serialize(error)
        for oid in return_ids:
            try:
                if not self.store.contains(oid):
                    self.store.put_serialized(oid, data, bufs, ser.TAG_ERROR, True)
            except Exception:
                pass

    def _deserialize_entry(self, oid, r):
        pickled, bufs, tag, is_error, raw = r
        if tag == ser.TAG_GPU:
            from ray_memory_management_amd._private import gpu_object_store as gos

            return gos.get_tensor(self, oid, pickled), False
        value = ser.deserialize(pickled, bufs)
        return value, is_error

    on_block = None  # worker processes: bounce queued direct tasks when the running one blocks

    def _set_blocked(self, blocked: bool):
        if self.mode == WORKER_MODE and self.current_task_id is not None and self.current_actor_id is None:
            if blocked and self.on_block is not None:
                try:
                    self.on_block()
                except Exception as e:  # pragma: no cover
                    logger.warning("bouncing queued direct tasks failed: %r", e)
            if self.blocked != blocked:
                self.blocked = blocked
                try:
                    self.send((P.BLOCKED if blocked else P.UNBLOCKED,))
                except Exception:
                    pass

    def get(self, refs: Sequence[ObjectRef], timeout: Optional[float] = None):
        deadline = None if timeout is None else time.time() + timeout
        out = []
        blocked = False
        try:
            for ref in refs:
                if not isinstance(ref, ObjectRef):
                    raise TypeError(f"get() expects ObjectRefs, got {type(ref)}")
                oid = ref.binary()
                r = self.store.get_serialized(oid, 0)
                while r is None:
                    if not blocked:
                        blocked = True
                        self._set_blocked(True)
                    if not self.connected:
                        raise exc.LocalRayletDiedError()
                    if deadline is not None:
                        rem = deadline - time.time()
                        if rem <= 0:
                            raise exc.GetTimeoutError(f"Get timed out: some object(s) not ready: {ref}")
                        slice_ms = int(min(rem, 1.0) * 1000) or 1
                    else:
                        slice_ms = 1000
                    r = self.store.get_serialized(oid, slice_ms)
                value, is_error = self._deserialize_entry(oid, r)
                if is_error:
                    if isinstance(value, exc.RayTaskError):
                        raise value.as_instanceof_cause()
                    if isinstance(value, BaseException):
                        raise value
                out.append(value)
        finally:
            if blocked:
                self._set_blocked(False)
        return out

    def wait(self, refs, num_returns=1, timeout=None, fetch_local=True):
        if not refs:
            return [], []
        oids = [r.binary() for r in refs]
        blocked = False
        tm = -1 if timeout is None else int(timeout * 1000)
        try:
            ready_mask = self.store.wait(oids, num_returns, 0)
            if sum(ready_mask) < num_returns and tm != 0:
                blocked = True
                self._set_blocked(True)
                ready_mask = self.store.wait(oids, num_returns, tm)
        finally:
            if blocked:
                self._set_blocked(False)
        ready, not_ready = [], []
        for r, ok in zip(refs, ready_mask):
            if ok and len(ready) < num_returns:
                ready.append(r)
            else:
                not_ready.append(r)
        return ready, not_ready

    # ------------------------------------------------------------------ submission
    def export(self, fid: bytes, blob: bytes) -> Optional[bytes]:
        if fid in self.exported:
            return None
        self.exported.add(fid)
        return blob

    @property
    def namespace(self):
        """The namespace of the job the current task belongs to (reference: a worker runs in its job's
        namespace, so named-actor lookups inside tasks and actors resolve like the driver's). Workers
        resolve it lazily from the head's job table."""
        ns = self._namespace
        if ns is None and self.mode != SCRIPT_MODE:
            ns = self._namespace = self._job_namespace(self.job_id)
        return ns

    @namespace.setter
    def namespace(self, ns):
        self._namespace = ns

    def enter_job(self, job_id):
        """A task / actor of job `job_id` is about to run here: nested submissions belong to that job."""
        if job_id is not None and job_id != self.job_id:
            self.job_id = job_id
            self._namespace = None

    def _job_namespace(self, job_id):
        try:
            for j in self.request(lambda rid: (P.STATE, rid, "jobs", None)):
                if j.get("job_id") == job_id:
                    return j.get("namespace")
        except Exception:  # noqa: BLE001 - head unreachable: no namespace
            pass
        return None

    def prepare_args(self, args, kwargs):
        """Returns (encoded_args, encoded_kwargs, arg_refs, keep_alive)."""
        arg_refs: List[bytes] = []
        keep: List[Any] = []

        def enc(v):
            if type(v) in ser._PRIMITIVES:  # hot path: small scalars pickle directly
                return ("v", ser.pickle.dumps(v, protocol=5))
            if isinstance(v, ObjectRef):
                self.note_escaped(v._id)
                arg_refs.append(v.binary())
                keep.append(v)
                return ("r", v.binary())
            # serialize ONCE (nested CUDA tensors become GPU objects here): a second pass for the
            # by-ref case would create a second, unreferenced set of GPU objects
            with self.gpu_sink():
                data, bufs, contained = ser.serialize(v)
            size = len(data) + sum(memoryview(b).nbytes for b in bufs)
            if size > ser.INLINE_THRESHOLD:
                ref = self._put_serialized(_ids.new_put_id(), data, bufs, contained)
                keep.append(ref)
                arg_refs.append(ref.binary())
                return ("r", ref.binary())
            if contained:
                arg_refs.extend(contained)
            if bufs:  # small out-of-band buffers travel with the spec (writable on the worker)
                return ("b", (data, [bytearray(b) for b in bufs]))
            return ("v", data)

        ea = [enc(a) for a in args]
        ek = {k: enc(v) for k, v in kwargs.items()}
        return ea, ek, arg_refs, keep

    def submit_task(self, spec: dict, keep, blob: Optional[bytes] = None) -> List[ObjectRef]:
        task_id = _ids.new_task_id()
        spec["task_id"] = task_id
        nr = spec.get("num_returns", 1)
        n = nr if isinstance(nr, int) else 1
        ret_ids = [_ids.object_id_for_return(task_id, i) for i in range(1, n + 1)]
        refs = [ObjectRef(o) for o in ret_ids]
        spec["return_ids"] = ret_ids
        spec["job_id"] = self.job_id
        spec["parent_task_id"] = self.current_task_id
        tr = sys.modules.get(_TRACING_MOD)
        if tr is not None and tr._exporter is not None:
            tr.inject(spec, spec.get("name", "task"), {"ray.task_id": task_id.hex()})
        if self.config.get("direct_task_submission", True):
            d = self.direct
            if d is None:
                from ray_memory_management_amd._private.direct_task import DirectTaskSubmitter

                d = self.direct = DirectTaskSubmitter(self)
            if d.eligible(spec):
                fn_blob = spec.pop("fn_blob", None)
                if fn_blob is not None:  # the head still needs it (head-path tasks, lineage resubmits)
                    self.send((P.FN_EXPORT, spec["fn_id"], fn_blob))
                if spec.get("arg_refs"):  # the head must know the args' refs before the worker drops its own
                    self.send(None)
                d.submit(spec, keep, fn_blob if fn_blob is not None else blob)
                return refs
        self.send((P.SUBMIT_TASK, spec))
        return refs

    def submit_actor_task(self, actor_id: bytes, spec: dict, keep, max_task_retries: int,
                          arg_refs=None) -> List[ObjectRef]:
        task_id = _ids.new_task_id()
        spec["task_id"] = task_id
        nr = spec.get("num_returns", 1)
        n = nr if isinstance(nr, int) else 1
        ret_ids = [_ids.object_id_for_return(task_id, i) for i in range(1, n + 1)]
        refs = [ObjectRef(o) for o in ret_ids]
        spec["return_ids"] = ret_ids
        tr = sys.modules.get(_TRACING_MOD)
        if tr is not None and tr._exporter is not None:
            tr.inject(spec, spec.get("name", spec.get("method", "actor_task")),
                      {"ray.task_id": task_id.hex(), "ray.actor_id": actor_id.hex()})
        conn = self.actor_conns.get(actor_id)
        if conn is None:
            conn = self.actor_conns.setdefault(actor_id, ActorConn(self, actor_id, max_task_retries))
        if arg_refs:  # refs and actor handles nested inside inline args stay alive until the call is done
            have = {k.binary() for k in keep if isinstance(k, ObjectRef)}
            keep = list(keep) + [_ActorCallPin(self, r) if r[:1] == b"\xaa" and r[-3:] == b"\xaa\xaa\xaa"
                                 else ObjectRef(r) for r in arg_refs if r not in have]
        # flush ref deltas first so the actor never sees a ref the head does not know about
        self.send(None)
        conn.submit(spec, keep)
        return refs

    # ------------------------------------------------------------------ cancellation / gpu
    def _cancel_current(self, task_id):
        if self.current_task_id == task_id and self.main_thread_id is not None:
            ctypes.pythonapi.PyThreadState_SetAsyncExc(ctypes.c_ulong(self.main_thread_id),
                                                       ctypes.py_object(exc.TaskCancelledError))

    main_thread_id = None

    def _free_gpu(self, oids):
        from ray_memory_management_amd._private import gpu_object_store as gos

        for o in oids:
            gos.free(self, o)

    def record_event(self, ev: dict):
        with self.events_lock:
            self.events.append(ev)
            if len(self.events) >= 256:
                evs, self.events = self.events, []
                try:
                    self.send((P.EVENTS, evs))
                except Exception:
                    pass

    def flush_events(self):
        with self.events_lock:
            evs, self.events = self.events, []
        if evs:
            try:
                self.send((P.EVENTS, evs))
            except Exception:
                pass

    def shutdown(self):
        self._flusher_stop.set()
        try:
            if self.direct is not None:
                self.direct.flush()
            self.flush_events()
            self.send(None)
        except Exception:
            pass
        if self.direct is not None:
            self.direct.close()
        for c in self.actor_conns.values():
            c.close()
        try:
            self.sock.close()
        except OSError:
            pass


_gc_count = 0


def _collect_garbage():
    """Head-triggered global GC: drop unreachable ObjectRefs (reference cycles) so their objects
    can be freed under memory pressure (reference: CoreWorker::HandleLocalGC)."""
    global _gc_count
    import gc

    gc.collect()
    _gc_count += 1


def _is_cuda_tensor(v) -> bool:
    t = type(v)
    if t.__module__ != "torch" or t.__name__ not in ("Tensor", "Parameter"):
        return False
    try:
        return v.is_cuda
    except Exception:
        return False


# ====================================================================== driver bootstrap

_head_proc: Optional[subprocess.Popen] = None
_session_dir: Optional[str] = None
_local_mode = False


def _detect_gpus() -> int:
    """Count GPUs from the KFD topology without initialising HIP in this process."""
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in os.listdir(base):
            try:
                with open(os.path.join(base, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except OSError:
                continue
    except OSError:
        return 0
    if env is not None and env != "":
        n = min(n, len([x for x in env.split(",") if x != ""]))
    return n


def _default_store_size() -> int:
    try:
        import psutil

        total = psutil.virtual_memory().available
    except Exception:
        total = 8 << 30
    size = int(total * 0.3)
    try:
        st = os.statvfs("/dev/shm")
        shm_free = st.f_bavail * st.f_frsize
        size = min(size, int(shm_free * 0.9))
    except OSError:
        pass
    return max(64 << 20, min(size, 200 << 30))


_client = None  # util.client.ClientWorker when connected with ray.init("ray://host:port")
_TRACING_MOD = "ray_memory_management_amd.util.tracing.tracing_helper"  # loaded only when a hook is set
_system_config_used: dict = {}  # the _system_config this driver started its cluster with (ray._config)


# Keyword arguments of the reference's init (python/ray/_private/worker.py:1190-1213) beyond the named
# parameters. Supported ones act; the rest are accepted for compatibility and warn when set to a value this
# single-node runtime cannot honour. Anything else raises, as the reference does (worker.py:1256-1260).
_INIT_KWARGS_SUPPORTED = {"_memory", "_tracing_startup_hook", "_persistent", "dashboard_host", "dashboard_port",
                          "_enable_object_reconstruction", "job_config", "configure_logging", "logging_format",
                          "_skip_env_hook", "_node_name", "allow_multiple"}
_INIT_KWARGS_IGNORED = {"_redis_max_memory": None, "_plasma_directory": None, "_node_ip_address": ("127.0.0.1", None),
                        "_driver_object_store_memory": None, "_redis_password": None, "_metrics_export_port": None,
                        "_lru_evict": (False, None), "storage": None, "_java_worker_options": None}


def _check_init_kwargs(kwargs: dict) -> None:
    unknown = [k for k in kwargs if k not in _INIT_KWARGS_SUPPORTED and k not in _INIT_KWARGS_IGNORED]
    if unknown:
        raise RuntimeError(f"Unknown keyword argument(s): {', '.join(sorted(unknown))}")
    for k, v in kwargs.items():
        ok = _INIT_KWARGS_IGNORED.get(k, "supported")
        if ok == "supported":
            continue
        if v is None or (isinstance(ok, tuple) and v in ok):
            continue
        import warnings

        warnings.warn(f"ray.init({k}={v!r}) has no effect in this runtime (single-node shared-memory store under "
                      f"/dev/shm; no Redis, no external storage URI)", RuntimeWarning, stacklevel=3)


def is_initialized() -> bool:
    return global_worker is not None or _local_mode or _client is not None


def init(address: Optional[str] = None, *, num_cpus: Optional[int] = None, num_gpus: Optional[int] = None,
         resources: Optional[Dict[str, float]] = None, object_store_memory: Optional[int] = None,
         local_mode: bool = False, ignore_reinit_error: bool = False, namespace: Optional[str] = None,
         runtime_env: Optional[dict] = None, include_dashboard: Optional[bool] = None,
         logging_level=logging.INFO, log_to_driver: bool = True, _system_config: Optional[dict] = None,
         _temp_dir: Optional[str] = None, **kwargs):
    """Start (or connect to) a local cluster. Parity: reference python/ray/_private/worker.py:init."""
    global global_worker, _head_proc, _session_dir, _local_mode, _client
    _check_init_kwargs(kwargs)
    if _system_config and _system_config.get("object_spilling_config") is not None:
        from ray_memory_management_amd._private.external_storage import validate_spilling_config

        validate_spilling_config(_system_config["object_spilling_config"])  # raises before anything starts
    if isinstance(address, str) and address.startswith("ray://"):  # Ray Client mode
        with _init_lock:
            if is_initialized():
                if ignore_reinit_error:
                    return RayContext()
                raise RuntimeError("Maybe you called ray.init twice by accident?")
            from ray_memory_management_amd.util import client as _cl

            _client = _cl.connect(address, namespace)
            return RayContext()
    with _init_lock:
        if is_initialized():
            if ignore_reinit_error:
                return RayContext()
            raise RuntimeError("Maybe you called ray.init twice by accident? This error can be suppressed by "
                               "passing in 'ignore_reinit_error=True' or by calling 'ray.shutdown()' prior to 'ray.init()'.")
        if local_mode:
            from ray_memory_management_amd._private import local_mode as lm

            lm.start(num_cpus=num_cpus, num_gpus=num_gpus, resources=resources)
            _local_mode = True
            return RayContext()
        cfg = dict(_system_config or {})
        if kwargs.get("_tracing_startup_hook"):  # every worker of the job runs it too (RMM_CONFIG)
            cfg["_tracing_startup_hook"] = kwargs["_tracing_startup_hook"]
        global _system_config_used
        _system_config_used = dict(cfg)
        if address is None:  # jobs started by the job manager / `rmm start` users connect this way
            address = os.environ.get("RMM_ADDRESS") or None
        if address in ("auto",) or (address and address.startswith("rmm://")):
            sess = _find_session(address)
            head_sock = os.path.join(sess, "sockets", "head.sock")
            info = json.load(open(os.path.join(sess, "session.json")))
            store_name = info["store_name"]
            _session_dir = sess
        else:
            base = _temp_dir or os.path.join(tempfile.gettempdir(), "rmm")
            os.makedirs(base, exist_ok=True)
            sess = tempfile.mkdtemp(prefix=f"session_{time.strftime('%Y-%m-%d_%H-%M-%S')}_", dir=base)
            for sub in ("logs", "sockets", "spill"):
                os.makedirs(os.path.join(sess, sub), exist_ok=True)
            res = dict(resources or {})
            res["CPU"] = float(num_cpus if num_cpus is not None else (os.cpu_count() or 1))
            ng = num_gpus if num_gpus is not None else _detect_gpus()
            if ng:
                res["GPU"] = float(ng)
            osm = int(object_store_memory or _default_store_size())
            if kwargs.get("_memory") is not None:  # the node's schedulable `memory` resource (bytes)
                res["memory"] = float(kwargs["_memory"])
            try:
                import psutil

                res.setdefault("memory", float(int(psutil.virtual_memory().available * 0.7)))
            except Exception:
                pass
            res["object_store_memory"] = float(osm)
            store_name = f"/rmm-{uuid.uuid4().hex[:12]}"
            head_sock = os.path.join(sess, "sockets", "head.sock")
            env = dict(os.environ)
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
            # workers can import the driver's modules (reference: job code search path)
            env["RMM_DRIVER_SYS_PATH"] = json.dumps([p for p in sys.path if p and os.path.isdir(p)])
            cmd = [sys.executable, "-u", "-m", "ray_memory_management_amd._private.node", "--session-dir", sess,
                   "--store-name", store_name, "--object-store-memory", str(osm), "--resources", json.dumps(res),
                   "--config", json.dumps(cfg)]
            if kwargs.get("_persistent"):
                cmd.append("--persistent")
            log = open(os.path.join(sess, "logs", "head.log"), "ab")
            _head_proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                          start_new_session=True)
            log.close()
            ready = os.path.join(sess, "head.ready")
            t0 = time.time()
            while not os.path.exists(ready):
                if _head_proc.poll() is not None:
                    raise RuntimeError("head process failed to start:\n" +
                                       open(os.path.join(sess, "logs", "head.log")).read()[-4000:])
                if time.time() - t0 > 60:
                    raise RuntimeError("timed out starting the head process")
                time.sleep(0.005)
            with open(os.path.join(sess, "session.json"), "w") as f:
                json.dump({"store_name": store_name, "head_pid": _head_proc.pid}, f)
            _session_dir = sess
            with open(os.path.join(base, "latest_session"), "w") as f:
                f.write(sess)
        ns = namespace or f"anon-{uuid.uuid4().hex[:8]}"
        w = CoreWorker(SCRIPT_MODE, head_sock, store_name, sess, namespace=ns)
        w.main_thread_id = threading.main_thread().ident
        info = w.request(lambda rid: (P.REGISTER, "driver", {"pid": os.getpid(), "job_id": w.job_id,
                                                             "namespace": ns, "req_id": rid}))
        w.config = info.get("config", {})
        w.job_runtime_env = runtime_env
        hook = kwargs.get("_tracing_startup_hook") or w.config.get("_tracing_startup_hook")
        if hook:
            from ray_memory_management_amd.util.tracing.tracing_helper import _setup_tracing

            _setup_tracing(hook)
        global_worker = w
        _set_worker(w)
        atexit.register(shutdown)
        if include_dashboard and _head_proc is not None:
            _start_dashboard(sess, kwargs.get("dashboard_host", "127.0.0.1"), int(kwargs.get("dashboard_port", 8265)))
        return RayContext()


_dashboard_proc = None
_dashboard_url = None


def _start_dashboard(sess: str, host: str, port: int):
    """Launch the dashboard process (dashboard/head.py) next to the head; it connects as a client
    driver. Parity: reference ray.init(include_dashboard=True, dashboard_host, dashboard_port)."""
    global _dashboard_proc, _dashboard_url
    ready = os.path.join(sess, "dashboard.json")
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    log = open(os.path.join(sess, "logs", "dashboard.log"), "ab")
    _dashboard_proc = subprocess.Popen(
        [sys.executable, "-u", "-m", "ray_memory_management_amd.dashboard", "--address", f"rmm://{sess}",
         "--host", host, "--port", str(port), "--ready-file", ready],
        env=env, stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True)
    log.close()
    t0 = time.time()
    while not os.path.exists(ready):
        if _dashboard_proc.poll() is not None or time.time() - t0 > 60:
            logger.warning("dashboard failed to start; see %s", os.path.join(sess, "logs", "dashboard.log"))
            _dashboard_proc = None
            return
        time.sleep(0.01)
    _dashboard_url = json.load(open(ready))["url"]


def _stop_dashboard():
    global _dashboard_proc, _dashboard_url
    p, _dashboard_proc, _dashboard_url = _dashboard_proc, None, None
    if p is not None and p.poll() is None:
        p.terminate()
        try:
            p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def _find_session(address):
    if address and address.startswith("rmm://"):
        return address[len("rmm://"):]
    base = os.path.join(tempfile.gettempdir(), "rmm")
    with open(os.path.join(base, "latest_session")) as f:
        return f.read().strip()


def _shm_unlink(name: str) -> None:
    """Remove this session's store segment name (processes that still map it keep their mapping)."""
    try:
        from _posixshmem import shm_unlink

        shm_unlink(name)
    except (ImportError, OSError):
        pass


def shutdown(_exiting_interpreter: bool = False):
    global global_worker, _head_proc, _local_mode, _client
    tr = sys.modules.get(_TRACING_MOD)
    if tr is not None:  # the hook was this job's: the next init() installs its own
        tr.set_exporter(None)
        tr._setup_tracing._done = None
    with _init_lock:
        if _client is not None:
            _client.close()
            _client = None
            return
        if _local_mode:
            from ray_memory_management_amd._private import local_mode as lm

            lm.stop()
            _local_mode = False
            return
        w = global_worker
        if w is None:
            return
        from ray_memory_management_amd._private import gpu_object_store as gos

        gos.shutdown_process_store(w)
        _stop_dashboard()
        if _head_proc is not None:
            try:
                w.send((P.SHUTDOWN,))
            except Exception:
                pass
        w.shutdown()
        global_worker = None
        _set_worker(None)
        if _head_proc is not None:
            try:
                _head_proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                _head_proc.kill()
                _head_proc.wait()
                _shm_unlink(w.store_name)  # the head this driver started could not clean up its segment
            _head_proc = None


class RayContext(dict):
    def __init__(self):
        super().__init__(session_dir=_session_dir, address=f"rmm://{_session_dir}" if _session_dir else None,
                         dashboard_url=_dashboard_url)
        self.address_info = dict(self)
        self.dashboard_url = _dashboard_url

    def __enter__(self):
        return self

    def __exit__(self, *a):
        shutdown()


def _require_worker() -> CoreWorker:
    if global_worker is None:
        if _local_mode:
            raise RuntimeError("local mode worker")
        # auto-init like the reference
        init()
    return global_worker


# ====================================================================== public API

def put(value, *, _owner=None) -> ObjectRef:
    if _client is not None:
        return _client.put(value)
    if _local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return lm.put(value)
    return _require_worker().put_object(value)


def get(object_refs, *, timeout: Optional[float] = None):
    if _client is not None:
        return _client.get(object_refs, timeout)
    if _local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return lm.get(object_refs, timeout)
    w = _require_worker()
    from ray_memory_management_amd.object_ref import ObjectRefGenerator

    if isinstance(object_refs, ObjectRefGenerator):
        object_refs = list(object_refs)
    if isinstance(object_refs, ObjectRef):
        return w.get([object_refs], timeout)[0]
    if isinstance(object_refs, (list, tuple)):
        return w.get(list(object_refs), timeout)
    raise ValueError("'object_refs' must either be an ObjectRef or a list of ObjectRefs.")


def wait(object_refs, *, num_returns: int = 1, timeout: Optional[float] = None, fetch_local: bool = True):
    if _client is not None:
        return _client.wait(object_refs, num_returns, timeout)
    if _local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return lm.wait(object_refs, num_returns, timeout)
    if isinstance(object_refs, ObjectRef):
        raise TypeError("wait() expected a list of ObjectRef, got a single ObjectRef")
    object_refs = list(object_refs)
    if len(set(object_refs)) != len(object_refs):
        raise ValueError("Wait requires a list of unique object refs.")
    if num_returns <= 0:
        raise ValueError("Invalid number of objects to return %d." % num_returns)
    if num_returns > len(object_refs):
        raise ValueError("num_returns cannot be greater than the number of objects provided.")
    if timeout is not None and timeout < 0:
        raise ValueError(f"The 'timeout' argument must be nonnegative. Received {timeout}")
    for r in object_refs:
        if not isinstance(r, ObjectRef):
            raise TypeError(f"wait() expected a list of ray.ObjectRef, got list containing {type(r)}")
    return _require_worker().wait(object_refs, num_returns, timeout, fetch_local)


def kill(actor, *, no_restart: bool = True):
    from ray_memory_management_amd.actor import ActorHandle

    if _client is not None:
        return _client.kill(actor, no_restart)
    if not isinstance(actor, ActorHandle):
        raise ValueError("ray.kill() only supported for actors. Got: {}.".format(type(actor)))
    if _local_mode:
        return
    w = _require_worker()
    w.send((P.KILL_ACTOR, actor._actor_id, no_restart))
    if no_restart:
        # calls submitted by this process after kill() fail deterministically
        conn = w.actor_conns.setdefault(actor._actor_id, ActorConn(w, actor._actor_id, 0))
        with conn.lock:
            conn.dead_error = exc.RayActorError(actor._actor_id.hex(), "The actor was killed by ray.kill().")


def cancel(object_ref: ObjectRef, *, force: bool = False, recursive: bool = True):
    if _client is not None:
        return _client.cancel(object_ref, force)
    if not isinstance(object_ref, ObjectRef):
        raise TypeError("ray.cancel() only supported for non-actor object refs.")
    if _local_mode:
        return
    w = _require_worker()
    tid = object_ref.binary()[:16]
    for conn in list(w.actor_conns.values()):  # a call still queued / in flight to an actor
        with conn.lock:
            specs = [e[0] for e in conn.inflight.values()] + [e[0] for e in conn.queued]
        if any(sp.get("task_id") == tid for sp in specs):
            raise TypeError("ray.cancel() only supported for non-actor object refs.")
    if w.direct is not None and w.direct.cancel(object_ref.binary()[:16], force):
        return
    w.send((P.CANCEL, object_ref.binary()[:16], force, recursive))


def get_actor(name: str, namespace: Optional[str] = None):
    from ray_memory_management_amd.actor import ActorHandle

    if not name:
        raise ValueError("Please supply a non-empty value to get_actor")
    if _client is not None:
        return _client.get_actor(name, namespace)
    w = _require_worker()
    ns = namespace if namespace is not None else w.namespace
    spec = w.request(lambda rid: (P.GET_ACTOR, rid, name, ns))
    if spec is None:
        raise ValueError(f"Failed to look up actor with name '{name}'. This could because 1. You are trying to look "
                         f"up a named actor you didn't create. 2. The named actor died. 3. You did not use a namespace "
                         f"matching the namespace of the actor.")
    return ActorHandle._from_spec(spec)


def get_gpu_ids():
    if _local_mode:
        return []
    w = _require_worker()
    return list(w.gpu_ids)


def remote(*args, **kwargs):
    from ray_memory_management_amd.actor import make_actor_class
    from ray_memory_management_amd.remote_function import RemoteFunction

    def make(obj, opts):
        import inspect

        if inspect.isclass(obj):
            return make_actor_class(obj, opts)
        if callable(obj):
            return RemoteFunction(obj, opts)
        raise TypeError("The @remote decorator must be applied to either a function or a class.")

    if len(args) == 1 and not kwargs and callable(args[0]):
        return make(args[0], {})
    if args:
        raise TypeError("The @remote decorator must be applied either with no arguments and no parentheses, "
                        "for example '@remote', or it must be applied using some of the arguments like "
                        "'@remote(num_returns=2, resources={\"CustomResource\": 1})'.")
    return lambda obj: make(obj, kwargs)


def timeline(filename: Optional[str] = None):
    """Chrome-trace events of task execution. Parity: reference python/ray/_private/state.py:timeline."""
    w = _require_worker()
    w.flush_events()
    time.sleep(0.05)
    evs = w.request(lambda rid: (P.STATE, rid, "timeline", None))
    if filename:
        with open(filename, "w") as f:
            json.dump(evs, f)
        return None
    return evs


def _state(what, arg=None):
    w = _require_worker()
    return w.request(lambda rid: (P.STATE, rid, what, arg))


def cluster_resources():
    if _client is not None:
        return _client.cluster_resources()
    if _local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return lm.resources()
    return _state("cluster_resources")


def available_resources():
    if _client is not None:
        return _client.available_resources()
    if _local_mode:
        from ray_memory_management_amd._private import local_mode as lm

        return lm.resources()
    return _state("available_resources")


def nodes():
    if _client is not None:
        return _client.nodes()
    return _state("nodes")
