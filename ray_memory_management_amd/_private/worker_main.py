"""Worker process: executes normal tasks dispatched by the head, or hosts one actor.

Parity: reference python/ray/_private/workers/default_worker.py + the execution half of
python/ray/_raylet.pyx (execute_task, store task outputs, actor creation, async/threaded actors,
concurrency groups) and src/ray/core_worker/transport/direct_actor_transport.cc (actor task
receiving, in-order execution per caller).
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import inspect
import json
import os
import queue
import socket
import sys
import threading
import time
import traceback

import cloudpickle

from ray_memory_management_amd import exceptions as exc
from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import serialization as ser
from ray_memory_management_amd._private import worker as _w
from ray_memory_management_amd._private.ids import object_id_for_return
from ray_memory_management_amd.object_ref import ObjectRef, _set_worker


def _apply_runtime_env():
    spec = os.environ.get("RMM_RUNTIME_ENV")
    if not spec:
        return
    env = json.loads(spec)
    wd = env.get("working_dir")
    if wd and os.path.isdir(wd):
        os.chdir(wd)
        sys.path.insert(0, wd)
    for m in env.get("py_modules") or []:
        if os.path.isdir(m):
            sys.path.insert(0, os.path.dirname(os.path.abspath(m)))
            sys.path.insert(0, m)


class Executor:
    def __init__(self, w: _w.CoreWorker):
        self.w = w
        self.fns = {}
        self.call_counts = collections.Counter()
        self.actor = None
        self.actor_spec = None
        self.actor_server = None
        self.actor_q: "queue.Queue" = queue.Queue()
        self.pool = None
        self.group_pools = {}
        self.loop = None
        self.exiting = False
        self.pid = os.getpid()
        self.cancelled_direct = set()
        self.pending_blobs = {}
        self.pending_acks = {}  # direct conn -> [lock, [ack, ...]]
        self.acks_since = 0.0

    # ------------------------------------------------------------------ direct task socket
    def start_direct_server(self) -> str:
        """Listening socket owners push leased tasks to (reference: the worker's gRPC
        CoreWorkerService PushTask endpoint)."""
        path = os.path.join(self.w.session_dir, "sockets", f"w-{self.w.worker_id.hex()[:20]}.sock")
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(path)
        srv.listen(64)
        threading.Thread(target=self._direct_accept, args=(srv,), daemon=True, name="rmm-direct-accept").start()
        return path

    def flush_acks(self):
        self.acks_since = 0.0
        for s, (lock, acks) in list(self.pending_acks.items()):
            if acks:
                batch = list(acks)
                acks.clear()
                try:
                    P.send(s, (P.REPLY, 0, batch), lock)
                except OSError:
                    pass

    def bounce_direct(self):
        """The running task blocked in get(): hand every queued, unstarted direct task back to its
        owner (status "requeue") so it runs elsewhere instead of waiting behind the blocked one."""
        self.flush_acks()
        q = self.w.task_queue
        with q.mutex:
            bounce = [m for m in q.queue if m[0] == P.DIRECT_TASK]
            if not bounce:
                return
            rest = [m for m in q.queue if m[0] != P.DIRECT_TASK]
            q.queue.clear()
            q.queue.extend(rest)
        for _, s, lock, spec, blob, info in bounce:
            if blob is not None:
                self.pending_blobs[spec["fn_id"]] = blob  # the owner will not resend it on this conn
            try:
                P.send(s, (P.REPLY, 0, [(spec["task_id"], "requeue", 0.0, 0.0)]), lock)
            except OSError:
                pass

    def _direct_accept(self, srv):
        while True:
            try:
                s, _ = srv.accept()
            except OSError:
                return
            threading.Thread(target=self._direct_conn, args=(s,), daemon=True, name="rmm-direct").start()

    def _direct_conn(self, s):
        lock = threading.Lock()
        rd = P.FrameReader()
        try:
            while True:
                data = s.recv(1 << 16)
                if not data:
                    return
                for m in rd.feed(data):
                    if m[0] == P.DIRECT_TASK:
                        info = m[2]
                        for spec, blob, attempt in m[1]:
                            self.w.task_queue.put((P.DIRECT_TASK, s, lock, spec, blob,
                                                   {**info, "attempt": attempt}))
                    elif m[0] == P.CANCEL_TASK:
                        if self.w.current_task_id == m[1]:
                            self.w._cancel_current(m[1])
                        else:
                            self.cancelled_direct.add(m[1])
        except (OSError, EOFError):
            pass

    # ------------------------------------------------------------------ argument handling
    def resolve(self, enc):
        kind, v = enc
        if kind == "v":
            return ser.loads_inline(v)
        if kind == "b":
            return ser.deserialize(v[0], v[1])
        return self.w.get([ObjectRef(v)])[0]

    def resolve_all(self, args, kwargs):
        # fetch all by-ref args in one batched get so errors surface in order
        return [self.resolve(a) for a in args], {k: self.resolve(v) for k, v in kwargs.items()}

    # ------------------------------------------------------------------ outputs
    def store_outputs(self, return_ids, num_returns, result, contained_map, holds):
        if num_returns == 0:
            return
        if num_returns == "dynamic":
            refs = []
            tid = return_ids[0][:16]
            for i, v in enumerate(result):
                oid = object_id_for_return(tid, 1000 + i)
                self._put_value(oid, v, contained_map, holds)
                refs.append(ObjectRef(oid))
            from ray_memory_management_amd.object_ref import ObjectRefGenerator

            self._put_value(return_ids[0], ObjectRefGenerator(refs), contained_map, holds)
            holds.extend(refs)
            return
        if num_returns == 1:
            values = [result]
        else:
            if not isinstance(result, (tuple, list)) or len(result) != num_returns:
                raise ValueError(f"Task returned {result!r} but num_returns={num_returns}")
            values = list(result)
        for oid, v in zip(return_ids, values):
            self._put_value(oid, v, contained_map, holds)

    def _put_value(self, oid, v, contained_map, holds):
        if _w._is_cuda_tensor(v) and self.w.config.get("gpu_object_store", True):
            from ray_memory_management_amd._private import gpu_object_store as gos

            gos.put_tensor(self.w, oid, v)
            self.w.send((P.GPU_OBJECT, oid))
            return
        with self.w.gpu_sink():
            data, bufs, contained = ser.serialize(v)
        if contained:
            contained_map[oid] = contained
            for c in contained:  # keep inner objects alive until TASK_DONE reached the head
                holds.append(ObjectRef(c))
        if not self.w.store.put_serialized(oid, data, bufs, ser.TAG_PICKLE, False):
            pass  # already exists (retry of a task whose output survived)

    def store_error(self, return_ids, err):
        data, bufs, _ = ser.serialize(err)
        for oid in return_ids:
            try:
                self.w.store.put_serialized(oid, data, bufs, ser.TAG_ERROR, True)
            except Exception:
                pass

    # ------------------------------------------------------------------ normal tasks
    def execute(self, spec, blob, info):
        status, contained_map, holds, t0, t1, exit_after = self._run(spec, blob, info)
        self.w.send((P.TASK_DONE, spec["task_id"], status, contained_map, {"exit": exit_after}))
        del holds
        if exit_after:
            self.w.flush_events()
            os._exit(0)

    def execute_direct(self, s, lock, spec, blob, info):
        """A task pushed by its owner over a lease (direct task transport): outputs go to the store
        as usual, nested-ref bookkeeping to the head, and the completion ack to the owner."""
        tid = spec["task_id"]
        if tid in self.cancelled_direct:
            self.cancelled_direct.discard(tid)
            self.store_error(spec["return_ids"], exc.TaskCancelledError(tid.hex()))
            t = time.time()
            status, contained_map, holds, t0, t1, exit_after = "err", {}, [], t, t, False
        else:
            if self.acks_since and time.time() - self.acks_since > 0.001:
                self.flush_acks()  # never hold finished acks across a task that may run long
            status, contained_map, holds, t0, t1, exit_after = self._run(spec, blob, info)
        for outer, inners in contained_map.items():
            self.w.send((P.CONTAINED, outer, inners))
        if contained_map:
            self.w.send(None)
        # acks are coalesced while more direct work is queued (one frame per burst)
        acks = self.pending_acks.setdefault(s, [lock, []])
        acks[1].append((tid, status, t0, t1))
        if not self.acks_since:
            self.acks_since = time.time()
        if len(acks[1]) >= 16 or self.w.task_queue.empty():
            self.flush_acks()
        del holds
        if exit_after:
            self.w.flush_events()
            os._exit(0)

    def _run(self, spec, blob, info):
        w = self.w
        fid = spec["fn_id"]
        fn = self.fns.get(fid)
        if fn is None:
            if blob is None:
                blob = self.pending_blobs.pop(fid, None)
            if blob is None:
                raise RuntimeError("function blob missing")
            fn = cloudpickle.loads(blob)
            self.fns[fid] = fn
        w.enter_job(spec.get("job_id"))
        w.assigned_resources = spec.get("resources")
        w.current_task_id = spec["task_id"]
        w.current_task_name = spec.get("name")
        w.gpu_ids = list(info.get("gpu_ids") or [])
        if w.gpu_ids:
            vis = ",".join(map(str, w.gpu_ids))
            if os.environ.get("HIP_VISIBLE_DEVICES") is None:
                os.environ["HIP_VISIBLE_DEVICES"] = vis
                os.environ["CUDA_VISIBLE_DEVICES"] = vis
        st = spec.get("strategy") or {}
        w.placement_group_capture = None
        if st.get("type") == "PLACEMENT_GROUP" and st.get("capture"):
            from ray_memory_management_amd.util.placement_group import PlacementGroup
            from ray_memory_management_amd._private.ids import PlacementGroupID

            w.placement_group_capture = PlacementGroup(PlacementGroupID(st["pg_id"]))
        env_vars = (spec.get("runtime_env") or {}).get("env_vars") or {}
        saved_env = {k: os.environ.get(k) for k in env_vars}
        for k, v in env_vars.items():
            os.environ[str(k)] = str(v)
        status = "ok"
        contained_map = {}
        holds = []
        t0 = time.time()
        try:
            try:
                args, kwargs = self.resolve_all(spec["args"], spec["kwargs"])
            except exc.RayTaskError as e:
                # an argument was an error object: propagate it as this task's output
                self.store_error(spec["return_ids"], e)
                status = "err"
                raise _Handled()
            except exc.RayError as e:
                self.store_error(spec["return_ids"], e)
                status = "err"
                raise _Handled()
            if "_trace_ctx" in spec:
                from ray_memory_management_amd.util.tracing.tracing_helper import execution_span

                with execution_span(spec, spec.get("name", "task"), {"ray.task_id": spec["task_id"].hex()}):
                    result = fn(*args, **kwargs)
            else:
                result = fn(*args, **kwargs)
            if inspect.isgenerator(result) and spec.get("num_returns") not in ("dynamic",):
                result = list(result) if spec.get("num_returns", 1) != 1 else list(result)
            self.store_outputs(spec["return_ids"], spec.get("num_returns", 1), result, contained_map, holds)
        except _Handled:
            pass
        except exc.TaskCancelledError:
            self.store_error(spec["return_ids"], exc.TaskCancelledError(spec["task_id"].hex()))
            status = "err"
        except KeyboardInterrupt:
            self.store_error(spec["return_ids"], exc.TaskCancelledError(spec["task_id"].hex()))
            status = "err"
        except BaseException as e:  # noqa: BLE001
            if isinstance(e, SystemExit) and not isinstance(e, Exception):
                self.exiting = True
            retry_ex = spec.get("retry_exceptions", False)
            retryable = (retry_ex is True or (isinstance(retry_ex, (list, tuple)) and isinstance(e, tuple(retry_ex))))
            max_retries = spec.get("max_retries", 0)
            if retryable and (max_retries < 0 or info.get("attempt", 0) < max_retries):
                status = "retry"
            else:
                err = exc.RayTaskError.from_exception(e, spec.get("name", "task"), pid=self.pid)
                self.store_error(spec["return_ids"], err)
                status = "err"
        finally:
            for k, v in saved_env.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            w.current_task_id = None
            w.placement_group_capture = None
        t1 = time.time()
        w.record_event({"cat": "task", "name": spec.get("name", "task"), "ph": "X", "pid": f"node{info.get('node_id', 1)}",
                        "tid": f"worker {self.pid}", "ts": t0 * 1e6, "dur": (t1 - t0) * 1e6,
                        "args": {"task_id": spec["task_id"].hex(), "status": status}})
        self.call_counts[fid] += 1
        mc = spec.get("max_calls", 0)
        exit_after = bool(mc and self.call_counts[fid] >= mc) or self.exiting
        return status, contained_map, holds, t0, t1, exit_after

    # ------------------------------------------------------------------ actors
    def create_actor(self, spec, blob, info):
        w = self.w
        self.actor_spec = spec
        w.current_actor_id = spec["actor_id"]
        w.enter_job(spec.get("job_id"))
        w.actor_restart_count = int(info.get("restart") or 0)
        w.assigned_resources = spec.get("resources")
        w.gpu_ids = list(info.get("gpu_ids") or [])
        for k, v in ((spec.get("runtime_env") or {}).get("env_vars") or {}).items():
            os.environ[str(k)] = str(v)
        st = spec.get("strategy") or {}
        if st.get("type") == "PLACEMENT_GROUP" and st.get("capture"):
            from ray_memory_management_amd.util.placement_group import PlacementGroup
            from ray_memory_management_amd._private.ids import PlacementGroupID

            w.placement_group_capture = PlacementGroup(PlacementGroupID(st["pg_id"]))
        try:
            cls = cloudpickle.loads(blob) if blob is not None else None
            if cls is None:
                raise RuntimeError("actor class blob missing")
            args, kwargs = self.resolve_all(spec["args"], spec["kwargs"])
            from ray_memory_management_amd.actor import ActorHandle

            w.actor_handle_for_self = ActorHandle(spec["actor_id"], spec["class_name"], spec["method_meta"],
                                                  spec.get("max_task_retries", 0), _count=False)
            self.actor = cls.__new__(cls)
            self.actor.__init__(*args, **kwargs)
        except BaseException as e:  # noqa: BLE001
            err = exc.RayTaskError.from_exception(e, f"{spec['class_name']}.__init__", pid=self.pid)
            w.send((P.ACTOR_FAILED_INIT, spec["actor_id"], ser.dumps_inline(err)[0]))
            time.sleep(0.2)
            os._exit(1)
        max_conc = spec.get("max_concurrency", 1)
        if spec.get("is_async"):
            self.loop = asyncio.new_event_loop()
            self.sem = None
            threading.Thread(target=self._run_loop, args=(max_conc,), daemon=True).start()
        elif max_conc > 1:
            self.pool = concurrent.futures.ThreadPoolExecutor(max_conc)
        for g, n in (spec.get("concurrency_groups") or {}).items():
            if not spec.get("is_async"):
                self.group_pools[g] = concurrent.futures.ThreadPoolExecutor(int(n))
        path = os.path.join(w.session_dir, "sockets", f"actor-{spec['actor_id'].hex()}-{self.pid}.sock")
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(path)
        srv.listen(256)
        self.actor_server = srv
        threading.Thread(target=self._accept_loop, args=(srv,), daemon=True).start()
        w.send((P.ACTOR_READY, spec["actor_id"], path))

    def _run_loop(self, max_conc):
        asyncio.set_event_loop(self.loop)
        self.sem = asyncio.Semaphore(max_conc)
        self.loop.run_forever()

    def _accept_loop(self, srv):
        while True:
            try:
                s, _ = srv.accept()
            except OSError:
                return
            threading.Thread(target=self._conn_loop, args=(s,), daemon=True).start()

    def _conn_loop(self, s):
        lock = threading.Lock()
        try:
            while True:
                m = P.recv(s)
                if m[0] == P.ACTOR_TASK:
                    self.actor_q.put((s, lock, m[1]))
        except (ConnectionError, OSError, EOFError):
            pass

    def _ack(self, s, lock, seq):
        try:
            P.send(s, (P.REPLY, 0, [seq]), lock)
        except OSError:
            pass

    def run_actor_task(self, s, lock, spec):
        w = self.w
        borrowed = False
        name = spec["method"]
        ret_ids = spec["return_ids"]
        t0 = time.time()
        holds = []
        contained_map = {}
        try:
            if name == "__ray_terminate__":
                self._ack(s, lock, spec["seq"])
                self.store_outputs(ret_ids, 1, None, contained_map, holds)
                w.flush_events()
                w.send(None)
                os._exit(0)
            if name == "__ray_ready__":
                result = True
            else:
                _w.actor_task_id.set(spec["task_id"])
                args, kwargs = self.resolve_all(spec["args"], spec["kwargs"])
                borrowed = w.pending_borrows()  # refs taken out of the caller's arguments
                t_res = time.time()
                m = getattr(self.actor, name)
                if "_trace_ctx" in spec:
                    from ray_memory_management_amd.util.tracing.tracing_helper import execution_span

                    with execution_span(spec, spec.get("name", name), {"ray.task_id": spec["task_id"].hex()}):
                        result = m(*args, **kwargs)
                else:
                    result = m(*args, **kwargs)
                if inspect.iscoroutine(result):
                    raise RuntimeError("coroutine returned from a non-async actor path")
                t_ret = time.time()
            self.store_outputs(ret_ids, spec.get("num_returns", 1), result, contained_map, holds)
            st = getattr(w, "task_stamps", None)
            if st is not None and name not in ("__ray_ready__",):
                # (method, arrived, args resolved, method returned, outputs stored): hand-off probes
                st.append((name, t0, t_res, t_ret, time.time()))
        except BaseException as e:  # noqa: BLE001
            from ray_memory_management_amd.actor import _ActorExit

            if isinstance(e, _ActorExit):
                self.store_outputs(ret_ids, spec.get("num_returns", 1), None, contained_map, holds)
                self._ack(s, lock, spec["seq"])
                w.send((P.ACTOR_EXITING, spec.get("actor_id") or w.current_actor_id))
                w.flush_events()
                w.send(None)
                time.sleep(0.05)
                os._exit(0)
            if isinstance(e, exc.RayError) and not isinstance(e, exc.RayTaskError) and name != "__init__":
                self.store_error(ret_ids, e)
            else:
                self.store_error(ret_ids, exc.RayTaskError.from_exception(e, spec.get("name", name), pid=self.pid))
        if contained_map:
            for outer, inners in contained_map.items():
                w.send((P.CONTAINED, outer, inners))
        t1 = time.time()
        w.record_event({"cat": "actor_task", "name": spec.get("name", name), "ph": "X", "pid": "actors",
                        "tid": f"actor {self.pid}", "ts": t0 * 1e6, "dur": (t1 - t0) * 1e6})
        if borrowed:  # borrows taken from the call's arguments reach the head before the caller may drop its refs
            w.flush_refs_sync()
        self._ack(s, lock, spec["seq"])
        del holds

    async def run_async_actor_task(self, s, lock, spec):
        async with self.sem:
            borrowed = False
            name = spec["method"]
            ret_ids = spec["return_ids"]
            holds, contained_map = [], {}
            try:
                if name == "__ray_ready__":
                    result = True
                elif name == "__ray_terminate__":
                    self.store_outputs(ret_ids, 1, None, contained_map, holds)
                    self._ack(s, lock, spec["seq"])
                    os._exit(0)
                else:
                    _w.actor_task_id.set(spec["task_id"])
                    loop = asyncio.get_running_loop()
                    args, kwargs = await loop.run_in_executor(None, self.resolve_all, spec["args"], spec["kwargs"])
                    borrowed = self.w.pending_borrows()
                    m = getattr(self.actor, name)
                    result = m(*args, **kwargs)
                    if inspect.isawaitable(result):
                        result = await result
                self.store_outputs(ret_ids, spec.get("num_returns", 1), result, contained_map, holds)
            except BaseException as e:  # noqa: BLE001
                from ray_memory_management_amd.actor import _ActorExit

                if isinstance(e, _ActorExit):
                    self._ack(s, lock, spec["seq"])
                    self.w.send((P.ACTOR_EXITING, self.w.current_actor_id))
                    os._exit(0)
                self.store_error(ret_ids, exc.RayTaskError.from_exception(e, spec.get("name", name), pid=self.pid))
            if contained_map:
                for outer, inners in contained_map.items():
                    self.w.send((P.CONTAINED, outer, inners))
            if borrowed and self.w.pending_borrows():  # see run_actor_task
                await asyncio.get_running_loop().run_in_executor(None, self.w.flush_refs_sync)
            self._ack(s, lock, spec["seq"])

    def actor_loop(self):
        while True:
            s, lock, spec = self.actor_q.get()
            if self.loop is not None:
                asyncio.run_coroutine_threadsafe(self.run_async_actor_task(s, lock, spec), self.loop)
                continue
            g = spec.get("concurrency_group")
            if g and g in self.group_pools:
                self.group_pools[g].submit(self.run_actor_task, s, lock, spec)
            elif self.pool is not None:
                self.pool.submit(self.run_actor_task, s, lock, spec)
            else:
                self.run_actor_task(s, lock, spec)


class _Handled(Exception):
    pass


def main():
    import faulthandler
    import signal as _signal

    # `rmm stack` / debugging: SIGUSR1 dumps every thread's stack into this worker's log
    faulthandler.register(_signal.SIGUSR1, all_threads=True)
    for p in json.loads(os.environ.get("RMM_DRIVER_SYS_PATH", "[]")):
        if p not in sys.path:
            sys.path.append(p)
    _apply_runtime_env()
    head = os.environ["RMM_HEAD_SOCKET"]
    store = os.environ["RMM_STORE_NAME"]
    sess = os.environ["RMM_SESSION_DIR"]
    wid = bytes.fromhex(os.environ["RMM_WORKER_ID"])
    node = int(os.environ.get("RMM_NODE_ID", "1"))
    w = _w.CoreWorker(_w.WORKER_MODE, head, store, sess, worker_id=wid, node_id=node)
    w.main_thread_id = threading.main_thread().ident
    _w.global_worker = w
    _set_worker(w)
    hook = w.config.get("_tracing_startup_hook")
    if hook:  # the job's tracing setup (reference: _tracing_startup_hook run in every worker)
        try:
            from ray_memory_management_amd.util.tracing.tracing_helper import _setup_tracing

            _setup_tracing(hook)
        except Exception as e:  # noqa: BLE001
            print(f"tracing startup hook {hook!r} failed: {e!r}", file=sys.stderr)
    ex = Executor(w)
    direct_addr = ex.start_direct_server()
    w.on_block = ex.bounce_direct
    w.send((P.REGISTER, "worker", {"worker_id": wid, "pid": os.getpid(), "direct_addr": direct_addr}))
    info = None
    prof_dir = os.environ.get("RMM_WORKER_PROFILE_DIR")  # control-plane profiling: cProfile per worker
    prof = None
    if prof_dir:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    while True:
        m = w.task_queue.get()
        t = m[0]
        if t == P.EXECUTE:
            try:
                ex.execute(m[1], m[2], m[3])
            except KeyboardInterrupt:
                pass
        elif t == P.DIRECT_TASK:
            try:
                ex.execute_direct(m[1], m[2], m[3], m[4], m[5])
            except KeyboardInterrupt:
                pass
        elif t == P.CREATE_ACTOR_INSTANCE:
            ex.create_actor(m[1], m[2], m[3])
            threading.Thread(target=_drain_head_queue, args=(w,), daemon=True).start()
            ex.actor_loop()
        elif t == P.EXIT:
            break
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.path.join(prof_dir, f"worker-{os.getpid()}.prof"))
    w.flush_events()
    w.shutdown()
    os._exit(0)


def _drain_head_queue(w):
    while True:
        m = w.task_queue.get()
        if m[0] == P.EXIT:
            w.flush_events()
            os._exit(0)


if __name__ == "__main__":
    main()
