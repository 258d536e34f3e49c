"""Head node process: GCS + raylet roles for one machine (plus virtual nodes for tests).

Parity (behaviour, re-designed): reference src/ray/raylet/node_manager.cc (task dispatch, worker
lifecycle, blocked-worker resource release), src/ray/raylet/worker_pool.cc (process pool keyed by
runtime env), src/ray/raylet/local_task_manager.cc (dispatch queue), src/ray/gcs/gcs_server/
{gcs_actor_manager,gcs_placement_group_manager,gcs_kv_manager,gcs_job_manager}.cc,
src/ray/core_worker/reference_count.cc (we count centrally: every process reports batched
deltas), src/ray/core_worker/task_manager.cc (retries), src/ray/raylet/local_object_manager.cc
(threshold spilling), python/ray/_private/memory_monitor.py.

Design: ONE event-loop thread owns all state. Heavy lifting is native: the C++ scheduler
(`_sched`) decides placement/resources/dependencies; the shared-memory store (`_store`) is the
data plane — object seals reach this loop through the store's sealed-object ring (a watcher thread
blocks on the in-segment condvar and pokes the loop through a self-pipe).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import pickle
import selectors
import signal
import socket
import subprocess
import sys
import threading
import time
import traceback
from typing import Any, Dict, List, Optional

from ray_memory_management_amd._native import sched_ext, store_ext
from ray_memory_management_amd._private import protocol as P
from ray_memory_management_amd._private import serialization as ser
from ray_memory_management_amd._private.ids import ID_SIZE, object_id_for_return
from ray_memory_management_amd import exceptions as exc

PENDING, RUNNING, FINISHED, FAILED, CANCELLED = "PENDING", "RUNNING", "FINISHED", "FAILED", "CANCELLED"
ACTOR_PENDING, ACTOR_ALIVE, ACTOR_RESTARTING, ACTOR_DEAD = (
    "PENDING_CREATION", "ALIVE", "RESTARTING", "DEAD")


def actor_ref_key(actor_id: bytes) -> bytes:
    """Pseudo object id used to reference-count actor handles."""
    return b"\xaa" + actor_id[:16] + b"\xaa\xaa\xaa"


def _is_actor_key(oid: bytes) -> bool:
    return oid[:1] == b"\xaa" and oid[-3:] == b"\xaa\xaa\xaa"


def pg_rewrite(res: dict, pg_hex: str, bidx: int) -> dict:
    """Resources of a task placed in a bundle: the derived per-bundle names the native scheduler
    commits when the group is placed (reference naming, bundle_spec.cc)."""
    out = {}
    for k, v in res.items():
        if v <= 0:
            continue
        out[f"{k}_group_{bidx}_{pg_hex}" if bidx >= 0 else f"{k}_group_{pg_hex}"] = v
    out[f"bundle_group_{bidx}_{pg_hex}" if bidx >= 0 else f"bundle_group_{pg_hex}"] = 0.001
    return out


def _cpu_part(res: dict) -> dict:
    return {k: v for k, v in res.items() if k == "CPU" or k.startswith("CPU_group_")}



def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    # a zombie child still answers kill(0): treat it as gone
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return False

class Conn:
    __slots__ = ("sock", "reader", "kind", "worker", "pid", "lock", "job_id", "alive", "wbuf", "held")

    def __init__(self, sock):
        self.sock = sock
        self.reader = P.FrameReader()
        self.kind = None
        self.worker = None
        self.pid = None
        self.lock = threading.Lock()
        self.job_id = None
        self.alive = True
        self.held = {}  # oid -> net references this process holds (its REF_DELTAS summed)

    def send(self, msg):
        if not self.alive:
            return
        try:
            P.send(self.sock, msg, self.lock)
        except OSError:
            self.alive = False


class WorkerRec:
    __slots__ = ("worker_id", "pid", "proc", "conn", "node", "env_key", "state", "task", "actor_id",
                 "fns", "gpu_key", "blocked", "start_time", "tasks_run", "lease", "idle_since", "calls",
                 "direct_addr", "assigned_time", "exit_detail")

    def __init__(self, worker_id, proc, node, env_key, gpu_key):
        self.worker_id = worker_id
        self.pid = proc.pid if proc else None
        self.proc = proc
        self.conn: Optional[Conn] = None
        self.node = node
        self.env_key = env_key
        self.gpu_key = gpu_key
        self.state = "STARTING"
        self.task = None
        self.actor_id = None
        self.fns = set()
        self.blocked = False
        self.start_time = time.time()
        self.tasks_run = 0
        self.lease = None
        self.idle_since = time.time()
        self.calls = collections.Counter()
        self.direct_addr = None  # the worker's direct-task socket (leased task submission)
        self.assigned_time = 0.0  # when its current task / lease / actor was assigned (memory-pressure victim order)
        self.exit_detail = None   # why the head killed it (e.g. the memory monitor's "System memory low ...")


class TaskRec:
    __slots__ = ("spec", "state", "worker", "node", "assign", "retries_left", "attempt", "submit_time",
                 "start_time", "end_time", "arg_refs", "owner_conn", "cancelled", "error", "pinned_bytes")

    def __init__(self, spec, owner_conn):
        self.spec = spec
        self.state = PENDING
        self.worker = None
        self.node = None
        self.assign = None
        self.retries_left = spec.get("max_retries", 3)
        self.attempt = 0
        self.submit_time = time.time()
        self.start_time = None
        self.end_time = None
        self.arg_refs = spec.get("arg_refs", [])
        self.owner_conn = owner_conn
        self.cancelled = False
        self.error = None
        self.pinned_bytes = None


class ActorRec:
    def __init__(self, spec, owner_conn):
        self.spec = spec
        self.actor_id = spec["actor_id"]
        self.state = ACTOR_PENDING
        self.worker: Optional[WorkerRec] = None
        self.address = None
        self.name = spec.get("name")
        self.namespace = spec.get("namespace")
        self.detached = spec.get("lifetime") == "detached"
        self.restarts_left = spec.get("max_restarts", 0)
        self.num_restarts = 0
        self.node = None
        self.assign = None
        self.waiters: List[tuple] = []
        self.owner_conn = owner_conn
        self.job_id = spec.get("job_id")
        self.death_cause = None
        self.pid = None
        self.task_key = None
        self.start_time = time.time()


class PGRec:
    def __init__(self, pg_id, bundles, strategy, name, lifetime, job_id):
        self.pg_id = pg_id
        self.bundles = bundles
        self.strategy = strategy
        self.name = name
        self.lifetime = lifetime
        self.job_id = job_id
        self.state = "PENDING"
        self.waiters: List[tuple] = []
        self.nodes = []


class Head:
    def __init__(self, args):
        self.args = args
        self.session_dir = args.session_dir
        self._event_loggers = {}
        self.sock_path = os.path.join(self.session_dir, "sockets", "head.sock")
        self.store_name = args.store_name
        self.config = json.loads(args.config) if args.config else {}
        self.spill_dirs = self._spill_dirs()
        for d in self.spill_dirs:
            os.makedirs(d, exist_ok=True)
        cap = int(args.object_store_memory)
        min_spill = int(self.config.get("min_spilling_size", min(100 << 20, max(1 << 20, cap // 16))))
        self.spill_threshold = float(self.config.get("object_spilling_threshold", 0.8))
        self.store = store_ext().ObjectStore.create_segment(
            self.store_name, cap,
            ":".join(self.spill_dirs),
            self.spill_threshold, min_spill, bool(self.config.get("object_store_fallback_allocation", True)),
            float(self.config.get("oom_grace_period_s", 2.0)),
            # reference ray_config_def.h:150 preallocate_plasma_memory (RAY_preallocate_plasma_memory=1)
            populate=bool(self.config.get("preallocate_plasma_memory",
                                          os.environ.get("RAY_preallocate_plasma_memory") == "1")))
        if not self.config.get("automatic_object_spilling_enabled", True):
            # reference: spilling off, but a full store still falls back to file-backed allocation
            # (plasma_allocator.cc fallback mmap) after the grace period
            self.store.set_spill_enabled(False)
        # memory-pressure machinery (reference: local_object_manager.cc IO-worker spilling,
        # local_task_manager.cc:615 PinTaskArgsIfMemoryAvailable, node_manager.cc:2799
        # TriggerGlobalGC, file_system_monitor.cc)
        import concurrent.futures

        self.max_io_workers = int(self.config.get("max_io_workers", 4))
        self.io_pool = concurrent.futures.ThreadPoolExecutor(self.max_io_workers, thread_name_prefix="rmm-io")
        self.spills_in_flight = 0
        self.spill_lock = threading.Lock()
        self.max_spill_bytes_per_job = int(self.config.get("max_spill_bytes_per_io_worker", 1 << 30))
        self.task_args_fraction = float(self.config.get("max_task_args_memory_fraction", 0.7))
        self.pinned_arg_bytes = 0
        self.pinned_arg_tasks = 0
        self.disk_threshold = float(self.config.get("local_fs_capacity_threshold", 0.95))
        self.disk_check_interval = float(self.config.get("local_fs_monitor_interval_ms", 1000)) / 1000.0
        self.last_disk_check = 0.0
        self.gc_seen = 0
        self.last_global_gc = 0.0
        self.gc_min_interval = float(self.config.get("global_gc_min_interval_s", 1.0))
        self.gc_high_usage = float(self.config.get("high_plasma_storage_usage", 0.7))
        self.gc_auto_interval = float(self.config.get("automatic_gc_min_interval_s", 30.0))
        self.mem_stats = collections.Counter()
        self._pins_pending = {}  # pid -> proc: exited clients whose store pins are released once gone
        self._death_reports = {}  # pid -> (proc, event fields, time): WORKER_DIED waiting for the exit code
        self.sched = sched_ext().Scheduler()
        self.sched.set_spread_threshold(float(self.config.get("scheduler_spread_threshold", 0.5)))
        self.nodes: Dict[int, dict] = {}
        self.head_node = 1
        res = json.loads(args.resources)
        self._add_node(self.head_node, res, head=True)
        self.sel = selectors.DefaultSelector()
        self.lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.lsock.bind(self.sock_path)
        self.lsock.listen(512)
        self.lsock.setblocking(False)
        self.sel.register(self.lsock, selectors.EVENT_READ, ("listen", None))
        self.wake_r, self.wake_w = os.pipe()
        os.set_blocking(self.wake_r, False)
        self.sel.register(self.wake_r, selectors.EVENT_READ, ("wake", None))
        self.pending_calls = collections.deque()
        self.pending_lock = threading.Lock()
        self.conns: Dict[int, Conn] = {}
        self.workers: Dict[bytes, WorkerRec] = {}
        self.idle: Dict[tuple, List[WorkerRec]] = collections.defaultdict(list)
        self.starting: Dict[tuple, int] = collections.Counter()
        self.tasks: Dict[bytes, TaskRec] = {}
        self.finished_tasks = collections.OrderedDict()
        self.direct_tasks = collections.deque(maxlen=10000)  # rows of directly submitted tasks
        self.lease_stats = collections.Counter()
        self.task_keys: Dict[int, bytes] = {}
        self.key_counter = 0
        self.dispatch_q: Dict[int, collections.deque] = collections.defaultdict(collections.deque)
        self.actors: Dict[bytes, ActorRec] = {}
        self.named_actors: Dict[tuple, bytes] = {}
        self.pgs: Dict[bytes, PGRec] = {}
        self.named_pgs: Dict[tuple, bytes] = {}
        self.kv: Dict[bytes, Dict[bytes, bytes]] = collections.defaultdict(dict)
        self.fn_table: Dict[bytes, bytes] = {}
        self.refcounts: Dict[bytes, int] = collections.defaultdict(int)
        self.contained: Dict[bytes, List[bytes]] = {}
        self.freed_early: set = set()
        self.recently_freed: "collections.OrderedDict[bytes, None]" = collections.OrderedDict()
        self.gpu_owner: Dict[bytes, bytes] = {}
        from ray_memory_management_amd._private.object_recovery import ObjectRecoveryManager

        self.recovery = ObjectRecoveryManager(self, int(self.config.get("max_lineage_entries", 200_000)))
        self.jobs: Dict[bytes, dict] = {}
        self.events = collections.deque(maxlen=int(self.config.get("timeline_max_events", 200000)))
        self.seal_cursor = 0
        self.running = True
        self.driver_conn = None
        self.next_node_id = 2
        self.max_workers = int(self.config.get("max_workers", max(64, 4 * int(res.get("CPU", 1)))))
        self.prestart = int(self.config.get("prestart_workers", min(2, int(res.get("CPU", 1)))))
        self.idle_timeout = float(self.config.get("idle_worker_killing_time_threshold_ms", 60000)) / 1000.0
        # scheduler warnings pushed to drivers (reference node_manager.cc:372 PublishInfeasibleTaskError,
        # :889 WarnResourceDeadlock with debug_dump_period_milliseconds = 10 s)
        self.deadlock_period = float(self.config.get("resource_deadlock_check_period_s", 10.0))
        self._infeasible_warned = set()
        self._deadlock_warned = 0
        self._deadlock_next = time.time() + self.deadlock_period
        self.pushed_errors = collections.deque(maxlen=1000)
        self.memory_monitor = None
        self.autoscaler = None
        if self.config.get("autoscaler"):
            from ray_memory_management_amd.autoscaler._private.monitor import Monitor

            self.autoscaler = Monitor(self, self.config["autoscaler"])
        self.last_housekeeping = 0.0
        # GCS persistence (reference gcs_server/gcs_table_storage + redis_store_client: with external
        # storage the GCS tables survive a head restart): internal KV, function/class table entries of
        # detached actors, detached actor specs, job history — snapshotted to `gcs_storage_path`
        self.gcs_path = self.config.get("gcs_storage_path")
        self.gcs_dirty = False
        self.gcs_last_flush = 0.0
        self.gcs_flush_s = float(self.config.get("gcs_storage_flush_interval_ms", 100)) / 1000.0
        self.gcs_restored = {"kv_namespaces": 0, "actors": 0, "jobs": 0}
        self.watcher = threading.Thread(target=self._seal_watcher, daemon=True)
        self.watcher.start()
        # memory-pressure worker killing (reference keys memory_usage_threshold_fraction /
        # memory_monitor_interval_ms, 0 disables; the round-5 keys are accepted as aliases)
        self.exit_details = collections.OrderedDict()  # worker id / direct addr / actor id -> exit detail
        self.dead_workers = collections.deque(maxlen=1000)  # state API rows of exited workers
        mm_ms = self.config.get("memory_monitor_interval_ms", self.config.get("memory_monitor_refresh_ms", 250))
        if float(mm_ms) > 0:
            from ray_memory_management_amd._private import memory_monitor as _mm

            thr = self.config.get("memory_usage_threshold_fraction", self.config.get("memory_usage_threshold", 0.95))
            src, sdir = self.config.get("memory_monitor_test_usage_file"), self.config.get("memory_monitor_test_usage_dir")
            usage = _mm.file_usage_source(src) if src else _mm.dir_usage_source(sdir) if sdir else None
            self.memory_monitor = _mm.MemoryMonitor(threshold=float(thr), interval_s=float(mm_ms) / 1000.0,
                                                    usage_fn=usage)

    def _spill_dirs(self):
        """Spill directories: `spill_dir` (str or list) or the reference's object_spilling_config
        JSON ({"type": "filesystem", "params": {"directory_path": str | [str, ...]}})."""
        c = self.config
        dirs = c.get("spill_dir")
        if not dirs and c.get("object_spilling_config"):
            sc = c["object_spilling_config"]
            sc = json.loads(sc) if isinstance(sc, str) else sc
            dirs = (sc.get("params") or {}).get("directory_path")
        if not dirs:
            dirs = [os.path.join(self.session_dir, "spill")]
        if isinstance(dirs, str):
            dirs = [dirs]
        return [os.path.abspath(d) for d in dirs]

    # ------------------------------------------------------------------ nodes
    def _add_node(self, node_id, resources, head=False):
        resources = {k: float(v) for k, v in resources.items() if v}
        resources.setdefault("node:__internal_head__" if head else f"node:{node_id}", 1.0)
        resources[f"node:{node_id}"] = 1.0
        self.sched.add_node(node_id, resources)
        self.nodes[node_id] = {"node_id": node_id, "resources": resources, "alive": True,
                               "start_time": time.time(), "is_head": head}
        if not head:
            self._broadcast_nodes()

    def _multi_node(self) -> bool:
        return sum(1 for n in self.nodes.values() if n["alive"]) > 1

    def _broadcast_nodes(self):
        """Owners submit tasks directly over leases only on a single-node cluster (no object can be
        lost with a node, so the head need not hold every task's lineage up front)."""
        for c in list(self.conns.values()):
            if c.kind is not None:
                self._send_nb(c, (P.NODES_CHANGED, self._multi_node()))

    def _remove_node(self, node_id):
        if node_id not in self.nodes or node_id == self.head_node:
            return False
        self.nodes[node_id]["alive"] = False
        self._event("CLUSTER_LIFECYCLE", "ERROR", "NODE_REMOVED", f"Node {self._hex(node_id)} was removed; "
                    "its running work is retried or reconstructed.", node_id=self._hex(node_id))
        # returns a running task already sealed on the node die with it (its TaskDone may still be
        # in flight); the task itself is retried when its worker's death is processed
        for t in list(self.tasks.values()):
            if t.node == node_id and t.state == RUNNING:
                rets = self.recovery.returns_of(t.spec)
                try:
                    sealed = bool(rets) and all(self.store.contains(o) for o in rets)
                except Exception:
                    sealed = False
                if sealed and t.spec.get("actor_id") is None and not t.spec.get("actor_creation"):
                    # the task sealed its returns but its TaskDone is still in flight: it finished on
                    # this node, so record it (lineage) and let node_removed below treat its
                    # returns as lost with the node
                    if t.worker is not None and t.worker.task == t.spec["task_id"]:
                        t.worker.task = None
                    self._release_task_resources(t)
                    self._finish(t, FINISHED)
                    continue
                for oid in rets:
                    try:
                        self.store.delete([oid])
                    except Exception:
                        pass
        for w in list(self.workers.values()):
            if w.node == node_id:
                self._kill_worker(w)
        self.sched.remove_node(node_id)
        # the node's primary object copies are gone with it: recover them through lineage
        self.recovery.node_removed(node_id)
        return True

    # ------------------------------------------------------------------ plumbing
    def _wake(self):
        try:
            os.write(self.wake_w, b"x")
        except OSError:
            pass

    def call_soon(self, fn, *a):
        with self.pending_lock:
            self.pending_calls.append((fn, a))
        self._wake()

    def _seal_watcher(self):
        seq = self.store.seal_seq()
        while self.running:
            nseq = self.store.wait_seal_seq(seq, 200)
            if nseq != seq:
                seq = nseq
                self._wake()

    # ------------------------------------------------------------------ GCS persistence
    def _gcs_snapshot(self) -> dict:
        det = []
        for a in self.actors.values():
            if a.detached and a.state != ACTOR_DEAD and not a.spec.get("arg_refs"):
                spec = {k: v for k, v in a.spec.items() if not k.startswith("_")}
                det.append((spec, self.fn_table.get(spec["class_id"])))
        jobs = [{k: v for k, v in j.items() if k != "conn"} for j in self.jobs.values()]
        return {"version": 1, "kv": {ns: dict(d) for ns, d in self.kv.items()}, "detached_actors": det,
                "jobs": jobs, "time": time.time()}

    def _gcs_flush(self, force=False):
        if not self.gcs_path or not (self.gcs_dirty or force):
            return
        os.makedirs(self.gcs_path, exist_ok=True)
        dst = os.path.join(self.gcs_path, "gcs_snapshot.pkl")
        tmp = dst + f".tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            pickle.dump(self._gcs_snapshot(), f, protocol=5)
        os.replace(tmp, dst)  # atomic: a crash mid-write keeps the previous snapshot
        self.gcs_dirty = False
        self.gcs_last_flush = time.time()

    def _gcs_restore(self):
        """Head restart with the same storage: reload KV and job history, recreate detached actors
        (fresh state, like a restart after their node died)."""
        path = os.path.join(self.gcs_path, "gcs_snapshot.pkl") if self.gcs_path else None
        if not path or not os.path.exists(path):
            return
        with open(path, "rb") as f:
            snap = pickle.load(f)  # written by this head process type only (trusted local file)
        for ns, d in snap.get("kv", {}).items():
            self.kv[ns].update(d)
        self.gcs_restored["kv_namespaces"] = len(snap.get("kv", {}))
        for j in snap.get("jobs", []):
            j = dict(j)
            j["alive"] = False
            j.setdefault("end_time", j.get("end_time") or snap.get("time"))
            self.jobs.setdefault(j["job_id"], j)
        self.gcs_restored["jobs"] = len(snap.get("jobs", []))
        for spec, blob in snap.get("detached_actors", []):
            if blob is not None:
                spec = dict(spec, class_blob=blob)
            self._create_actor(None, None, spec)
            self.gcs_restored["actors"] += 1

    def serve(self):
        self._gcs_restore()
        os.makedirs(os.path.dirname(self.sock_path), exist_ok=True)
        ready_file = os.path.join(self.session_dir, "head.ready")
        with open(ready_file, "w") as f:
            f.write(str(os.getpid()))
        for _ in range(self.prestart):
            self._start_worker(self.head_node, ("", ""), None)
        while self.running:
            try:
                events = self.sel.select(timeout=0.05)
            except InterruptedError:
                continue
            for key, _ in events:
                kind, conn = key.data
                if kind == "listen":
                    self._accept()
                elif kind == "wake":
                    try:
                        while os.read(self.wake_r, 4096):
                            pass
                    except (BlockingIOError, OSError):
                        pass
                else:
                    self._read(conn)
            self._drain_calls()
            self._poll_sealed()
            self._schedule()
            now = time.time()
            if now - self.last_housekeeping > 0.1:
                self.last_housekeeping = now
                self._housekeeping()
                if self.gcs_dirty and now - self.gcs_last_flush >= self.gcs_flush_s:
                    self._gcs_flush()
        self._gcs_flush(force=bool(self.gcs_path))
        self._shutdown()

    def _drain_calls(self):
        while True:
            with self.pending_lock:
                if not self.pending_calls:
                    return
                fn, a = self.pending_calls.popleft()
            try:
                fn(*a)
            except Exception:
                traceback.print_exc()

    def _accept(self):
        while True:
            try:
                s, _ = self.lsock.accept()
            except (BlockingIOError, OSError):
                return
            s.setblocking(True)
            c = Conn(s)
            self.conns[s.fileno()] = c
            s.setblocking(False)
            self.sel.register(s, selectors.EVENT_READ, ("conn", c))

    def _read(self, c: Conn):
        try:
            data = c.sock.recv(1 << 20)
        except BlockingIOError:
            return
        except OSError:
            data = b""
        if not data:
            self._disconnect(c)
            return
        try:
            msgs = c.reader.feed(data)
        except Exception:
            traceback.print_exc()
            self._disconnect(c)
            return
        for m in msgs:
            try:
                self._handle(c, m)
            except Exception:
                traceback.print_exc()

    def _send_nb(self, c: Conn, msg):
        """Send from the loop thread: sockets are non-blocking for reads; writes block briefly."""
        if not c.alive:
            return
        s = c.sock
        try:
            s.setblocking(True)
            P.send(s, msg, c.lock)
        except OSError:
            c.alive = False
        finally:
            try:
                s.setblocking(False)
            except OSError:
                pass

    def _reply(self, c, req_id, value):
        self._send_nb(c, (P.REPLY, req_id, value))

    # ------------------------------------------------------------------ dispatch table
    def _handle(self, c: Conn, m):
        t = m[0]
        if t == P.REF_DELTAS:
            held = c.held
            for oid, d in m[1]:
                n = held.get(oid, 0) + d
                if n:
                    held[oid] = n
                else:
                    held.pop(oid, None)
            # increments first: one batch covers a time window in which the process may have read a ref
            # out of an object (+1 inner) and then dropped that object (-1 outer); the batch is keyed by
            # object, so its order is not that order, and applying the -1 first could free the inner
            # object (a pending task's return) while the process now holds it
            d = m[1]
            if len(d) > 1:
                d = [x for x in d if x[1] > 0] + [x for x in d if x[1] <= 0]
            self._ref_deltas(d)
        elif t == P.SUBMIT_TASK:
            self._submit_task(c, m[1])
        elif t == P.DIRECT_DONE:
            self._direct_done(m[1])
        elif t == P.LEASE_REQUEST:
            self._lease_request(c, m[1], m[2])
        elif t == P.LEASE_RETURN:
            self._lease_return(m[1], m[2])
        elif t == P.EXIT_DETAIL:  # why a worker / actor died, if the head killed it (owner-side errors)
            self._reply(c, m[1], self.exit_details.get(m[2]))
        elif t == P.FN_EXPORT:
            self.fn_table[m[1]] = m[2]
        elif t == P.TASK_DONE:
            self._task_done(c, m[1], m[2], m[3], m[4] if len(m) > 4 else None)
        elif t == P.REGISTER:
            self._register(c, m[1], m[2])
        elif t == P.CREATE_ACTOR:
            self._create_actor(c, m[1], m[2])
        elif t == P.WAIT_ACTOR:
            self._wait_actor(c, m[1], m[2])
        elif t == P.ACTOR_READY:
            self._actor_ready(c, m[1], m[2])
        elif t == P.ACTOR_FAILED_INIT:
            self._actor_failed_init(c, m[1], m[2])
        elif t == P.CONTAINED:
            self._add_contained(m[1], m[2])
        elif t == P.BLOCKED:
            self._blocked(c, True)
        elif t == P.UNBLOCKED:
            self._blocked(c, False)
        elif t == P.KV_PUT:
            ns, k, v, overwrite = m[2], m[3], m[4], m[5]
            existed = k in self.kv[ns]
            if overwrite or not existed:
                self.kv[ns][k] = v
                self.gcs_dirty = True
            if m[1] is not None:
                self._reply(c, m[1], existed)
        elif t == P.KV_GET:
            self._reply(c, m[1], self.kv[m[2]].get(m[3]))
        elif t == P.KV_DEL:
            ns, k, prefix = m[2], m[3], m[4]
            if prefix:
                ks = [x for x in self.kv[ns] if x.startswith(k)]
            else:
                ks = [k] if k in self.kv[ns] else []
            for x in ks:
                del self.kv[ns][x]
            self.gcs_dirty = self.gcs_dirty or bool(ks)
            if m[1] is not None:
                self._reply(c, m[1], len(ks))
        elif t == P.KV_KEYS:
            self._reply(c, m[1], [x for x in self.kv[m[2]] if x.startswith(m[3])])
        elif t == P.GET_ACTOR:
            self._get_actor(c, m[1], m[2], m[3])
        elif t == P.KILL_ACTOR:
            self._kill_actor(m[1], m[2], "ray.kill() was called")
        elif t == P.CANCEL:
            self._cancel(m[1], m[2], m[3])
        elif t == P.PG_CREATE:
            self._pg_create(c, m[1], m[2])
        elif t == P.PG_REMOVE:
            self._pg_remove(m[1])
        elif t == P.PG_WAIT:
            self._pg_wait(c, m[1], m[2])
        elif t == P.PG_TABLE:
            self._reply(c, m[1], self._pg_table(m[2]))
        elif t == P.STATE:
            self._reply(c, m[1], self._state(m[2], m[3] if len(m) > 3 else None))
        elif t == P.EVENTS:
            self.events.extend(m[1])
        elif t == P.GPU_OBJECT:
            if m[1] in self.recently_freed:
                # the readers' ref deltas (another socket) won the race: the object was already
                # freed before its owner registered it — free the HBM copy right away
                self._send_nb(c, (P.FREE_GPU, [m[1]]))
                return
            self.gpu_owner[m[1]] = c.worker.worker_id if c.worker else b"driver:" + str(c.pid).encode()
            self.gpu_owner_conn = getattr(self, "gpu_owner_conn", {})
            self.gpu_owner_conn[m[1]] = c
        elif t == P.ADD_NODE:
            nid = self.next_node_id
            self.next_node_id += 1
            self._add_node(nid, m[2])
            self._reply(c, m[1], nid)
        elif t == P.REMOVE_NODE:
            self._reply(c, m[1], self._remove_node(m[2]))
        elif t == P.JOB_INFO:
            self._reply(c, m[1], {"session_dir": self.session_dir, "store_name": self.store_name,
                                  "config": self.config})
        elif t == P.ACTOR_EXITING:
            a = self.actors.get(m[1])
            if a is not None:
                a.restarts_left = 0
                a.death_cause = "The actor exited via exit_actor()."
        elif t == P.GLOBAL_GC:
            self._global_gc("requested")
        elif t == P.SHUTDOWN:
            self.running = False
        else:
            print(f"[head] unknown message {t}", file=sys.stderr)

    # ------------------------------------------------------------------ registration / workers
    def _register(self, c: Conn, kind, info):
        c.kind = kind
        c.pid = info.get("pid")
        if self._multi_node():
            self._send_nb(c, (P.NODES_CHANGED, True))
        if kind == "driver":
            job_id = info.get("job_id")
            c.job_id = job_id
            self.gcs_dirty = True
            self.jobs[job_id] = {"job_id": job_id, "pid": c.pid, "start_time": time.time(), "end_time": None,
                                 "namespace": info.get("namespace"), "alive": True, "conn": c}
            self._event("JOBS", "INFO", "JOB_STARTED", f"Driver pid {c.pid} connected.",
                        job_id=self._hex(job_id), pid=c.pid, namespace=info.get("namespace"))
            if self.driver_conn is None:
                self.driver_conn = c
            self._reply(c, info["req_id"], {
                "store_name": self.store_name, "session_dir": self.session_dir, "node_id": self.head_node,
                "config": self.config, "resources": self.sched.cluster_total()})
            return
        wid = info["worker_id"]
        w = self.workers.get(wid)
        if w is None:
            # a worker started by someone else (should not happen) — adopt
            return
        w.conn = c
        c.worker = w
        w.direct_addr = info.get("direct_addr")
        w.state = "IDLE"
        w.idle_since = time.time()
        self.starting[(w.node, w.env_key, w.gpu_key)] -= 1
        if w.actor_id is not None:
            a = self.actors.get(w.actor_id)
            if a is None or a.state == ACTOR_DEAD:
                self._kill_worker(w)
                return
            w.state = "ACTOR"
            w.assigned_time = time.time()
            self._send_nb(c, (P.CREATE_ACTOR_INSTANCE, a.spec, self.fn_table.get(a.spec["class_id"]),
                              {"gpu_ids": a.assign[1] if a.assign else [], "node_id": a.node,
                               "restart": a.num_restarts}))
            return
        self.idle[(w.node, w.env_key, w.gpu_key)].append(w)

    def _worker_env(self, node, env_key, gpu_ids, runtime_env):
        env = dict(os.environ)
        env["RMM_SESSION_DIR"] = self.session_dir
        env["RMM_STORE_NAME"] = self.store_name
        env["RMM_NODE_ID"] = str(node)
        env["RMM_HEAD_SOCKET"] = self.sock_path
        env["PYTHONUNBUFFERED"] = "1"
        env["RMM_CONFIG"] = json.dumps(self.config)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        if gpu_ids is not None:
            vis = ",".join(str(g) for g in gpu_ids)
            env["HIP_VISIBLE_DEVICES"] = vis
            env["CUDA_VISIBLE_DEVICES"] = vis
            env["RMM_GPU_IDS"] = vis
            # every GPU of the node, for collective groups that widen their visibility
            # (_private/gpu_visibility.py: RCCL peers should see each other's devices)
            n_gpu = int(float((self.nodes.get(node) or {}).get("resources", {}).get("GPU", 0)))
            env["RMM_NODE_GPU_IDS"] = ",".join(str(g) for g in range(n_gpu))
        if runtime_env:
            for k, v in (runtime_env.get("env_vars") or {}).items():
                env[str(k)] = str(v)
            if runtime_env.get("working_dir") or runtime_env.get("py_modules"):
                env["RMM_RUNTIME_ENV"] = json.dumps({k: runtime_env[k] for k in ("working_dir", "py_modules")
                                                     if runtime_env.get(k)})
        env.pop("RMM_DRIVER", None)
        return env

    _forker = None
    _fork_ok = None

    def _fork_client(self):
        """The worker fork server (_private/forkserver.py): workers are fork()s of a template that
        imported the runtime once (~ms each instead of a fresh interpreter). Off with
        worker_fork_server=False / RMM_NO_FORKSERVER=1; any failure falls back to Popen."""
        if self._fork_ok is None:
            self._fork_ok = bool(self.config.get("worker_fork_server", True)) and not os.environ.get("RMM_NO_FORKSERVER")
            if self._fork_ok:
                try:
                    from ray_memory_management_amd._private.forkserver import ForkClient

                    self._forker = ForkClient(self.session_dir, self._worker_env(1, "", None, None))
                except Exception as e:  # noqa: BLE001
                    print(f"[head] worker fork server unavailable ({e!r}); spawning interpreters", file=sys.stderr)
                    self._fork_ok = False
        return self._forker if self._fork_ok else None

    def _start_worker(self, node, key, gpu_ids, actor_id=None, runtime_env=None):
        env_key, gpu_key = key
        wid = os.urandom(16)
        env = self._worker_env(node, env_key, gpu_ids, runtime_env)
        env["RMM_WORKER_ID"] = wid.hex()
        log_dir = os.path.join(self.session_dir, "logs")
        log_path = os.path.join(log_dir, f"worker-{wid.hex()[:12]}.log")
        proc = None
        fk = self._fork_client()
        if fk is not None:
            try:
                proc = fk.spawn(env, log_path)
            except Exception as e:  # noqa: BLE001
                print(f"[head] fork server failed ({e!r}); spawning interpreters", file=sys.stderr)
                self._fork_ok = False
        if proc is None:
            out = open(log_path, "ab")
            cmd = [sys.executable, "-u", "-m", "ray_memory_management_amd._private.worker_main"]
            proc = subprocess.Popen(cmd, env=env, stdout=out, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                    start_new_session=True)
            out.close()
        w = WorkerRec(wid, proc, node, env_key, gpu_key)
        w.actor_id = actor_id
        self.workers[wid] = w
        self.starting[(node, env_key, gpu_key)] += 1
        return w

    def _event(self, source: str, severity: str, label: str, message: str, **fields):
        """Append a cluster event (reference RAY_EVENT) under <session>/logs/events/."""
        lg = self._event_loggers.get(source)
        if lg is None:
            from ray_memory_management_amd._private.event_log import EventLogger

            lg = self._event_loggers[source] = EventLogger(self.session_dir, source)
        try:
            lg.emit(severity, label, message, **fields)
        except Exception:  # noqa: BLE001 - events never fail the head
            pass

    @staticmethod
    def _hex(x):
        return x.hex() if isinstance(x, (bytes, bytearray)) else x

    def _kill_worker(self, w: WorkerRec, force=True):
        if w.proc is not None and w.proc.poll() is None:
            try:
                if force:
                    w.proc.kill()
                else:
                    w.proc.terminate()
            except OSError:
                pass
        w.state = "DEAD"

    def _disconnect(self, c: Conn):
        if not c.alive and c.sock.fileno() < 0:
            return
        c.alive = False
        try:
            self.sel.unregister(c.sock)
        except Exception:
            pass
        self.conns.pop(c.sock.fileno(), None)
        try:
            c.sock.close()
        except OSError:
            pass
        self._release_owner_leases(c)
        if c.kind == "driver":
            self._driver_exit(c)
        elif c.worker is not None:
            self._worker_died(c.worker)
        self._release_conn_refs(c)

    def _release_conn_refs(self, c: Conn) -> None:
        """A process disconnected (exited, or was killed before it could flush its ref deltas): drop
        the references it still held, so objects it was borrowing are freed once nobody else holds
        them. Each process contributes at most +1 per object (its first local ref) and -1 when its
        last one goes, so c.held is exactly what it still holds. Reference
        src/ray/core_worker/reference_count.cc: a borrower's refs are released when the owner's
        WaitForRefRemoved on it fails (the borrower died)."""
        held, c.held = c.held, {}
        drop = [(oid, -n) for oid, n in held.items() if n > 0]
        if drop:
            self.mem_stats["dead_client_refs_released"] = self.mem_stats.get("dead_client_refs_released", 0) + len(drop)
            self._ref_deltas(drop)

    def _emit_worker_died(self, fields: dict, code) -> None:
        sig = -code if isinstance(code, int) and code < 0 else None
        how = (f"killed by signal {sig}" + (" (SIGKILL: OOM killer or an external kill)" if sig == 9 else
                                            " (SIGSEGV)" if sig == 11 else "")) if sig else f"exit code {code}"
        self._event("RAYLET", "ERROR", "WORKER_DIED",
                    f"Worker pid {fields['pid']} died unexpectedly ({how}) in state {fields.pop('state')}.",
                    exit_code=code, signal=sig, **fields)

    def _release_client_pins(self, pid: int, proc=None) -> None:
        """A client process is gone: release every object-store pin it still held (objects it was
        reading when it was killed, its creator pins) so they can be freed / evicted / spilled again.
        Reference plasma/store.cc:323 DisconnectClient. Only once the process has really exited (a
        worker whose socket closed may still be unwinding its views); until then it is retried from
        the housekeeping tick."""
        alive = proc.poll() is None if proc is not None else _pid_alive(pid)
        if alive:
            self._pins_pending[pid] = proc
            return
        self._pins_pending.pop(pid, None)
        try:
            n = self.store.release_client(pid)
        except Exception:
            return
        if n:
            self.mem_stats["client_pins_released"] = self.mem_stats.get("client_pins_released", 0) + n

    def _driver_exit(self, c: Conn):
        job = self.jobs.get(c.job_id)
        if job:
            job["alive"] = False
            job["end_time"] = time.time()
            self.gcs_dirty = True
            self._event("JOBS", "INFO", "JOB_FINISHED", f"Driver pid {job.get('pid')} exited.",
                        job_id=self._hex(c.job_id), pid=job.get("pid"))
        # kill non-detached actors of this job, except those owned (directly or through other actors) by a
        # detached actor: in the reference an actor fate-shares with its owner, and a detached owner outlives
        # the job (e.g. Serve replicas and proxies created by its detached controller)
        for a in list(self.actors.values()):
            if a.job_id == c.job_id and not a.detached and a.state != ACTOR_DEAD and not self._owned_by_detached(a):
                a.restarts_left = 0
                self._kill_actor(a.actor_id, True, "The driver exited.")
        # release the driver's references
        if c is self.driver_conn and not self.args.persistent:
            self.running = False

    def _owned_by_detached(self, a) -> bool:
        for _ in range(64):  # owner chain: creating connection -> its worker's actor -> that actor's owner
            w = getattr(a.owner_conn, "worker", None)
            aid = getattr(w, "actor_id", None) if w is not None else None
            a = self.actors.get(aid) if aid is not None else None
            if a is None or a.state == ACTOR_DEAD:
                return False
            if a.detached:
                return True
        return False

    def _worker_died(self, w: WorkerRec):
        if w.state == "GONE":
            return
        prev_state = w.state
        w.state = "GONE"
        self.workers.pop(w.worker_id, None)
        self.dead_workers.append({"worker_id": w.worker_id.hex(), "pid": w.pid, "state": "DEAD", "node_id": w.node,
                                  "actor_id": w.actor_id.hex() if w.actor_id else None, "tasks_run": w.tasks_run,
                                  "exit_detail": w.exit_detail})
        for lst in self.idle.values():
            if w in lst:
                lst.remove(w)
        if prev_state == "STARTING":
            self.starting[(w.node, w.env_key, w.gpu_key)] -= 1
        if w.pid:
            try:
                self.store.abort_creator(w.pid)
            except Exception:
                pass
        if w.proc is not None:
            try:
                w.proc.wait(timeout=0.05)
            except Exception:
                pass
        if w.pid:
            self._release_client_pins(w.pid, w.proc)
        if prev_state != "DEAD":  # not a kill the head asked for (those report their own reason)
            t0 = self.tasks.get(w.task) if w.task is not None else None
            fields = dict(pid=w.pid, worker_id=self._hex(w.worker_id),
                          task_id=self._hex(t0.spec["task_id"]) if t0 is not None else None,
                          job_id=self._hex(t0.spec.get("job_id")) if t0 is not None else None,
                          actor_id=self._hex(w.actor_id), state=prev_state)
            code = w.proc.poll() if w.proc is not None else None
            if code is None and w.proc is not None:
                # the exit status is not known yet (a fork-server worker's arrives as the template's
                # reap report): the event waits for it, at most 2 s (housekeeping)
                self._death_reports[w.pid] = (w.proc, fields, time.time())
            else:
                self._emit_worker_died(fields, code)
        if w.task is not None:
            t = self.tasks.get(w.task)
            w.task = None
            if t is not None and t.spec.get("_lease") is not None:
                self.tasks.pop(t.spec["task_id"], None)
                self._release_task_resources(t)
                t = None
            if t is not None:
                self._release_task_resources(t)
                if t.cancelled:
                    self._fail_task(t, exc.TaskCancelledError(t.spec["task_id"].hex()), CANCELLED)
                elif t.retries_left != 0:
                    if t.retries_left > 0:
                        t.retries_left -= 1
                    t.attempt += 1
                    t.state = PENDING
                    self._enqueue(t)
                else:
                    err = exc.OutOfMemoryError(w.exit_detail) if t.error == "oom" and w.exit_detail \
                        else exc.WorkerCrashedError()
                    self._fail_task(t, err, FAILED)
        if w.actor_id is not None:
            a = self.actors.get(w.actor_id)
            if a is not None and a.worker is w:
                self._actor_died(a)
        # GPU objects live in the dead process's HBM arena: they are lost
        lost = [o for o, owner in self.gpu_owner.items() if owner == w.worker_id]
        if lost:
            conns = getattr(self, "gpu_owner_conn", {})
            for o in lost:
                self.gpu_owner.pop(o, None)
                conns.pop(o, None)
            self.recovery.objects_lost(lost, f"the worker process {w.pid} owning them died", owner_died=True)

    def _blocked(self, c: Conn, blocked: bool):
        w = c.worker
        if w is None or w.task is None or w.blocked == blocked:
            return
        t = self.tasks.get(w.task)
        if t is None or t.assign is None:
            return
        w.blocked = blocked
        cpu_only = _cpu_part(t.spec["_res"])
        if not cpu_only:
            return
        if blocked:
            self.sched.release(t.node, cpu_only)
        else:
            self.sched.acquire(t.node, cpu_only, True)

    # ------------------------------------------------------------------ refcounting
    def _ref_deltas(self, deltas):
        rc = self.refcounts
        for oid, d in deltas:
            n = rc[oid] + d
            if n <= 0:
                del rc[oid]
                self._free(oid)
            else:
                rc[oid] = n

    def _add_contained(self, outer, inners):
        if not inners:
            return
        if outer not in self.refcounts and outer in self.recently_freed:
            # the outer object was already freed: its owner read it and dropped it before this CONTAINED
            # (sent by the producing worker on another connection) arrived. Holding the inner refs for a gone
            # object would leak them; whoever deserialized the outer holds the inner refs on their own (their
            # +1 reached the head before their drop of the outer, hence before this message)
            return
        self.contained.setdefault(outer, []).extend(inners)
        rc = self.refcounts
        for i in inners:
            rc[i] += 1

    def _free(self, oid: bytes):
        if oid[:1] == b"\xaa" and oid[-3:] == b"\xaa\xaa\xaa":
            self._actor_out_of_scope(oid[1:17])
            return
        self.recovery.object_freed(oid)
        rf = self.recently_freed
        rf[oid] = None
        if len(rf) > 100_000:
            rf.popitem(last=False)
        deleted = self.store.delete([oid])
        if not deleted:
            self.freed_early.add(oid)
        owner = self.gpu_owner.pop(oid, None)
        if owner is not None:
            c = getattr(self, "gpu_owner_conn", {}).pop(oid, None)
            if c is not None:
                self._send_nb(c, (P.FREE_GPU, [oid]))
        inner = self.contained.pop(oid, None)
        if inner:
            self._ref_deltas([(i, -1) for i in inner])

    def _poll_sealed(self):
        cur, oids, overflow = self.store.poll_sealed(self.seal_cursor)
        self.seal_cursor = cur
        if not oids:
            return
        self.sched.objects_ready(oids)
        if self.freed_early:
            dead = [o for o in oids if o in self.freed_early]
            if dead:
                for o in dead:
                    self.freed_early.discard(o)
                    if o not in self.refcounts:
                        self.store.delete([o])

    # ------------------------------------------------------------------ tasks
    def _new_key(self, task_id):
        self.key_counter += 1
        self.task_keys[self.key_counter] = task_id
        return self.key_counter

    def _submit_task(self, c: Conn, spec):
        fn_blob = spec.pop("fn_blob", None)
        if fn_blob is not None:
            self.fn_table[spec["fn_id"]] = fn_blob
        t = TaskRec(spec, c)
        self.tasks[spec["task_id"]] = t
        for r in t.arg_refs:
            self.refcounts[r] += 1
        self._enqueue(t)

    # ------------------------------------------------------------------ worker leases
    def _lease_request(self, c: Conn, req_id, ls):
        """Reference node_manager.cc HandleRequestWorkerLease: the lease is scheduled like a task
        (resources, worker pool keyed by runtime env / GPUs) and, once placed, the owner gets the
        worker's direct address instead of the worker getting an EXECUTE."""
        spec = {"task_id": ls["lease_id"], "name": "lease", "resources": ls["resources"], "strategy": None,
                "env_key": ls.get("env_key", ""), "runtime_env": ls.get("runtime_env"), "fn_id": None,
                "arg_refs": [], "max_retries": 0, "num_returns": 0, "_lease": req_id}
        t = TaskRec(spec, c)
        self.tasks[spec["task_id"]] = t
        self.lease_stats["requested"] += 1
        self._enqueue(t)

    def _lease_return(self, lease_id, kill: bool):
        t = self.tasks.pop(lease_id, None)
        if t is None or t.spec.get("_lease") is None:
            return
        self.lease_stats["returned"] += 1
        if t.state == PENDING:
            key = t.spec.get("_key")
            if key is not None and self.sched.cancel(key):
                self.task_keys.pop(key, None)
            for q in self.dispatch_q.values():
                if t in q:
                    q.remove(t)
                    self._release_task_resources(t)
            return
        self._release_task_resources(t)
        w = t.worker
        if w is not None and w.task == lease_id:
            w.task = None
            w.tasks_run += 1
            if kill:
                self._kill_worker(w)
            else:
                self._make_idle(w)

    def _release_owner_leases(self, c: Conn):
        for lid in [tid for tid, t in self.tasks.items() if t.owner_conn is c and t.spec.get("_lease") is not None]:
            self._lease_return(lid, False)

    def _direct_done(self, items):
        """Completion records of directly submitted tasks: lineage for reconstruction + the state
        API / timeline row (reference: owner-side task events reported to GCS)."""
        for lineage, rec in items:
            if lineage is not None:
                self.recovery.task_finished(lineage, rec[3])
        self.direct_tasks.extend(rec for _, rec in items)

    def _resubmit(self, spec):
        """Re-run a finished task to recompute its lost returns (lineage reconstruction)."""
        t = TaskRec(spec, None)
        t.attempt = 1
        self.tasks[spec["task_id"]] = t
        for r in t.arg_refs:
            self.refcounts[r] += 1
        self._enqueue(t)
        self._wake()

    def _strategy_args(self, spec):
        st = spec.get("strategy") or {}
        kind = st.get("type", "DEFAULT")
        if kind == "SPREAD":
            return 1, -1, False, "", -1
        if kind == "NODE_AFFINITY":
            return 2, int(st["node_id"]), bool(st.get("soft", False)), "", -1
        if kind == "PLACEMENT_GROUP":
            return 3, -1, False, st["pg_id"].hex(), int(st.get("bundle_index", -1))
        return 0, -1, False, "", -1

    def _enqueue(self, t: TaskRec):
        spec = t.spec
        deps = [r for r in t.arg_refs if not _is_actor_key(r) and not self.store.contains(r)]
        key = self._new_key(spec["task_id"])
        t.spec["_key"] = key
        strat, aff, soft, pg, bidx = self._strategy_args(spec)
        if strat == 3:
            pgrec = self.pgs.get(bytes.fromhex(pg))
            if pgrec is None or pgrec.state == "REMOVED":
                self._fail_task(t, exc.TaskPlacementGroupRemoved("placement group was removed"), FAILED)
                return
            spec["_res"] = pg_rewrite(spec["resources"], pg, bidx)
            strat, pg, bidx = 0, "", -1
        else:
            spec["_res"] = spec["resources"]
        self.sched.submit(key, spec["_res"], strat, aff, soft, pg, bidx, deps)

    def _schedule(self):
        placed = self.sched.schedule_placement_groups()
        for pg_hex in placed:
            self._pg_placed(bytes.fromhex(pg_hex))
        assigns = self.sched.schedule(1 << 20)
        for key, node, gpu_ids, amounts in assigns:
            tid = self.task_keys.pop(key, None)
            if tid is None:
                continue
            if isinstance(tid, tuple):  # actor creation
                self._actor_placed(tid[1], node, gpu_ids, amounts)
                continue
            t = self.tasks.get(tid)
            if t is None or t.cancelled:
                self.sched.release(node, t.spec.get("_res", {}) if t else {}, gpu_ids, amounts)
                if t is not None:
                    self._fail_task(t, exc.TaskCancelledError(tid.hex()), CANCELLED)
                continue
            t.node = node
            t.assign = (node, gpu_ids, amounts)
            self.dispatch_q[node].append(t)
        for node, q in self.dispatch_q.items():
            while q:
                t = q[0]
                if not self._dispatch(t):
                    break
                q.popleft()

    def _gpu_key(self, gpu_ids):
        return ",".join(map(str, gpu_ids)) if gpu_ids else ""

    def _pin_task_args(self, t: TaskRec) -> bool:
        """Reference local_task_manager.cc:615 PinTaskArgsIfMemoryAvailable: a task's by-ref
        arguments stay pinned in the store while it runs; a new task is held back when pinning its
        args would push the pinned total over max_task_args_memory_fraction of the store (unless
        nothing is pinned, so one oversized task can still make progress)."""
        if getattr(t, "pinned_bytes", None) is not None:
            return True
        refs = [r for r in t.arg_refs if not _is_actor_key(r)]
        n = 0
        if refs:
            n = sum(max(0, x) for x in self.store.sizes(refs))
        cap = self.store.capacity()
        if n and self.pinned_arg_tasks > 0 and self.pinned_arg_bytes + n > self.task_args_fraction * cap:
            self.mem_stats["task_args_backpressure"] += 1
            return False
        t.pinned_bytes = n
        if n:
            self.pinned_arg_bytes += n
            self.pinned_arg_tasks += 1
        return True

    def _unpin_task_args(self, t: TaskRec):
        n = getattr(t, "pinned_bytes", None)
        if n:
            self.pinned_arg_bytes -= n
            self.pinned_arg_tasks -= 1
        t.pinned_bytes = None

    def _dispatch(self, t: TaskRec) -> bool:
        spec = t.spec
        node, gpu_ids, amounts = t.assign
        env_key = spec.get("env_key", "")
        gkey = self._gpu_key(gpu_ids)
        key = (node, env_key, gkey)
        pool = self.idle.get(key)
        w = None
        while pool:
            cand = pool.pop()
            if cand.state == "IDLE" and cand.conn is not None and cand.conn.alive:
                w = cand
                break
        if w is None:
            # GPU tasks may reuse a never-GPU worker only by spawning with the right devices
            n_start = self.starting[key]
            waiting = sum(1 for x in self.dispatch_q[node] if x.spec.get("env_key", "") == env_key)
            if n_start < max(1, waiting) and len(self.workers) < self.max_workers + 32:
                self._start_worker(node, (env_key, gkey), gpu_ids if gpu_ids else None,
                                   runtime_env=spec.get("runtime_env"))
            return False
        if spec.get("_lease") is not None:  # a worker lease: hand the worker to the owner
            w.state = "BUSY"
            w.task = spec["task_id"]
            t.worker = w
            t.state = RUNNING
            t.start_time = w.assigned_time = time.time()
            self.lease_stats["granted"] += 1
            multi = self._multi_node()
            self._reply(t.owner_conn, spec["_lease"], ("granted", spec["task_id"], w.direct_addr, w.worker_id,
                                                      gpu_ids, node, multi))
            return True
        if not self._pin_task_args(t):
            pool = self.idle.setdefault(key, [])
            pool.append(w)
            return False
        fid = spec["fn_id"]
        blob = None
        if fid not in w.fns:
            blob = self.fn_table.get(fid)
            w.fns.add(fid)
        w.state = "BUSY"
        w.task = spec["task_id"]
        t.worker = w
        t.state = RUNNING
        t.start_time = w.assigned_time = time.time()
        self._send_nb(w.conn, (P.EXECUTE, spec, blob, {"gpu_ids": gpu_ids, "attempt": t.attempt,
                                                       "node_id": node}))
        return True

    def _release_task_resources(self, t: TaskRec):
        self._unpin_task_args(t)
        if t.assign is not None:
            node, gpu_ids, amounts = t.assign
            req = dict(t.spec.get("_res", t.spec["resources"]))
            if t.worker is not None and t.worker.blocked:
                for k in _cpu_part(req):
                    req.pop(k)
                t.worker.blocked = False
            self.sched.release(node, req, gpu_ids, amounts)
            t.assign = None

    def _finish(self, t: TaskRec, state):
        t.state = state
        t.end_time = time.time()
        self.tasks.pop(t.spec["task_id"], None)
        if state == FINISHED:
            self.recovery.task_finished(t.spec, t.node)
        if t.arg_refs:
            self._ref_deltas([(r, -1) for r in t.arg_refs])
            t.arg_refs = []
        self.finished_tasks[t.spec["task_id"]] = t
        while len(self.finished_tasks) > 10000:
            self.finished_tasks.popitem(last=False)

    def _task_done(self, c: Conn, task_id, status, contained, info):
        w = c.worker
        t = self.tasks.get(task_id)
        if w is not None and w.task == task_id:
            w.task = None
            w.blocked = w.blocked  # released below
            w.tasks_run += 1
        if t is None:
            if w is not None:
                self._make_idle(w)
            return
        self._release_task_resources(t)
        if contained:
            for outer, inners in contained.items():
                self._add_contained(outer, inners)
        if info and info.get("events"):
            self.events.extend(info["events"])
        if status == "retry" and t.retries_left != 0 and not t.cancelled:
            if t.retries_left > 0:
                t.retries_left -= 1
            t.attempt += 1
            t.state = PENDING
            if w is not None:
                self._make_idle(w)
            self._enqueue(t)
            return
        self._finish(t, FINISHED if status == "ok" else FAILED)
        if status == "ok" and t.node is not None and not self.nodes.get(t.node, {}).get("alive", True):
            # finished on a node removed meanwhile: its outputs went down with the node
            self.recovery.objects_lost(self.recovery.returns_of(t.spec), f"node {t.node} was removed")
        if w is not None:
            if info and info.get("exit"):
                self._kill_worker(w, force=False)
            else:
                self._make_idle(w)

    def _make_idle(self, w: WorkerRec):
        if w.state in ("DEAD", "GONE"):
            return
        w.state = "IDLE"
        w.idle_since = time.time()
        self.idle[(w.node, w.env_key, w.gpu_key)].append(w)

    def _fail_task(self, t: TaskRec, error: BaseException, state=FAILED):
        spec = t.spec
        self._store_error(spec["task_id"], spec.get("num_returns", 1), error)
        self._finish(t, state)

    def _store_error(self, task_id, num_returns, error):
        n = num_returns if isinstance(num_returns, int) else 1
        data, bufs, _ = ser.serialize(error)
        for i in range(1, max(n, 1) + 1):
            oid = object_id_for_return(task_id, i)
            try:
                if self.store.state(oid) == 1:  # CREATING by a dead process
                    self.store.abort(oid)
                self.store.put_serialized(oid, data, bufs, ser.TAG_ERROR, True)
            except Exception:
                traceback.print_exc()

    def _cancel(self, task_id, force, recursive):
        t = self.tasks.get(task_id)
        if t is None:
            return
        t.cancelled = True
        if t.state == PENDING:
            key = t.spec.get("_key")
            if key is not None and self.sched.cancel(key):
                self.task_keys.pop(key, None)
            for node, q in self.dispatch_q.items():
                if t in q:
                    q.remove(t)
                    self._release_task_resources(t)
            self._fail_task(t, exc.TaskCancelledError(task_id.hex()), CANCELLED)
        elif t.state == RUNNING and t.worker is not None:
            if force:
                self._kill_worker(t.worker)
            elif t.worker.conn is not None:
                self._send_nb(t.worker.conn, (P.CANCEL_TASK, task_id))

    # ------------------------------------------------------------------ actors
    def _create_actor(self, c: Conn, req_id, spec):
        fn_blob = spec.pop("class_blob", None)
        if fn_blob is not None:
            self.fn_table[spec["class_id"]] = fn_blob
        name = spec.get("name")
        if name:
            key = (spec.get("namespace"), name)
            existing = self.named_actors.get(key)
            if existing is not None and self.actors[existing].state != ACTOR_DEAD:
                if req_id is not None:
                    self._reply(c, req_id, ("exists", existing))
                return
            self.named_actors[key] = spec["actor_id"]
        a = ActorRec(spec, c)
        self.actors[a.actor_id] = a
        if a.detached:
            self.gcs_dirty = True
        for r in spec.get("arg_refs", []):
            self.refcounts[r] += 1
        if req_id is not None:
            self._reply(c, req_id, ("ok", a.actor_id))
        self._schedule_actor(a)

    def _schedule_actor(self, a: ActorRec):
        spec = a.spec
        key = self._new_key(("actor", a.actor_id))
        self.task_keys[key] = ("actor", a.actor_id)
        a.task_key = key
        strat, aff, soft, pg, bidx = self._strategy_args(spec)
        deps = [r for r in spec.get("arg_refs", []) if not _is_actor_key(r) and not self.store.contains(r)]
        if strat == 3:
            spec["_pres"] = pg_rewrite(spec["placement_resources"], pg, bidx)
            spec["_lres"] = pg_rewrite(spec["resources"], pg, bidx)
            strat, pg, bidx = 0, "", -1
        else:
            spec["_pres"], spec["_lres"] = spec["placement_resources"], spec["resources"]
        self.sched.submit(key, spec["_pres"], strat, aff, soft, pg, bidx, deps)

    def _actor_placed(self, actor_id, node, gpu_ids, amounts):
        a = self.actors.get(actor_id)
        if a is None or a.state == ACTOR_DEAD:
            self.sched.release(node, a.spec.get("_pres", {}) if a else {}, gpu_ids, amounts)
            return
        # Keep only the lifetime resources; return the scheduling-only part.
        pres, lres = a.spec["_pres"], a.spec["_lres"]
        extra = {k: v - lres.get(k, 0.0) for k, v in pres.items() if v - lres.get(k, 0.0) > 0}
        if extra:
            self.sched.release(node, extra, [], [])
        if not any(k == "GPU" or k.startswith("GPU_group_") for k in lres):
            gpu_ids, amounts = [], []
        a.node = node
        a.assign = (node, gpu_ids, amounts)
        w = self._start_worker(node, (a.spec.get("env_key", ""), "actor"), gpu_ids if gpu_ids else None,
                               actor_id=actor_id, runtime_env=a.spec.get("runtime_env"))
        a.worker = w
        a.pid = w.pid

    def _actor_ready(self, c: Conn, actor_id, address):
        a = self.actors.get(actor_id)
        if a is None:
            return
        a.state = ACTOR_ALIVE
        a.address = address
        for wc, rid in a.waiters:
            self._reply(wc, rid, ("alive", address, a.num_restarts))
        a.waiters.clear()

    def _actor_failed_init(self, c: Conn, actor_id, err_blob):
        a = self.actors.get(actor_id)
        if a is None:
            return
        a.restarts_left = 0
        a.death_cause = err_blob
        self._kill_actor(actor_id, True, err_blob)

    def _wait_actor(self, c: Conn, req_id, actor_id):
        a = self.actors.get(actor_id)
        if a is None:
            self._reply(c, req_id, ("dead", "actor not found", 0))
        elif a.state == ACTOR_ALIVE:
            self._reply(c, req_id, ("alive", a.address, a.num_restarts))
        elif a.state == ACTOR_DEAD:
            self._reply(c, req_id, ("dead", a.death_cause, a.num_restarts))
        else:
            a.waiters.append((c, req_id))

    def _get_actor(self, c: Conn, req_id, name, namespace):
        aid = self.named_actors.get((namespace, name))
        if aid is None or self.actors[aid].state == ACTOR_DEAD:
            self._reply(c, req_id, None)
        else:
            self._reply(c, req_id, self.actors[aid].spec)

    def _actor_died(self, a: ActorRec):
        if a.assign is not None:
            node, gpu_ids, amounts = a.assign
            self.sched.release(node, a.spec.get("_lres", a.spec["resources"]), gpu_ids, amounts)
            a.assign = None
        a.worker = None
        a.address = None
        if a.state != ACTOR_DEAD and a.restarts_left != 0:
            if a.restarts_left > 0:
                a.restarts_left -= 1
            a.num_restarts += 1
            a.state = ACTOR_RESTARTING
            self._event("GCS", "WARNING", "ACTOR_RESTARTED", f"Actor {a.actor_id.hex()} is restarting "
                        f"(restart {a.num_restarts}).", actor_id=a.actor_id.hex(), job_id=self._hex(a.job_id),
                        num_restarts=a.num_restarts, class_name=a.spec.get("class_name"))
            self._schedule_actor(a)
            return
        if a.state != ACTOR_DEAD:
            self._event("GCS", "ERROR", "ACTOR_DIED", f"Actor {a.actor_id.hex()} died: "
                        f"{a.death_cause or 'the actor process died unexpectedly'}.", actor_id=a.actor_id.hex(),
                        job_id=self._hex(a.job_id), class_name=a.spec.get("class_name"))
        self._mark_actor_dead(a, a.death_cause or "The actor process died unexpectedly.")

    def _mark_actor_dead(self, a: ActorRec, cause):
        a.state = ACTOR_DEAD
        self.gcs_dirty = self.gcs_dirty or a.detached
        a.death_cause = cause
        for wc, rid in a.waiters:
            self._reply(wc, rid, ("dead", cause, a.num_restarts))
        a.waiters.clear()
        if a.name and self.named_actors.get((a.namespace, a.name)) == a.actor_id:
            del self.named_actors[(a.namespace, a.name)]
        refs = a.spec.get("arg_refs", [])
        if refs:
            a.spec["arg_refs"] = []
            self._ref_deltas([(r, -1) for r in refs])

    def _kill_actor(self, actor_id, no_restart, cause):
        a = self.actors.get(actor_id)
        if a is None or a.state == ACTOR_DEAD:
            return
        if no_restart:
            a.restarts_left = 0
        if isinstance(cause, str):
            a.death_cause = a.death_cause or cause
        if a.task_key is not None and a.state in (ACTOR_PENDING, ACTOR_RESTARTING) and a.worker is None:
            if self.sched.cancel(a.task_key):
                self.task_keys.pop(a.task_key, None)
        w = a.worker
        if w is not None:
            self._kill_worker(w)
            if no_restart:
                # resources are released when the process exit is observed
                pass
        else:
            if a.restarts_left == 0:
                self._mark_actor_dead(a, a.death_cause)

    def _actor_out_of_scope(self, actor_id):
        a = self.actors.get(actor_id)
        if a is None or a.detached or a.name or a.state == ACTOR_DEAD:
            return
        a.restarts_left = 0
        self._kill_actor(actor_id, True, "All references to the actor were removed.")

    # ------------------------------------------------------------------ placement groups
    def _pg_create(self, c, req_id, info):
        pg_id = info["pg_id"]
        name = info.get("name")
        if name:
            key = (info.get("namespace"), name)
            if key in self.named_pgs:
                self._reply(c, req_id, ("exists", None))
                return
            self.named_pgs[key] = pg_id
        pg = PGRec(pg_id, info["bundles"], info["strategy"], name, info.get("lifetime"), info.get("job_id"))
        self.pgs[pg_id] = pg
        strat = {"PACK": 0, "SPREAD": 1, "STRICT_PACK": 2, "STRICT_SPREAD": 3}[info["strategy"]]
        self.sched.create_placement_group(pg_id.hex(), info["bundles"], strat)
        self._reply(c, req_id, ("ok", None))

    def _pg_placed(self, pg_id):
        pg = self.pgs.get(pg_id)
        if pg is None:
            return
        pg.state = "CREATED"
        pg.nodes = self.sched.placement_group_nodes(pg_id.hex())
        for wc, rid in pg.waiters:
            self._reply(wc, rid, True)
        pg.waiters.clear()

    def _pg_wait(self, c, req_id, pg_id):
        pg = self.pgs.get(pg_id)
        if pg is None or pg.state == "REMOVED":
            self._reply(c, req_id, False)
        elif pg.state == "CREATED":
            self._reply(c, req_id, True)
        else:
            pg.waiters.append((c, req_id))

    def _pg_remove(self, pg_id):
        pg = self.pgs.get(pg_id)
        if pg is None:
            return
        # kill actors / fail tasks using the group
        for a in list(self.actors.values()):
            st = a.spec.get("strategy") or {}
            if st.get("type") == "PLACEMENT_GROUP" and st.get("pg_id") == pg_id and a.state != ACTOR_DEAD:
                a.restarts_left = 0
                self._kill_actor(a.actor_id, True, "The placement group was removed.")
        for t in list(self.tasks.values()):
            st = t.spec.get("strategy") or {}
            if st.get("type") == "PLACEMENT_GROUP" and st.get("pg_id") == pg_id:
                if t.state == PENDING:
                    t.cancelled = True
                    key = t.spec.get("_key")
                    if key is not None and self.sched.cancel(key):
                        self.task_keys.pop(key, None)
                    self._fail_task(t, exc.TaskPlacementGroupRemoved("placement group was removed"), FAILED)
                elif t.worker is not None:
                    self._kill_worker(t.worker)
        self.sched.remove_placement_group(pg_id.hex())
        pg.state = "REMOVED"
        for wc, rid in pg.waiters:
            self._reply(wc, rid, False)
        pg.waiters.clear()
        if pg.name:
            self.named_pgs = {k: v for k, v in self.named_pgs.items() if v != pg_id}

    def _pg_table(self, pg_id):
        def info(pg):
            return {"placement_group_id": pg.pg_id.hex(), "name": pg.name or "", "bundles": dict(enumerate(pg.bundles)),
                    "strategy": pg.strategy, "state": pg.state, "bundles_to_node_id": pg.nodes}
        if pg_id is None:
            return {pg.pg_id.hex(): info(pg) for pg in self.pgs.values()}
        if isinstance(pg_id, tuple):  # lookup by name
            pid = self.named_pgs.get(pg_id)
            return info(self.pgs[pid]) if pid else None
        pg = self.pgs.get(pg_id)
        return info(pg) if pg else None

    # ------------------------------------------------------------------ state API
    def _state(self, what, arg):
        if what == "cluster_resources":
            return self.sched.cluster_total()
        if what == "available_resources":
            # object_store_memory is reported as the store's free bytes (reference: the raylet reports
            # plasma usage against the resource, python/ray/tests/test_memory_scheduling.py:46)
            return self._store_adjusted(self.sched.cluster_available())
        if what == "nodes":
            out = []
            for nid, n in self.nodes.items():
                out.append({"NodeID": nid, "Alive": n["alive"], "Resources": self.sched.total(nid) if n["alive"] else {},
                            "Available": (self._store_adjusted(self.sched.available(nid)) if n["is_head"]
                                          else self.sched.available(nid)) if n["alive"] else {},
                            "IsHead": n["is_head"],
                            "NodeManagerAddress": "127.0.0.1", "ObjectStoreSocketName": self.store_name,
                            "alive": n["alive"]})
            return out
        if what == "actors":
            return [{"actor_id": a.actor_id.hex(), "class_name": a.spec.get("class_name"), "state": a.state,
                     "name": a.name or "", "namespace": a.namespace, "pid": a.pid, "node_id": a.node,
                     "num_restarts": a.num_restarts, "death_cause": a.death_cause if isinstance(a.death_cause, str) else None,
                     "job_id": a.job_id.hex() if a.job_id else None, "lifetime": "detached" if a.detached else "non_detached"}
                    for a in self.actors.values()]
        if what == "tasks":
            out = []
            for coll in (self.tasks, self.finished_tasks):
                for tid, t in coll.items():
                    if t.spec.get("_lease") is not None:
                        continue
                    out.append({"task_id": tid.hex(), "name": t.spec.get("name"), "state": t.state,
                                "func_or_class_name": t.spec.get("name"), "node_id": t.node, "attempt": t.attempt,
                                "start_time": t.start_time, "end_time": t.end_time, "required_resources": t.spec["resources"],
                                "worker_pid": t.worker.pid if t.worker else None})
            for tid, name, ok, node, attempt, t0, t1, res in self.direct_tasks:
                out.append({"task_id": tid.hex(), "name": name, "state": FINISHED if ok else FAILED,
                            "func_or_class_name": name, "node_id": node, "attempt": attempt, "start_time": t0,
                            "end_time": t1, "required_resources": res, "worker_pid": None})
            return out
        if what == "gcs":
            return {"storage_path": self.gcs_path, "restored": dict(self.gcs_restored), "dirty": self.gcs_dirty,
                    "last_flush": self.gcs_last_flush}
        if what == "leases":
            return {**dict(self.lease_stats), "held": sum(1 for t in self.tasks.values()
                                                          if t.spec.get("_lease") is not None and t.state == RUNNING)}
        if what == "workers":
            return [{"worker_id": w.worker_id.hex(), "pid": w.pid, "state": w.state, "node_id": w.node,
                     "actor_id": w.actor_id.hex() if w.actor_id else None, "tasks_run": w.tasks_run,
                     "exit_detail": w.exit_detail}
                    for w in self.workers.values()] + list(self.dead_workers)
        if what == "objects":
            objs = self.store.list_objects()
            for o in objs:
                o["object_id"] = o["object_id"].hex()
                o["reference_count"] = self.refcounts.get(bytes.fromhex(o["object_id"]), 0)
            return objs
        if what == "ref_holders":  # who holds an object: per-connection counts + containing objects
            oid = bytes.fromhex(arg) if isinstance(arg, str) else arg
            out = [{"kind": c.kind, "pid": c.pid, "count": c.held[oid]} for c in self.conns.values()
                   if oid in c.held]
            out += [{"kind": "contained_in", "object_id": o.hex()} for o, inn in self.contained.items() if oid in inn]
            return {"reference_count": self.refcounts.get(oid, 0), "holders": out,
                    "recently_freed": oid in self.recently_freed, "freed_early": oid in self.freed_early}
        if what == "store_stats":
            return self.store.stats()
        if what == "jobs":
            return [{k: v for k, v in j.items() if k != "conn"} for j in self.jobs.values()]
        if what == "placement_groups":
            return self._pg_table(None)
        if what == "refcounts":
            return dict(self.refcounts)
        if what == "recovery":
            return self.recovery.stats()
        if what == "timeline":
            return list(self.events)
        if what == "summary":
            real = [t for t in self.tasks.values() if t.spec.get("_lease") is None]
            return {"pending_tasks": sum(1 for t in real if t.state == PENDING),
                    "running_tasks": sum(1 for t in real if t.state == RUNNING),
                    "workers": len(self.workers), "actors": len(self.actors),
                    "infeasible": len(self.sched.infeasible_tasks())}
        if what == "memory":
            return self.memory_monitor.snapshot() if self.memory_monitor else {}
        if what == "session_dir":
            return self.session_dir
        if what == "runtime_envs":
            envs = {}
            for rec in list(self.actors.values()) + list(self.tasks.values()) + list(self.finished_tasks.values()):
                re_ = (rec.spec or {}).get("runtime_env") if hasattr(rec, "spec") else None
                if re_:
                    key = json.dumps(re_, sort_keys=True, default=str)
                    envs.setdefault(key, {"runtime_env": re_, "ref_cnt": 0})["ref_cnt"] += 1
            return list(envs.values())
        if what == "memory_pressure":
            return {**dict(self.mem_stats), "pinned_arg_bytes": self.pinned_arg_bytes,
                    "pinned_arg_tasks": self.pinned_arg_tasks, "spills_in_flight": self.spills_in_flight,
                    "spill_dirs": self.spill_dirs, **self.store.oom_stats()}
        raise ValueError(f"unknown state query {what}")

    def _store_adjusted(self, avail: dict) -> dict:
        if "object_store_memory" in avail:
            try:
                used = self.store.stats()["bytes_in_use"]
            except Exception:  # noqa: BLE001
                used = 0
            avail = dict(avail)
            avail["object_store_memory"] = max(0.0, float(avail["object_store_memory"]) - float(used))
        return avail

    # ------------------------------------------------------------------ housekeeping
    def _housekeeping(self):
        now = time.time()
        if self.recovery.awaiting:
            self.recovery.expire_awaiting(now)
        # WORKER_DIED events waiting for the exit status
        for pid, (proc, fields, t0) in list(self._death_reports.items()):
            code = proc.poll()
            if code is not None or now - t0 > 2.0:
                self._death_reports.pop(pid, None)
                self._emit_worker_died(fields, code)
        # pins of exited clients whose release had to wait for the process to finish exiting
        for pid, proc in list(self._pins_pending.items()):
            self._release_client_pins(pid, proc)
        # reap dead worker processes that never connected / crashed
        for w in list(self.workers.values()):
            if w.proc is not None and w.proc.poll() is not None:
                if w.conn is None or not w.conn.alive or w.state == "DEAD":
                    self._worker_died(w)
        # threshold-driven spilling by a capped pool of IO workers (local_object_manager.cc:149,172)
        st = self.store.stats()
        cap = st["capacity"]
        if cap and st["bytes_in_use"] > self.spill_threshold * cap:
            excess = st["bytes_in_use"] - int(self.spill_threshold * cap)
            with self.spill_lock:
                free_slots = self.max_io_workers - self.spills_in_flight
            for _ in range(max(0, free_slots)):
                if excess <= 0:
                    break
                job = min(excess, self.max_spill_bytes_per_job)
                excess -= job
                with self.spill_lock:
                    self.spills_in_flight += 1
                self.io_pool.submit(self._io_spill, job)
        self._disk_monitor(now)
        self._maybe_global_gc(now, st)
        try:
            self._scheduler_warnings(now)
        except Exception as e:  # a diagnostic must never take the head down
            self.mem_stats["scheduler_warning_errors"] += 1
            print(f"[head] scheduler warning check failed: {e!r}", file=sys.stderr, flush=True)
        # idle worker reaping (keep prestart pool)
        idle_total = sum(len(v) for v in self.idle.values())
        if idle_total > self.prestart:
            for key, lst in self.idle.items():
                for w in list(lst):
                    if idle_total <= self.prestart:
                        break
                    if now - w.idle_since > self.idle_timeout and w.state == "IDLE":
                        lst.remove(w)
                        self._send_nb(w.conn, (P.EXIT,))
                        w.state = "DEAD"
                        idle_total -= 1
        if self.autoscaler is not None:
            self.autoscaler.tick()
        if self.memory_monitor is not None:
            self._memory_pressure(now)

    # ------------------------------------------------------------------ memory-pressure worker killing
    def _memory_pressure(self, now: float):
        """Reference node_manager.cc:2902-3001: above `memory_usage_threshold_fraction`, kill the worker whose
        task / lease / actor was assigned most recently -- retriable or not, task or actor -- and pick no new
        victim until that one is dead. Its task is retried by its owner while retries are left (head path:
        here; leased workers: the owner's direct submitter), else fails with OutOfMemoryError (a
        WorkerCrashedError) carrying the exit detail; an actor without restarts dies with it as the death
        cause (RayActorError)."""
        from ray_memory_management_amd._private import memory_monitor as _mm

        mm = self.memory_monitor
        if mm.target is not None:
            tw = mm.target
            gone = tw.state == "GONE" or (tw.proc.poll() is not None if tw.proc is not None else not _mm.pid_alive(tw.pid))
            if gone:
                mm.target = None
        above = mm.refresh(now)
        if not above:
            return
        if mm.target is not None:  # one eviction in flight: wait for it to return memory
            if now - mm.last_wait_log > 1.0:
                mm.last_wait_log = now
                self.mem_stats["memory_manager_eviction_waits"] += 1
            return
        cands = []
        for w in self.workers.values():
            if w.state in ("DEAD", "GONE", "STARTING") or w.conn is None:
                continue
            if w.task is None and w.actor_id is None:
                continue
            cands.append((w.assigned_time, w))
        victim = mm.pick_victim(cands)
        if victim is None:
            return
        t = self.tasks.get(victim.task) if victim.task is not None else None
        is_actor = victim.actor_id is not None
        a = self.actors.get(victim.actor_id) if is_actor else None
        if is_actor:
            name = (a.spec.get("class_name") if a is not None else None) or "actor"
            kind, ident = "actor", victim.actor_id.hex()
        elif t is not None and t.spec.get("_lease") is not None:
            name, kind, ident = "leased worker (direct tasks)", "task", self._hex(t.spec["task_id"])
        else:
            name = (t.spec.get("name") if t is not None else None) or "task"
            kind, ident = "task", self._hex(t.spec["task_id"]) if t is not None else "?"
        detail = _mm.format_eviction_message("127.0.0.1", mm.last_used, mm.last_total, mm.threshold, name, kind, ident)
        victim.exit_detail = detail
        ed = self.exit_details
        for key in (victim.worker_id, victim.direct_addr, victim.actor_id):
            if key is not None:
                ed[key] = detail
        while len(ed) > 10000:
            ed.popitem(last=False)
        if t is not None:
            t.error = "oom"
        if a is not None and a.restarts_left == 0:
            a.death_cause = detail
        mm.record_kill(is_actor, victim, now)
        self.mem_stats["memory_manager_actor_eviction_total" if is_actor else "memory_manager_task_eviction_total"] += 1
        self._event("RAYLET", "ERROR", "OUT_OF_MEMORY", detail, pid=victim.pid, worker_id=self._hex(victim.worker_id),
                    task_id=self._hex(t.spec["task_id"]) if t is not None else None,
                    actor_id=self._hex(victim.actor_id),
                    job_id=self._hex(t.spec.get("job_id")) if t is not None else None)
        print(f"[head] {detail}", file=sys.stderr, flush=True)
        self._kill_worker(victim)

    # ------------------------------------------------------------------ scheduler warnings
    def _push_error(self, job_id, etype: str, msg: str, **fields):
        """Send a warning to the job's driver (printed there as "(raylet) ..." and kept in
        worker.pushed_errors), record it in the head's error table and as a cluster event."""
        self.pushed_errors.append({"type": etype, "message": msg, "job_id": self._hex(job_id), "time": time.time()})
        self._event("RAYLET", "WARNING", etype.upper(), msg, job_id=self._hex(job_id), **fields)
        targets = []
        job = self.jobs.get(job_id) if job_id is not None else None
        if job is not None and job.get("alive") and job.get("conn") is not None:
            targets.append(job["conn"])
        elif job_id is None or job is None:  # unknown job: every connected driver
            targets = [c for c in self.conns.values() if c.kind == "driver" and c.alive]
        for c in targets:
            self._send_nb(c, (P.PUSH_ERROR, etype, msg, job_id))

    def _scheduler_warnings(self, now: float):
        """Infeasible tasks / actors (no node can ever hold their resources) warn their driver once;
        a resource deadlock (ready tasks pending for two consecutive check periods while no worker runs an
        unblocked non-actor task: the resources are held by actors or by tasks blocked on each other)
        warns once per episode and triggers a global GC (actor handles caught in reference cycles may
        be holding the resources)."""
        inf = self.sched.infeasible_tasks()
        if inf or self._infeasible_warned:
            cur = set(inf)
            for key in cur - self._infeasible_warned:
                tid = self.task_keys.get(key)
                if tid is None:
                    continue
                if isinstance(tid, tuple):  # actor creation
                    a = self.actors.get(tid[1])
                    if a is None:
                        continue
                    res, job, what = (a.spec.get("_pres") or {}), a.job_id, tid[1]
                else:
                    t = self.tasks.get(tid)
                    if t is None:
                        continue
                    res, job, what = t.spec.get("_res", {}), t.spec.get("job_id"), tid
                    if job is None and t.owner_conn is not None:  # a worker lease: its owner's job
                        job = getattr(t.owner_conn, "job_id", None)
                if any("_group_" in k for k in res):  # placement-group bundles warn through the PG
                    continue
                req = ", ".join(f"{k}: {v:g}" for k, v in sorted(res.items()) if v)
                self._push_error(job, "infeasible_task",
                                 f"The actor or task with ID {self._hex(what)} cannot be scheduled right now. It "
                                 f"requires {{{req}}} for placement, however the cluster currently cannot provide "
                                 f"the requested resources (cluster total: {self._fmt_res(self.sched.cluster_total())}). "
                                 "The required resources may be added as autoscaling takes place or placement groups "
                                 "are scheduled. Otherwise, consider reducing the resource requirements of the task.",
                                 task_id=self._hex(what))
            self._infeasible_warned = cur
        if now < self._deadlock_next:
            return
        self._deadlock_next = now + self.deadlock_period
        ready = self.sched.num_pending() - len(self.sched.waiting_tasks()) - len(inf)
        # progress = some worker runs a (non-actor) task and is not blocked in get (reference
        # worker.h IsAvailableForScheduling); a long task backlog therefore never warns
        running = any(w.task is not None and not w.blocked and w.actor_id is None for w in self.workers.values())
        if ready <= 0 or running:
            self._deadlock_warned = 0
            return
        self._deadlock_warned += 1
        if self._deadlock_warned < 2:
            return
        self._global_gc("resource deadlock")
        if self._deadlock_warned > 2:
            return
        ex = next((t for t in self.tasks.values() if t.state == PENDING and t.assign is None), None)
        job = ex.spec.get("job_id") if ex is not None else None
        res = ex.spec.get("_res", {}) if ex is not None else {}
        req = ", ".join(f"{k}: {v:g}" for k, v in sorted(res.items()) if v)
        self._push_error(job, "resource_deadlock",
                         f"The actor or task with ID {self._hex(ex.spec['task_id']) if ex is not None else '?'} cannot "
                         "be scheduled right now. You can ignore this message if this cluster is expected to "
                         "auto-scale. Otherwise, this is likely due to all cluster resources being claimed by actors "
                         "or by tasks waiting on each other. To resolve the issue, consider creating fewer actors or "
                         f"increasing the resources available to this cluster.\nRequired resources for this actor or "
                         f"task: {{{req}}}\nAvailable resources: {self._fmt_res(self.sched.cluster_available())} In "
                         f"total there are {ready} pending tasks / actors.", pending=ready)

    @staticmethod
    def _fmt_res(d) -> str:
        try:
            return "{" + ", ".join(f"{k}: {v:g}" for k, v in sorted(dict(d).items()) if v and "_group_" not in k) + "}"
        except Exception:
            return str(d)

    def _io_spill(self, nbytes):
        try:
            freed = self.store.spill(nbytes)
            self.mem_stats["io_spill_jobs"] += 1
            self.mem_stats["io_spilled_bytes"] += freed
        except Exception:
            traceback.print_exc()
        finally:
            with self.spill_lock:
                self.spills_in_flight -= 1

    def _disk_monitor(self, now):
        """Reference src/ray/common/file_system_monitor.cc: spilling (and fallback files) stop when
        a spill directory's filesystem is over local_fs_capacity_threshold; a put that then cannot
        be satisfied raises OutOfDiskError."""
        if now - self.last_disk_check < self.disk_check_interval:
            return
        self.last_disk_check = now
        full = False
        for d in self.spill_dirs:
            try:
                v = os.statvfs(d)
            except OSError:
                continue
            total = v.f_blocks * v.f_frsize
            if total and 1.0 - (v.f_bavail * v.f_frsize) / total > self.disk_threshold:
                full = True
        if full != self.store.disk_full():
            self.store.set_disk_full(full)
            self.mem_stats["disk_full_transitions"] += 1
            if full:
                self._event("RAYLET", "WARNING", "DISK_FULL", "A spill directory's filesystem is over "
                            f"local_fs_capacity_threshold {self.disk_threshold}: spilling stops.",
                            dirs=list(self.spill_dirs))
            else:
                self._event("RAYLET", "INFO", "DISK_OK", "Spill directories have space again.")

    def _maybe_global_gc(self, now, st):
        """A create starved past its first retry bumps the store's gc_requests; the head then
        broadcasts a GC to every worker and driver (node_manager.cc:2799 TriggerGlobalGC). Also
        triggered periodically while the store is above high_plasma_storage_usage."""
        req = self.store.gc_requests()
        cap = st.get("capacity") or 0
        if req != self.gc_seen and now - self.last_global_gc >= self.gc_min_interval:
            self.gc_seen = req
            self._global_gc("store pressure")
        elif cap and st["bytes_in_use"] > self.gc_high_usage * cap and now - self.last_global_gc >= self.gc_auto_interval:
            self._global_gc("high usage")

    def _global_gc(self, reason):
        self.last_global_gc = time.time()
        self.mem_stats["global_gc"] += 1
        for c in list(self.conns.values()):
            if c.alive and (c.kind == "driver" or c.worker is not None):
                self._send_nb(c, (P.TRIGGER_GC, reason))

    def _shutdown(self):
        try:
            self.io_pool.shutdown(wait=False)
        except Exception:
            pass
        for w in list(self.workers.values()):
            if w.conn is not None and w.conn.alive:
                try:
                    self._send_nb(w.conn, (P.EXIT,))
                except Exception:
                    pass
        deadline = time.time() + 1.0
        for w in list(self.workers.values()):
            if w.proc is not None:
                try:
                    w.proc.wait(timeout=max(0.0, deadline - time.time()))
                except Exception:
                    pass
                if w.proc.poll() is None:
                    try:
                        w.proc.kill()
                    except OSError:
                        pass
        try:
            os.unlink(self.sock_path)
        except OSError:
            pass
        try:
            if self._forker is not None:
                self._forker.close()
        except OSError:
            pass
        # spill / fallback files die with the store (reference: the raylet deletes an owner's spilled
        # objects when it exits, test_object_spilling_2.py:366 test_file_deleted_when_driver_exits)
        for d in self.spill_dirs:
            try:
                for f in os.listdir(d):
                    if (f.startswith("rmm-spill-") or f.startswith("rmm-fallback-")) and f.endswith(".bin"):
                        try:
                            os.unlink(os.path.join(d, f))
                        except OSError:
                            pass
            except OSError:
                pass
        try:  # explicitly: other references to the store (IO threads) would keep `del` from unlinking
            from _posixshmem import shm_unlink

            shm_unlink(self.args.store_name)
        except (ImportError, OSError):
            pass
        del self.store


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--session-dir", required=True)
    ap.add_argument("--store-name", required=True)
    ap.add_argument("--object-store-memory", required=True)
    ap.add_argument("--resources", required=True)
    ap.add_argument("--config", default="")
    ap.add_argument("--persistent", action="store_true")
    args = ap.parse_args()
    os.makedirs(os.path.join(args.session_dir, "logs"), exist_ok=True)
    os.makedirs(os.path.join(args.session_dir, "sockets"), exist_ok=True)
    signal.signal(signal.SIGTERM, lambda *a: sys.exit(0))  # until the loop runs
    h = Head(args)

    def _term(*_):
        # `rmm stop`: leave the loop and shut down the normal way (workers told to exit, the GCS
        # flushed, the store segment unlinked) instead of unwinding out of it
        h.running = False
        try:
            os.write(h.wake_w, b"x")
        except OSError:
            pass

    signal.signal(signal.SIGTERM, _term)
    import faulthandler

    # `rmm stack` / debugging a stuck control plane: SIGUSR1 dumps every head thread's stack to its log
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    prof_path = os.environ.get("RMM_HEAD_PROFILE")  # control-plane profiling: cProfile of the loop
    prof = None
    if prof_path:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    try:
        h.serve()
    finally:
        h.running = False
        if prof is not None:
            prof.disable()
            prof.dump_stats(prof_path)


if __name__ == "__main__":
    main()
