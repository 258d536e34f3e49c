"""Serve controller: the single source of truth for deployments and their replicas.

Parity: reference python/ray/serve/controller.py + _private/deployment_state.py (reconcile
target vs running replicas, rolling updates on version change, health checks, graceful
shutdown) + _private/autoscaling_policy.py (BasicAutoscalingPolicy: desired replicas from the
smoothed number of ongoing requests per replica, with upscale / downscale delays).

A background thread reconciles every deployment every 50 ms; readers (handles, HTTP proxy)
poll `get_replicas(name, known_version)` which only ships the replica list when it changed.
"""
from __future__ import annotations

import math
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.serve.config import AutoscalingConfig, DeploymentConfig
from ray_memory_management_amd.serve.handle import _REFRESH_S, SERVE_NAMESPACE


class _DeploymentState:
    def __init__(self, name, spec):
        self.name = name
        self.spec = spec
        self.replicas: List[tuple] = []      # (tag, actor) ready
        self.starting: List[tuple] = []      # (tag, actor, ready_ref, t0)
        self.stopping: List[tuple] = []      # (tag, actor, ref, t0)
        self.version = 0                     # bumps whenever `replicas` changes
        self.target = spec["config"].num_replicas
        self.metrics: List[tuple] = []       # (ts, inflight) from handles
        self.last_scale = time.time()
        self.pending_direction = 0
        self.pending_since = 0.0
        self.last_health = time.time()
        self.code_version = spec.get("version")
        self.deleting = False
        if spec["config"].autoscaling_config is not None:
            a = spec["config"].autoscaling_config
            self.target = max(a.min_replicas, 1) if a.min_replicas else a.min_replicas


class ServeController:
    def __init__(self, http_options: Optional[dict] = None, detached: bool = False):
        self._deployments: Dict[str, _DeploymentState] = {}
        self._lock = threading.RLock()
        self._stop = False
        self._http_options = http_options or {}
        self._proxy = None
        self._replica_cls = None
        self._loop_t = threading.Thread(target=self._loop, daemon=True, name="serve-reconcile")
        self._loop_t.start()

    # ------------------------------------------------------------------ API
    def deploy(self, name: str, spec: Dict[str, Any]) -> bool:
        with self._lock:
            cur = self._deployments.get(name)
            if cur is None or cur.deleting:
                self._deployments[name] = _DeploymentState(name, spec)
                return True
            # no explicit version => every redeploy replaces the replicas (reference semantics)
            code_changed = spec.get("version") is None or spec.get("version") != cur.code_version
            old_cfg = cur.spec["config"]
            cur.spec = spec
            cur.code_version = spec.get("version")
            if spec["config"].autoscaling_config is None:
                cur.target = spec["config"].num_replicas
            if code_changed:
                # rolling update: new replicas come up, old ones drain once they are replaced
                for tag, actor in cur.replicas:
                    cur.stopping.append((tag, actor, actor.prepare_for_shutdown.remote(
                        old_cfg.graceful_shutdown_timeout_s), time.time()))
                cur.replicas = []
                cur.version += 1
            elif spec["config"].user_config != old_cfg.user_config:
                ray.get([a.reconfigure.remote(spec["config"].user_config) for _, a in cur.replicas])
            return True

    def delete_deployment(self, name: str) -> bool:
        with self._lock:
            st = self._deployments.get(name)
            if st is None:
                return False
            st.deleting = True
            st.target = 0
        return True

    def get_replicas(self, name: str, known_version: int = -1):
        with self._lock:
            st = self._deployments.get(name)
            if st is None:
                return -1, []
            if st.version == known_version:
                return st.version, None
            return st.version, [a for _, a in st.replicas]

    def record_handle_metrics(self, name: str, inflight: int, ts: float):
        with self._lock:
            st = self._deployments.get(name)
            if st is not None:
                st.metrics.append((time.time(), inflight))
                st.metrics = st.metrics[-200:]

    def wait_ready(self, name: str, timeout_s: float = 60.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            with self._lock:
                st = self._deployments.get(name)
                if st is None:
                    return False
                if len(st.replicas) >= st.target and not st.stopping and not st.starting:
                    return True
            time.sleep(0.02)
        raise TimeoutError(f"deployment {name!r} did not become ready in {timeout_s}s")

    def wait_deleted(self, name: str, timeout_s: float = 60.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            with self._lock:
                if name not in self._deployments:
                    return True
            time.sleep(0.02)
        return False

    def list_deployments(self) -> Dict[str, dict]:
        with self._lock:
            return {n: {"name": n, "num_replicas": len(s.replicas), "target_num_replicas": s.target,
                        "route_prefix": s.spec.get("route_prefix"), "version": s.code_version,
                        "user_config": s.spec["config"].user_config,
                        "max_concurrent_queries": s.spec["config"].max_concurrent_queries,
                        "ray_actor_options": s.spec.get("ray_actor_options"),
                        "status": "UPDATING" if s.starting or s.stopping or len(s.replicas) != s.target
                        else "HEALTHY"}
                    for n, s in self._deployments.items() if not s.deleting}

    def get_deployment_spec(self, name: str):
        with self._lock:
            st = self._deployments.get(name)
            return None if st is None or st.deleting else st.spec

    def get_route_table(self) -> Dict[str, str]:
        with self._lock:
            return {s.spec["route_prefix"]: n for n, s in self._deployments.items()
                    if s.spec.get("route_prefix") and not s.deleting}

    def get_http_config(self):
        return self._http_options

    def set_proxy(self, proxy):
        self._proxy = proxy
        return True

    def shutdown(self):
        with self._lock:
            for st in self._deployments.values():
                st.deleting = True
                st.target = 0
        t0 = time.time()
        while time.time() - t0 < 10:
            with self._lock:
                if not self._deployments:
                    break
            time.sleep(0.02)
        self._stop = True
        return True

    def ping(self):
        return True

    # ------------------------------------------------------------------ reconcile
    def _loop(self):
        while not self._stop:
            try:
                with self._lock:
                    for name in list(self._deployments):
                        self._reconcile(self._deployments[name])
            except Exception:  # keep the controller alive whatever a replica does
                import traceback

                traceback.print_exc()
            time.sleep(0.05)

    def _new_replica(self, st: _DeploymentState):
        from ray_memory_management_amd.serve.replica import ServeReplica

        if self._replica_cls is None:
            self._replica_cls = ray.remote(ServeReplica)
        spec = st.spec
        tag = f"{st.name}#{uuid.uuid4().hex[:6]}"
        opts = dict(spec.get("ray_actor_options") or {})
        opts.setdefault("num_cpus", 1)
        actor = self._replica_cls.options(name=f"SERVE_REPLICA::{tag}", namespace=SERVE_NAMESPACE,
                                          max_concurrency=spec["config"].max_concurrent_queries, **opts).remote(
            st.name, tag, spec["func_or_class"], spec.get("init_args", ()), spec.get("init_kwargs", {}),
            spec["config"].user_config, spec.get("ingress_app"))
        st.starting.append((tag, actor, actor.ready.remote(), time.time()))

    def _autoscale(self, st: _DeploymentState):
        a: AutoscalingConfig = st.spec["config"].autoscaling_config
        if a is None or st.deleting:
            return
        now = time.time()
        window = [m for t, m in st.metrics if now - t <= a.look_back_period_s]
        # handles only report while they send traffic: no report in the window means idle
        ongoing = sum(window) / len(window) if window else 0.0
        cur = max(len(st.replicas), 1)
        desired = math.ceil(ongoing / a.target_num_ongoing_requests_per_replica) if ongoing > 0 else a.min_replicas
        desired = int(min(max(desired, a.min_replicas), a.max_replicas))
        if desired == st.target:
            st.pending_direction = 0
            return
        direction = 1 if desired > st.target else -1
        if direction != st.pending_direction:
            st.pending_direction, st.pending_since = direction, now
            return
        delay = a.upscale_delay_s if direction > 0 else a.downscale_delay_s
        if now - st.pending_since >= delay:
            st.target = desired
            st.pending_direction = 0

    def _reconcile(self, st: _DeploymentState):
        cfg: DeploymentConfig = st.spec["config"]
        self._autoscale(st)
        # 1) starting replicas that became ready
        still = []
        for tag, actor, ref, t0 in st.starting:
            ready, _ = ray.wait([ref], timeout=0)
            if ready:
                try:
                    ray.get(ref)
                    st.replicas.append((tag, actor))
                    st.version += 1
                except Exception:
                    ray.kill(actor)  # constructor failed: retry
            else:
                still.append((tag, actor, ref, t0))
        st.starting = still
        # 2) scale
        n = len(st.replicas) + len(st.starting)
        for _ in range(max(st.target - n, 0)):
            self._new_replica(st)
        if len(st.replicas) > st.target:
            extra = len(st.replicas) - st.target
            victims, st.replicas = st.replicas[-extra:], st.replicas[:-extra]
            st.version += 1
            for tag, actor in victims:
                st.stopping.append((tag, actor, actor.prepare_for_shutdown.remote(cfg.graceful_shutdown_timeout_s),
                                    time.time()))
        # 3) drained replicas
        keep = []
        for tag, actor, ref, t0 in st.stopping:
            # keep a removed replica alive until every handle has re-read the replica set
            # (handles refresh every _REFRESH_S) so no request is routed to a dead actor
            if time.time() - t0 < 2.5 * _REFRESH_S:
                keep.append((tag, actor, ref, t0))
                continue
            ready, _ = ray.wait([ref], timeout=0)
            if ready or time.time() - t0 > cfg.graceful_shutdown_timeout_s + 5:
                try:
                    ray.kill(actor)
                except Exception:
                    pass
            else:
                keep.append((tag, actor, ref, t0))
        st.stopping = keep
        # 4) health checks
        if st.replicas and time.time() - st.last_health >= cfg.health_check_period_s:
            st.last_health = time.time()
            refs = [(tag, actor, actor.check_health.remote()) for tag, actor in st.replicas]
            bad = []
            for tag, actor, ref in refs:
                try:
                    ray.get(ref, timeout=cfg.health_check_timeout_s)
                except Exception:
                    bad.append((tag, actor))
            if bad:
                st.replicas = [r for r in st.replicas if r not in bad]
                st.version += 1
                for _, actor in bad:
                    try:
                        ray.kill(actor)
                    except Exception:
                        pass
        if st.deleting and not st.replicas and not st.starting and not st.stopping:
            del self._deployments[st.name]
