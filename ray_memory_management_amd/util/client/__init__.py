"""Ray Client: drive a cluster from a process outside it with the normal API.

Parity: reference python/ray/util/client/{__init__.py, worker.py (Worker: put / get / wait /
remote function + actor calls forwarded to the server, ClientObjectRef lifetimes),
api.py} and ``ray.init("ray://host:port")``. Connect with
``ray.init("ray://127.0.0.1:10001")`` against a server started by
``rmm start --head --ray-client-server-port 10001`` (or
``python -m ray_memory_management_amd.util.client.server``).
"""
from __future__ import annotations

import itertools
import socket
import threading
from typing import Any, List, Optional

import cloudpickle

from ray_memory_management_amd.util.client import common as C
from ray_memory_management_amd.util.client.common import ClientActorHandle, ClientObjectRef  # noqa: F401


class ClientWorker:
    def __init__(self, host: str, port: int, namespace: Optional[str] = None, timeout: float = 30.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.settimeout(None)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.lock = threading.Lock()
        self.send_lock = threading.Lock()
        self.ids = itertools.count(1)
        self.pending_release: List[bytes] = []
        self.namespace = namespace
        self.closed = False
        C._tls.client = self
        self.info = self.request("init", {"namespace": namespace})

    # ------------------------------------------------------------------ transport
    def request(self, op: str, payload: Any = None):
        with self.lock:
            if self.closed:
                raise ConnectionError("Ray Client is disconnected")
            rel, self.pending_release = self.pending_release, []
            if rel:
                self._roundtrip("release", rel)
            return self._roundtrip(op, payload)

    def _roundtrip(self, op, payload):
        rid = next(self.ids)
        C.send(self.sock, (rid, op, payload), self.send_lock)
        C._tls.client = self
        got_rid, (status, value) = cloudpickle.loads(C.recv(self.sock))
        self._attach(value)
        if status == "err":
            raise value
        return value

    def _attach(self, value, depth=0):
        """Bind unpickled stand-ins to this client (for release / method calls)."""
        if depth > 3:
            return
        if isinstance(value, (ClientObjectRef, ClientActorHandle)):
            value._client = self
        elif isinstance(value, (list, tuple)):
            for v in value:
                self._attach(v, depth + 1)
        elif isinstance(value, dict):
            for v in value.values():
                self._attach(v, depth + 1)

    def _release(self, oid: bytes):
        if not self.closed:
            self.pending_release.append(oid)

    def close(self):
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass

    # ------------------------------------------------------------------ API
    def put(self, value) -> ClientObjectRef:
        return self.request("put", value)

    def get(self, refs, timeout=None):
        single = isinstance(refs, ClientObjectRef)
        out = self.request("get", ([refs] if single else list(refs), timeout))
        return out[0] if single else out

    def wait(self, refs, num_returns=1, timeout=None):
        return self.request("wait", (list(refs), num_returns, timeout))

    def submit_task(self, fn, args, kwargs, opts):
        return self.request("task", (cloudpickle.dumps(fn), args, kwargs, dict(opts)))

    def create_actor(self, cls, args, kwargs, opts):
        h = self.request("actor", (cloudpickle.dumps(cls), args, kwargs, dict(opts)))
        h._class_name = cls.__name__
        return h

    def _call_actor(self, aid, name, args, kwargs, opts):
        return self.request("call", (aid, name, args, kwargs, dict(opts)))

    def kill(self, handle, no_restart=True):
        return self.request("kill", (handle._actor_id, no_restart))

    def cancel(self, ref, force=False):
        return self.request("cancel", (ref, force))

    def get_actor(self, name, namespace=None):
        return self.request("get_actor", (name, namespace if namespace is not None else self.namespace))

    def cluster_resources(self):
        return self.request("cluster_resources")

    def available_resources(self):
        return self.request("available_resources")

    def nodes(self):
        return self.request("nodes")


def connect(address: str, namespace: Optional[str] = None) -> ClientWorker:
    hostport = address[len("ray://"):] if address.startswith("ray://") else address
    host, _, port = hostport.rpartition(":")
    return ClientWorker(host or "127.0.0.1", int(port or 10001), namespace)


__all__ = ["ClientWorker", "ClientObjectRef", "ClientActorHandle", "connect"]
