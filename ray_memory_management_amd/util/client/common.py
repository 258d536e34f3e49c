"""Wire format shared by the Ray Client and its server: u32-length-prefixed cloudpickle frames
over TCP; object refs and actor handles cross the wire as ids (reference
python/ray/util/client/common.py: ClientObjectRef / ClientActorHandle stand-ins)."""
from __future__ import annotations

import io
import socket
import struct
import threading

import cloudpickle

_HDR = struct.Struct("<I")


class ClientObjectRef:
    """Client-side stand-in for an ObjectRef living in the cluster (released when collected)."""

    __slots__ = ("_id", "_client", "__weakref__")

    def __init__(self, oid: bytes, client=None):
        self._id = oid
        self._client = client

    def binary(self) -> bytes:
        return self._id

    def hex(self) -> str:
        return self._id.hex()

    def task_id(self):
        return self._id[:16]

    def __repr__(self):
        return f"ClientObjectRef({self._id.hex()})"

    def __hash__(self):
        return hash(self._id)

    def __eq__(self, other):
        return isinstance(other, ClientObjectRef) and other._id == self._id

    def __reduce__(self):
        return (_server_ref, (self._id,))

    def __del__(self):
        c = self._client
        if c is not None:
            try:
                c._release(self._id)
            except Exception:
                pass


class ClientActorHandle:
    def __init__(self, actor_id: bytes, class_name: str, client=None):
        self._actor_id = actor_id
        self._class_name = class_name
        self._client = client

    def __getattr__(self, item):
        if item.startswith("__") and item not in ("__ray_ready__", "__ray_terminate__"):
            raise AttributeError(item)
        return ClientActorMethod(self, item)

    def __repr__(self):
        return f"ClientActor({self._class_name}, {self._actor_id.hex()})"

    def __reduce__(self):
        return (_server_actor, (self._actor_id,))


class ClientActorMethod:
    def __init__(self, handle: ClientActorHandle, name: str, opts=None):
        self._h, self._name, self._opts = handle, name, dict(opts or {})

    def remote(self, *args, **kwargs):
        return self._h._client._call_actor(self._h._actor_id, self._name, args, kwargs, self._opts)

    def options(self, **opts):
        return ClientActorMethod(self._h, self._name, {**self._opts, **opts})


# ---- server-side resolution of ids inside pickled payloads (thread-local per connection)
_tls = threading.local()


def _server_ref(oid: bytes):
    table = getattr(_tls, "table", None)
    if table is None:  # unpickled on the client side (a ref echoed back): keep the stand-in
        return ClientObjectRef(oid, getattr(_tls, "client", None))
    return table.refs[oid]


def _server_actor(aid: bytes):
    table = getattr(_tls, "table", None)
    if table is None:
        return ClientActorHandle(aid, "Actor", getattr(_tls, "client", None))
    return table.actors[aid]


def send(sock: socket.socket, obj, lock: threading.Lock) -> None:
    data = cloudpickle.dumps(obj)
    with lock:
        sock.sendall(_HDR.pack(len(data)) + data)


def send_raw(sock: socket.socket, data: bytes, lock: threading.Lock) -> None:
    with lock:
        sock.sendall(_HDR.pack(len(data)) + data)


def recv(sock: socket.socket):
    (n,) = _HDR.unpack(_recv_exact(sock, 4))
    return _recv_exact(sock, n)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("client connection closed")
        got += k
    return bytes(buf)


def loads(data: bytes):
    return cloudpickle.loads(data)


class ServerPickler(cloudpickle.Pickler):
    """Pickles results on the server: ObjectRefs / ActorHandles become id stand-ins registered in
    the connection's table."""

    def __init__(self, f, table):
        super().__init__(f, protocol=5)
        self.table = table

    def reducer_override(self, obj):
        from ray_memory_management_amd.actor import ActorHandle
        from ray_memory_management_amd.object_ref import ObjectRef

        if isinstance(obj, ObjectRef):
            oid = obj.binary()
            self.table.refs[oid] = obj
            return (_server_ref, (oid,))
        if isinstance(obj, ActorHandle):
            aid = obj._actor_id
            self.table.actors[aid] = obj
            return (_server_actor, (aid,))
        return super().reducer_override(obj)


def server_dumps(obj, table) -> bytes:
    f = io.BytesIO()
    ServerPickler(f, table).dump(obj)
    return f.getvalue()
