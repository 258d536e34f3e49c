"""Framed message transport over Unix-domain sockets.

Frame = u32 little-endian length + pickle-5 payload. Payloads are tuples ``(msg_type, ...)``.
Parity: the reference uses gRPC + flatbuffers between core worker / raylet / GCS
(src/ray/rpc/*, src/ray/raylet/format/node_manager.fbs); on one node a Unix socket with pickled
tuples is lower latency and is all the control plane needs (the data plane is the shm store).
"""
from __future__ import annotations

import pickle
import socket
import struct
import threading

_HDR = struct.Struct("<I")
MAX_FRAME = 1 << 31

# ---- message types (worker/driver -> head)
REGISTER = 1
SUBMIT_TASK = 2
CREATE_ACTOR = 3
TASK_DONE = 4
REF_DELTAS = 5
KV_PUT = 6
KV_GET = 7
KV_DEL = 8
KV_KEYS = 9
GET_ACTOR = 10
KILL_ACTOR = 11
CANCEL = 12
PG_CREATE = 13
PG_REMOVE = 14
PG_WAIT = 15
PG_TABLE = 16
BLOCKED = 17
UNBLOCKED = 18
STATE = 19
ACTOR_READY = 20
WAIT_ACTOR = 21
CONTAINED = 22
SHUTDOWN = 23
ACTOR_FAILED_INIT = 24
EVENTS = 25
FREE = 26
JOB_INFO = 27
ADD_NODE = 28
REMOVE_NODE = 29
ACTOR_EXITING = 30
GPU_OBJECT = 31
GLOBAL_GC = 32
LEASE_REQUEST = 33   # owner asks for a worker lease (direct task submission)
LEASE_RETURN = 34    # owner hands a lease back (optionally: kill the worker)
DIRECT_DONE = 35     # batched completion records of directly submitted tasks (lineage + state)
FN_EXPORT = 36       # function blob for the head's table (first direct submission of a function)
EXIT_DETAIL = 37     # (EXIT_DETAIL, rid, worker id | direct addr | actor id) -> why the head killed it, or None

# ---- head -> worker
EXECUTE = 101
CREATE_ACTOR_INSTANCE = 102
EXIT = 103
CANCEL_TASK = 104
REPLY = 105
FREE_GPU = 106
TRIGGER_GC = 107
NODES_CHANGED = 108  # (NODES_CHANGED, multi_node: bool)
PUSH_ERROR = 109     # (PUSH_ERROR, error_type, message, job_id): a warning for the job's driver

# ---- caller -> actor (direct transport)
ACTOR_TASK = 201
ACTOR_HELLO = 202
DIRECT_TASK = 203    # owner -> leased worker: (DIRECT_TASK, spec, fn_blob, info)


def dumps(obj) -> bytes:
    return pickle.dumps(obj, protocol=5)


def send(sock: socket.socket, obj, lock: threading.Lock | None = None) -> None:
    data = pickle.dumps(obj, protocol=5)
    frame = _HDR.pack(len(data)) + data
    if lock is None:
        sock.sendall(frame)
    else:
        with lock:
            sock.sendall(frame)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("socket closed")
        got += k
    return bytes(buf)


def recv(sock: socket.socket):
    (n,) = _HDR.unpack(_recv_exact(sock, 4))
    return pickle.loads(_recv_exact(sock, n))


class FrameReader:
    """Incremental frame parser for non-blocking sockets (used by the head's event loop)."""

    __slots__ = ("buf",)

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes):
        self.buf += data
        out = []
        buf = self.buf
        pos = 0
        n = len(buf)
        while n - pos >= 4:
            (ln,) = _HDR.unpack_from(buf, pos)
            if n - pos - 4 < ln:
                break
            out.append(pickle.loads(bytes(buf[pos + 4:pos + 4 + ln])))
            pos += 4 + ln
        if pos:
            del buf[:pos]
        return out


def frame(obj) -> bytes:
    data = pickle.dumps(obj, protocol=5)
    return _HDR.pack(len(data)) + data
