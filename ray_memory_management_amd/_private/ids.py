"""Binary IDs. Parity: reference src/ray/common/id.h (TaskID/ObjectID/ActorID/...).

ObjectID (20 bytes) = TaskID (16 bytes) + big-endian u32 index; index 1..n are task returns,
index >= 0x80000000 are ``put`` objects. TaskIDs are minted locally by the submitting process as
(8-byte process prefix, 8-byte counter) — no round trip to the head.
"""
from __future__ import annotations

import itertools
import os
import struct
import threading

ID_SIZE = 20
TASK_ID_SIZE = 16
PUT_INDEX_BASE = 0x80000000

_prefix = os.urandom(8)
_counter = itertools.count(1)
_lock = threading.Lock()


def _reseed_after_fork():
    global _prefix, _counter
    _prefix = os.urandom(8)
    _counter = itertools.count(1)


os.register_at_fork(after_in_child=_reseed_after_fork)


def new_task_id() -> bytes:
    return _prefix + struct.pack(">Q", next(_counter))


def object_id_for_return(task_id: bytes, index: int) -> bytes:
    return task_id + struct.pack(">I", index)


def new_put_id() -> bytes:
    return new_task_id() + struct.pack(">I", PUT_INDEX_BASE)


def task_id_of(object_id: bytes) -> bytes:
    return object_id[:TASK_ID_SIZE]


def random_id(n: int = ID_SIZE) -> bytes:
    return os.urandom(n)


class BaseID:
    __slots__ = ("_b",)
    SIZE = ID_SIZE

    def __init__(self, b: bytes):
        if not isinstance(b, (bytes, bytearray)) or len(b) != self.SIZE:
            raise ValueError(f"{type(self).__name__} needs {self.SIZE} bytes")
        self._b = bytes(b)

    @classmethod
    def from_random(cls):
        return cls(os.urandom(cls.SIZE))

    @classmethod
    def from_hex(cls, h: str):
        return cls(bytes.fromhex(h))

    @classmethod
    def nil(cls):
        return cls(b"\xff" * cls.SIZE)

    def is_nil(self) -> bool:
        return self._b == b"\xff" * self.SIZE

    def binary(self) -> bytes:
        return self._b

    def hex(self) -> str:
        return self._b.hex()

    def __eq__(self, other):
        return type(other) is type(self) and other._b == self._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return f"{type(self).__name__}({self.hex()})"

    def __reduce__(self):
        return type(self), (self._b,)


class ObjectID(BaseID):
    SIZE = ID_SIZE


class TaskID(BaseID):
    SIZE = TASK_ID_SIZE


class ActorID(BaseID):
    SIZE = 16


class NodeID(BaseID):
    SIZE = 16


class JobID(BaseID):
    SIZE = 4


class WorkerID(BaseID):
    SIZE = 16


class PlacementGroupID(BaseID):
    SIZE = 16


class FunctionID(BaseID):
    SIZE = 20


class UniqueID(BaseID):
    SIZE = 20


class ActorClassID(BaseID):
    SIZE = 20
