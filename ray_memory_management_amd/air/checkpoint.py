"""Checkpoint: a dict- or directory-backed snapshot. Parity: reference python/ray/air/checkpoint.py
(from_dict/to_dict/from_directory/to_directory/as_directory, uri)."""
from __future__ import annotations

import contextlib
import os
import pickle
import shutil
import tempfile
import uuid
from typing import Any, Dict, Optional

_DICT_FILE = "dict_checkpoint.pkl"


class Checkpoint:
    def __init__(self, local_path: Optional[str] = None, data_dict: Optional[dict] = None, uri: Optional[str] = None):
        self._local_path = local_path
        self._data_dict = data_dict
        self._uri = uri
        self.id = uuid.uuid4().hex

    # ---- constructors
    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Checkpoint":
        return cls(data_dict=dict(data))

    @classmethod
    def from_directory(cls, path: str) -> "Checkpoint":
        return cls(local_path=os.path.abspath(path))

    @classmethod
    def from_uri(cls, uri: str) -> "Checkpoint":
        if uri.startswith("file://"):
            return cls.from_directory(uri[len("file://"):])
        raise ValueError(f"unsupported checkpoint uri {uri}")

    @classmethod
    def from_checkpoint(cls, other: "Checkpoint") -> "Checkpoint":
        return cls(other._local_path, other._data_dict, other._uri)

    # ---- accessors
    def to_dict(self) -> Dict[str, Any]:
        if self._data_dict is not None:
            return dict(self._data_dict)
        p = os.path.join(self._local_path, _DICT_FILE)
        if os.path.exists(p):
            with open(p, "rb") as f:
                return pickle.load(f)  # our own file format (written by to_directory)
        out = {}
        for root, _, files in os.walk(self._local_path):
            for fn in files:
                rel = os.path.relpath(os.path.join(root, fn), self._local_path)
                with open(os.path.join(root, fn), "rb") as f:
                    out[rel] = f.read()
        return out

    def to_directory(self, path: Optional[str] = None) -> str:
        path = path or tempfile.mkdtemp(prefix="checkpoint_")
        os.makedirs(path, exist_ok=True)
        if self._data_dict is not None:
            with open(os.path.join(path, _DICT_FILE), "wb") as f:
                pickle.dump(self._data_dict, f)
        elif self._local_path and os.path.abspath(self._local_path) != os.path.abspath(path):
            shutil.copytree(self._local_path, path, dirs_exist_ok=True)
        return path

    @contextlib.contextmanager
    def as_directory(self):
        if self._local_path is not None:
            yield self._local_path
        else:
            d = self.to_directory()
            try:
                yield d
            finally:
                shutil.rmtree(d, ignore_errors=True)

    def to_uri(self, uri: str) -> str:
        if not uri.startswith("file://"):
            raise ValueError("only file:// URIs are supported")
        self.to_directory(uri[len("file://"):])
        return uri

    @property
    def uri(self):
        return self._uri or (f"file://{self._local_path}" if self._local_path else None)

    def get_internal_representation(self):
        return ("local_path", self._local_path) if self._local_path else ("data_dict", self._data_dict)

    def __repr__(self):
        kind = "dict" if self._data_dict is not None else self._local_path
        return f"Checkpoint({kind})"

    def __eq__(self, other):
        return isinstance(other, Checkpoint) and other.get_internal_representation() == self.get_internal_representation()

    def __hash__(self):
        return hash(self.id)
