"""Remote debugger. Parity: reference python/ray/util/rpdb.py (`ray.util.pdb.set_trace()` inside a
task/actor opens a pdb session on a TCP socket and registers it in the cluster KV so a user can
attach — `rmm debug` there, any line client such as `nc` here)."""
from __future__ import annotations

import json
import os
import pdb
import socket
import sys
import time
import uuid


class _SocketIO:
    def __init__(self, conn):
        self._conn = conn
        self._r = conn.makefile("r")
        self._w = conn.makefile("w")

    def readline(self, *a):
        return self._r.readline(*a)

    def write(self, s):
        self._w.write(s)
        self._w.flush()

    def flush(self):
        self._w.flush()

    def close(self):
        for f in (self._r, self._w):
            try:
                f.close()
            except Exception:
                pass
        self._conn.close()


class RemotePdb(pdb.Pdb):
    def __init__(self, host: str = "127.0.0.1", port: int = 0, timeout: float = 300.0):
        self._listen = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._listen.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._listen.bind((host, port))
        self._listen.listen(1)
        self._listen.settimeout(timeout)
        self.address = self._listen.getsockname()
        self._io = None

    def wait_for_client(self):
        conn, _ = self._listen.accept()
        self._io = _SocketIO(conn)
        pdb.Pdb.__init__(self, stdin=self._io, stdout=self._io, nosigint=True)
        self.use_rawinput = False
        self.prompt = "(rmm-pdb) "

    def do_continue(self, arg):
        r = pdb.Pdb.do_continue(self, arg)
        self._close()
        return r

    do_c = do_cont = do_continue

    def _close(self):
        if self._io is not None:
            self._io.close()
            self._io = None
        self._listen.close()


def _register(address, breakpoint_uuid):
    try:
        from ray_memory_management_amd import internal

        internal._internal_kv_put(f"RMM_PDB_{breakpoint_uuid}", json.dumps(
            {"host": address[0], "port": address[1], "pid": os.getpid(), "time": time.time()}).encode(),
            namespace="rmm_pdb")
    except Exception:
        pass


def list_breakpoints():
    """Active breakpoints registered in the cluster KV: [{uuid, host, port, pid}]."""
    from ray_memory_management_amd import internal

    out = []
    for k in internal._internal_kv_list("RMM_PDB_", namespace="rmm_pdb"):
        v = internal._internal_kv_get(k, namespace="rmm_pdb")
        if v:
            key = k.decode() if isinstance(k, bytes) else k
            out.append({"uuid": key[len("RMM_PDB_"):], **json.loads(v)})
    return out


def set_trace(breakpoint_uuid: str = None, host: str = "127.0.0.1", port: int = 0, timeout: float = 300.0):
    """Stop here and serve a pdb session on host:port (printed to stderr and registered in KV)."""
    breakpoint_uuid = breakpoint_uuid or uuid.uuid4().hex
    dbg = RemotePdb(host, port, timeout)
    _register(dbg.address, breakpoint_uuid)
    print(f"RemotePdb session open at {dbg.address[0]}:{dbg.address[1]} (breakpoint {breakpoint_uuid})",
          file=sys.stderr, flush=True)
    try:
        dbg.wait_for_client()
    except socket.timeout:
        dbg._close()
        return
    finally:
        try:
            from ray_memory_management_amd import internal

            internal._internal_kv_del(f"RMM_PDB_{breakpoint_uuid}", namespace="rmm_pdb")
        except Exception:
            pass
    dbg.set_trace(sys._getframe().f_back)
