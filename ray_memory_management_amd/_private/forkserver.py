"""Worker fork server: start worker processes by fork() from a pre-imported template process.

Role parity: the reference's raylet worker pool starts worker processes (src/ray/raylet/
worker_pool.cc StartWorkerProcess, with prestart and maximum_startup_concurrency) — each a fresh
interpreter. Starting a Python interpreter and importing the runtime costs ~100+ ms of CPU per
worker, which bounds actor creation on one node (release/benchmarks/distributed/test_many_actors.py)
at a few dozen per second per CPU. Here the head starts ONE template process that imports the worker
modules once and never touches a GPU; each worker is a fork() of it (copy-on-write pages, a few
milliseconds), which then applies the worker's own environment (GPU visibility, runtime env) before
anything reads it and runs ``worker_main.main()``.

Protocol (Unix socket, JSON lines): the head sends {"env": {...}, "log": path} (fork a worker) or
{"kill": pid, "sig": n}; the template answers a fork with {"pid": child_pid} or {"error": msg} and,
unprompted, reports every child it reaps as {"exit": pid, "code": c} (c = exit status, or -signal as
in subprocess). The head therefore learns real exit codes (OOM kill -9 vs segfault -11), and every
signal to a worker is sent by the template, which only signals its own children that it has not
reaped yet: a recycled pid can never be hit.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import sys
import time


def _child(env: dict, log: str, listen: socket.socket, conn: socket.socket):
    try:
        listen.close()
        conn.close()
        os.setsid()
        signal.signal(signal.SIGCHLD, signal.SIG_DFL)
        signal.signal(signal.SIGINT, signal.SIG_DFL)
        signal.signal(signal.SIGTERM, signal.SIG_DFL)
        fd = os.open(log, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(fd, 1)
        os.dup2(fd, 2)
        os.close(fd)
        nul = os.open(os.devnull, os.O_RDONLY)
        os.dup2(nul, 0)
        os.close(nul)
        sys.stdout = os.fdopen(1, "w", buffering=1)
        sys.stderr = os.fdopen(2, "w", buffering=1)
        os.environ.clear()
        os.environ.update(env)
        import random

        random.seed()
        try:
            import numpy as np

            np.random.seed(None)
        except ImportError:
            pass
        from ray_memory_management_amd._private import worker_main

        worker_main.main()
    except SystemExit as e:
        os._exit(int(e.code or 0) if isinstance(e.code, int) else 1)
    except BaseException:  # noqa: BLE001
        import traceback

        traceback.print_exc()
        os._exit(1)
    os._exit(0)


def serve(path: str):
    # the modules every worker needs, imported ONCE here (none of them initialises a GPU)
    import numpy  # noqa: F401
    import cloudpickle  # noqa: F401

    from ray_memory_management_amd._private import worker_main  # noqa: F401

    for mod in filter(None, os.environ.get("RMM_FORKSERVER_PRELOAD", "").split(",")):
        try:
            __import__(mod)
        except ImportError:
            pass

    children = set()   # forked, not reaped yet: the only pids this process ever signals
    exited = []        # (pid, code) reaped, not reported yet

    def reap(*_):
        while True:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                return
            if pid == 0:
                return
            children.discard(pid)
            exited.append((pid, os.waitstatus_to_exitcode(status)))

    signal.signal(signal.SIGCHLD, reap)
    listen = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    listen.bind(path)
    listen.listen(64)
    head_pid = os.getppid()
    listen.settimeout(1.0)
    conn = None
    buf = b""

    def send(obj) -> None:
        if conn is not None:
            try:
                conn.sendall(json.dumps(obj).encode() + b"\n")
            except OSError:
                pass

    while True:
        if conn is None:
            try:
                conn, _ = listen.accept()
                conn.settimeout(0.05)  # exit reports go out within ~50 ms of the reap
            except socket.timeout:
                if os.getppid() != head_pid:  # the head is gone
                    return
                continue
            except InterruptedError:
                continue
        while exited:
            pid, code = exited.pop(0)
            send({"exit": pid, "code": code})
        try:
            data = conn.recv(1 << 20)
        except socket.timeout:
            if os.getppid() != head_pid:
                return
            continue
        except InterruptedError:
            continue
        except OSError:
            data = b""
        if not data:
            conn.close()
            conn, buf = None, b""
            continue
        buf += data
        while b"\n" in buf:
            line, buf = buf.split(b"\n", 1)
            try:
                req = json.loads(line)
                if "kill" in req:
                    pid = int(req["kill"])
                    if pid in children:  # still ours and not reaped: the pid cannot have been reused
                        try:
                            os.kill(pid, int(req.get("sig", signal.SIGKILL)))
                        except ProcessLookupError:
                            pass
                    continue
                # SIGCHLD stays blocked across fork + add: a child that exits at once is reaped only after
                # it is in `children`, so a reaped pid can never be left there (and later signalled after
                # the kernel reused it)
                signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGCHLD})
                try:
                    pid = os.fork()
                    if pid == 0:
                        signal.pthread_sigmask(signal.SIG_UNBLOCK, {signal.SIGCHLD})
                        _child(req["env"], req["log"], listen, conn)
                    children.add(pid)
                finally:
                    signal.pthread_sigmask(signal.SIG_UNBLOCK, {signal.SIGCHLD})
                reply = {"pid": pid}
            except Exception as e:  # noqa: BLE001
                reply = {"error": repr(e)}
            send(reply)


class ForkedProc:
    """Popen-like handle of a worker forked by the template. Not our child: its exit code arrives as the
    template's {"exit": pid, "code": c} report (the real status: -9 for an OOM kill, -11 for a
    segfault), and signals are sent by the template, which only signals children it has not reaped."""

    def __init__(self, pid: int, client: "ForkClient"):
        self.pid = pid
        self.returncode = None
        self._client = client

    def poll(self):
        if self.returncode is None:
            self._client.drain()
            code = self._client.exit_codes.pop(self.pid, None)
            if code is not None:
                self.returncode = code
            elif self._client.lost and not _pid_exists(self.pid):
                self.returncode = -1  # the template is gone: no exit report will come
        return self.returncode

    def wait(self, timeout=None):
        # a short wait (the head's reap-after-death) polls for ~the template's report period; never a
        # long sleep on the head's event loop
        deadline = None if timeout is None else time.time() + timeout
        while self.poll() is None:
            if deadline is not None and time.time() >= deadline:
                import subprocess

                raise subprocess.TimeoutExpired(f"pid {self.pid}", timeout)
            time.sleep(0.005)
        return self.returncode

    def send_signal(self, sig):
        if self.returncode is None:
            self._client.signal(self.pid, sig)

    def kill(self):
        self.send_signal(signal.SIGKILL)

    def terminate(self):
        self.send_signal(signal.SIGTERM)


def _pid_exists(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        pass
    return True


class ForkClient:
    """The head's side: start the template, ask it for workers."""

    def __init__(self, session_dir: str, env: dict):
        import subprocess

        self.path = os.path.join(session_dir, f"forkserver-{os.getpid()}.sock")
        try:
            os.unlink(self.path)
        except OSError:
            pass
        log = open(os.path.join(session_dir, "logs", "forkserver.log"), "ab")
        self.proc = subprocess.Popen([sys.executable, "-u", "-m", "ray_memory_management_amd._private.forkserver",
                                      self.path], env=env, stdout=log, stderr=subprocess.STDOUT,
                                     stdin=subprocess.DEVNULL, start_new_session=True)
        log.close()
        self.sock = None
        self.buf = b""
        t0 = time.time()
        while time.time() - t0 < 30.0:
            if self.proc.poll() is not None:
                raise RuntimeError("fork server exited at startup")
            try:
                s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                s.connect(self.path)
                s.settimeout(10.0)
                self.sock = s
                break
            except OSError:
                time.sleep(0.01)
        if self.sock is None:
            raise RuntimeError("fork server did not come up")

        self.exit_codes = {}  # pid -> exit code reported by the template, until its ForkedProc polls it
        self.lost = False     # the template's connection closed

    def _handle(self, line: bytes):
        rep = json.loads(line)
        if "exit" in rep:
            self.exit_codes[int(rep["exit"])] = int(rep["code"])
            return None
        return rep

    def drain(self) -> None:
        """Read the exit reports that arrived (non-blocking)."""
        if self.sock is None or self.lost:
            return
        try:
            self.sock.setblocking(False)
            while True:
                data = self.sock.recv(1 << 16)
                if not data:
                    self.lost = True
                    break
                self.buf += data
        except (BlockingIOError, InterruptedError):
            pass
        except OSError:
            self.lost = True
        finally:
            try:
                self.sock.settimeout(10.0)
            except OSError:
                pass
        while b"\n" in self.buf:
            line, self.buf = self.buf.split(b"\n", 1)
            self._handle(line)

    def spawn(self, env: dict, log: str) -> ForkedProc:
        self.sock.sendall(json.dumps({"env": env, "log": log}).encode() + b"\n")
        while True:
            while b"\n" not in self.buf:
                data = self.sock.recv(4096)
                if not data:
                    self.lost = True
                    raise RuntimeError("fork server closed the connection")
                self.buf += data
            line, self.buf = self.buf.split(b"\n", 1)
            rep = self._handle(line)
            if rep is not None:
                break
        if "pid" not in rep:
            raise RuntimeError(f"fork server: {rep.get('error')}")
        return ForkedProc(int(rep["pid"]), self)

    def signal(self, pid: int, sig: int) -> None:
        try:
            self.sock.sendall(json.dumps({"kill": int(pid), "sig": int(sig)}).encode() + b"\n")
        except OSError:
            self.lost = True

    def close(self):
        try:
            if self.sock is not None:
                self.sock.close()
        except OSError:
            pass
        if self.proc.poll() is None:
            self.proc.kill()
        try:
            os.unlink(self.path)
        except OSError:
            pass


if __name__ == "__main__":
    serve(sys.argv[1])
