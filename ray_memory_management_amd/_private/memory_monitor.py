"""Node memory monitor and the memory-pressure worker-killing policy.

Parity:
* reference python/ray/_private/memory_monitor.py (node usage from /proc/meminfo, cgroup limits);
* src/ray/common/memory_monitor.cc (a periodic usage check against `memory_usage_threshold_fraction`
  every `memory_monitor_interval_ms`, 0 disables);
* src/ray/raylet/node_manager.cc:2902-3001 CreateMemoryUsageRefreshCallback /
  WorkersWithLatestSubmittedTasks: above the threshold, the registered worker whose task was assigned
  most recently is killed -- task or actor, retriable or not -- with a "System memory low at node with IP
  ..." exit detail, and no new victim is picked until that one is dead (one eviction in flight, since a
  kill can take seconds to return memory).

The policy itself runs in the head (`Head._memory_pressure`); this module holds the usage source and
the victim choice so both are unit-testable. The usage source is injectable: `_system_config=
{"memory_monitor_test_usage_file": path}` reads "used total" (bytes) or a single fraction from a file, so
tests drive memory pressure deterministically without exhausting the machine's RAM;
`{"memory_monitor_test_usage_dir": path}` sums per-process "allocations" of live pids (a killed worker's
share disappears with it, as real memory does).
"""
from __future__ import annotations

import os
import time
from typing import Callable, Optional, Tuple


def _read_meminfo():
    info = {}
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                k, v = line.split(":", 1)
                info[k] = int(v.split()[0]) * 1024
    except OSError:
        pass
    return info


def get_used_and_total():
    # respect cgroup limits (containers)
    for lim_path, use_path in (("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory.current"),
                               ("/sys/fs/cgroup/memory/memory.limit_in_bytes",
                                "/sys/fs/cgroup/memory/memory.usage_in_bytes")):
        try:
            with open(lim_path) as f:
                lim = f.read().strip()
            with open(use_path) as f:
                used = int(f.read().strip())
            if lim != "max" and int(lim) < (1 << 60):
                return used, int(lim)
        except (OSError, ValueError):
            continue
    mi = _read_meminfo()
    total = mi.get("MemTotal", 0)
    avail = mi.get("MemAvailable", total)
    return total - avail, total


def file_usage_source(path: str) -> Callable[[], Tuple[int, int]]:
    """Usage from a file: "used total" in bytes, or one fraction in [0, 1] (of the real total). A missing
    or unreadable file falls back to the real node usage."""

    def read():
        try:
            with open(path) as f:
                parts = f.read().split()
        except OSError:
            return get_used_and_total()
        try:
            if len(parts) >= 2:
                return int(float(parts[0])), int(float(parts[1]))
            if len(parts) == 1:
                _, total = get_used_and_total()
                return int(float(parts[0]) * total), total
        except ValueError:
            pass
        return get_used_and_total()

    return read


def dir_usage_source(path: str, total: int = 16 << 30) -> Callable[[], Tuple[int, int]]:
    """Simulated node memory for tests: every process "allocates" by writing a byte count into
    `<path>/<its pid>`; usage is the sum over processes still alive, so a killed worker's memory is
    returned to the node exactly as a real kill returns it. `<path>/total` overrides the capacity."""

    def read():
        used, cap = 0, total
        try:
            names = os.listdir(path)
        except OSError:
            return 0, cap
        for n in names:
            try:
                with open(os.path.join(path, n)) as f:
                    v = int(float(f.read().strip() or 0))
            except (OSError, ValueError):
                continue
            if n == "total":
                cap = v
            elif n.isdigit() and pid_alive(int(n)):
                used += v
        return used, cap

    return read


def format_eviction_message(ip: str, used: int, total: int, threshold: float, name: str, kind: str,
                            ident: str) -> str:
    """The exit detail of a worker killed for memory (reference node_manager.cc:2932-2945)."""
    gb = 1024 ** 3
    frac = used / total if total else 0.0
    return (f"System memory low at node with IP {ip}. Used memory ({used / gb:.2f}GB) / total capacity "
            f"({total / gb:.2f}GB) ({frac:.6f}) exceeds threshold {threshold}, killing latest task with name "
            f"{name} and {kind} ID {ident} to avoid running out of memory.\n"
            "This may indicate a memory leak in a task or actor, or that too many tasks are running in parallel.")


class MemoryMonitor:
    """Periodic usage check (`interval_s`) against `threshold`, plus the single in-flight eviction target."""

    def __init__(self, threshold: float = 0.95, interval_s: float = 0.25,
                 usage_fn: Optional[Callable[[], Tuple[int, int]]] = None):
        self.threshold = float(threshold)
        self.interval_s = max(float(interval_s), 0.0)
        self.usage_fn = usage_fn or get_used_and_total
        self.last = 0.0
        self.last_used = 0
        self.last_total = 0
        self.above = False
        self.kills = 0
        self.task_evictions = 0
        self.actor_evictions = 0
        self.target = None          # the worker being evicted (one at a time)
        self.target_since = 0.0
        self.last_wait_log = 0.0

    def snapshot(self):
        used, total = self.usage_fn()
        return {"used": used, "total": total, "threshold": self.threshold, "kills": self.kills,
                "task_evictions": self.task_evictions, "actor_evictions": self.actor_evictions,
                "interval_ms": self.interval_s * 1000.0,
                "eviction_in_flight": self.target is not None}

    def refresh(self, now: Optional[float] = None) -> Optional[bool]:
        """Re-read usage if the interval elapsed: True / False above the threshold, None when not due."""
        now = time.time() if now is None else now
        if now - self.last < self.interval_s:
            return None
        self.last = now
        used, total = self.usage_fn()
        self.last_used, self.last_total = used, total
        self.above = total > 0 and used / total > self.threshold
        return self.above

    # kept for callers of the round-5 API
    def over_threshold(self) -> bool:
        return bool(self.refresh())

    @staticmethod
    def pick_victim(workers):
        """The worker whose task (or actor) was assigned most recently (WorkersWithLatestSubmittedTasks).
        `workers` yields (assigned_time, worker) for every worker with an assigned task or actor."""
        best = None
        for t, w in workers:
            if best is None or t > best[0]:
                best = (t, w)
        return None if best is None else best[1]

    def record_kill(self, is_actor: bool, target, now: Optional[float] = None):
        self.kills += 1
        if is_actor:
            self.actor_evictions += 1
        else:
            self.task_evictions += 1
        self.target = target
        self.target_since = time.time() if now is None else now


def pid_alive(pid: Optional[int]) -> bool:
    if not pid:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            st = f.read()
        return st[st.rindex(")") + 2] not in "ZX"
    except (OSError, ValueError, IndexError):
        return True
