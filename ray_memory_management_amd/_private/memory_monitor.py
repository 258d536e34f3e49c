"""Node memory monitor. Parity: reference python/ray/_private/memory_monitor.py and the raylet's
memory-pressure worker killing (src/ray/raylet/worker_killing_policy.cc in later versions):
when node memory usage crosses `memory_usage_threshold`, the most recently started retriable
task worker is killed (its task is retried), which is the reference's policy."""
from __future__ import annotations

import os
import time


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


class MemoryMonitor:
    def __init__(self, threshold: float = 0.95, min_interval: float = 0.25):
        self.threshold = threshold
        self.min_interval = min_interval
        self.last = 0.0
        self.last_used = 0
        self.last_total = 0
        self.kills = 0

    def snapshot(self):
        used, total = get_used_and_total()
        return {"used": used, "total": total, "threshold": self.threshold, "kills": self.kills}

    def over_threshold(self) -> bool:
        now = time.time()
        if now - self.last < self.min_interval:
            return False
        self.last = now
        used, total = get_used_and_total()
        self.last_used, self.last_total = used, total
        return total > 0 and used / total > self.threshold

    def pick_victim(self, head):
        if self.threshold >= 1.0 or not self.over_threshold():
            return None
        cands = []
        for w in head.workers.values():
            if w.task is None or w.state != "BUSY":
                continue
            t = head.tasks.get(w.task)
            if t is None or t.retries_left == 0:
                continue
            cands.append((t.start_time or 0, w))
        if not cands:
            return None
        cands.sort(key=lambda x: x[0])
        self.kills += 1
        return cands[-1][1]
