"""NUMA-local CPU placement for processes that drive a GPU.

A rollout worker polls completion words the GPU writes into pinned host memory and writes the envs'
newest frames there for the GPU to read over PCIe; a learner spins on its device syncs. When such a
process (and the pinned buffers it first-touches) lands on the socket the GPU is NOT attached to,
every one of those round trips crosses the inter-socket link. `pin_to_gpu` restricts the process
(all its current threads; threads created later inherit the mask) to the CPUs local to the GPU's PCIe
root, intersected with the CPUs it may use. It is a no-op when sysfs does not say, when the
intersection is smaller than `min_cpus`, or with RMM_NUMA_PIN=0.

Reference analogue: Ray leaves CPU placement to the OS (no NUMA binding of GPU workers); this is
an MI355X-node addition (8 GPUs over 2 sockets)."""
from __future__ import annotations

import os
from typing import Optional, Set


def parse_cpulist(text: str) -> Set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11} (the sysfs cpulist format)."""
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def pci_local_cpus(bus_id: str, sysfs: str = "/sys") -> Optional[Set[int]]:
    """CPUs local to the PCI device `bus_id` ('dddd:bb:dd.f'), or None when sysfs does not say."""
    dev = os.path.join(sysfs, "bus", "pci", "devices", bus_id.lower())
    try:
        with open(os.path.join(dev, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
        if cpus:
            return cpus
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(dev, "numa_node")) as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        with open(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read()) or None
    except (OSError, ValueError):
        return None


def pin_to_gpu(device: int = 0, min_cpus: int = 4, sysfs: str = "/sys") -> Optional[Set[int]]:
    """Restrict the calling thread to the CPUs local to visible GPU `device` (see the module doc).
    Returns the new CPU set, or None when nothing was changed."""
    if os.environ.get("RMM_NUMA_PIN", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    try:
        from ray_memory_management_amd._native import require_hip

        bus = require_hip().pci_bus_id(int(device))
    except Exception:  # noqa: BLE001 - no HIP, no device: nothing to place
        return None
    local = pci_local_cpus(bus, sysfs)
    if not local:
        return None
    cur = os.sched_getaffinity(0)
    want = cur & local
    if len(want) < min_cpus or want == cur:
        return None
    try:
        os.sched_setaffinity(0, want)
    except OSError:
        return None
    # the process's other threads too (sched_setaffinity is per thread on Linux; threads created later
    # inherit their creator's mask)
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(tid), want)
            except OSError:
                pass
    except OSError:
        pass
    return want
