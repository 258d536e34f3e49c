"""GPU reporter for the dashboard: per-GPU utilization / HBM and per-process GPU object-store state.

Parity: reference dashboard/modules/reporter/reporter_agent.py:92-98 (``_get_gpu_usage``: per-GPU
utilization and memory through gpustat / NVML, exported as node gauges). On an MI355X node the same
numbers come from the amdgpu driver's sysfs files (no HIP context: the dashboard process never
initialises the GPU), with amdsmi as the fallback when sysfs is not mounted:

  /sys/class/drm/cardN/device/gpu_busy_percent, mem_info_vram_{total,used}, mem_info_gtt_used,
  uevent (PCI_SLOT_NAME), hwmon/hwmon*/{temp1_input, power1_average}

and, because this framework has an HBM object store the reference does not, the occupancy and
spill state of every process's GPU store: each process that owns one publishes its counters into
the internal KV (namespace ``_rmm_reporter``) every ``gpu_store_report_interval_s`` seconds
(``publish_store_stats``); the dashboard lists them with their age and whether the process lives.
"""
from __future__ import annotations

import glob
import json
import os
import threading
import time
from typing import Dict, List

NAMESPACE = "_rmm_reporter"
_AMD_VENDOR = "0x1002"


def _read(path: str, cast=int, default=None):
    try:
        with open(path) as f:
            return cast(f.read().strip())
    except (OSError, ValueError):
        return default


def _sysfs_root() -> str:
    return os.environ.get("RMM_SYSFS_DRM_ROOT", "/sys/class/drm")


def gpu_devices() -> List[Dict]:
    """One dict per AMD GPU the driver exposes (sysfs; amdsmi if sysfs shows none)."""
    out = []
    cards = sorted(glob.glob(os.path.join(_sysfs_root(), "card[0-9]*")),
                   key=lambda p: int("".join(ch for ch in os.path.basename(p) if ch.isdigit()) or 0))
    for card in cards:
        dev = os.path.join(card, "device")
        if _read(os.path.join(dev, "vendor"), str, "") != _AMD_VENDOR:
            continue
        total = _read(os.path.join(dev, "mem_info_vram_total"))
        if total is None:
            continue
        pci = None
        try:
            with open(os.path.join(dev, "uevent")) as f:
                for line in f:
                    if line.startswith("PCI_SLOT_NAME="):
                        pci = line.split("=", 1)[1].strip().lower()
        except OSError:
            pass
        d = {"index": len(out), "card": os.path.basename(card), "pci_bus_id": pci,
             "busy_percent": _read(os.path.join(dev, "gpu_busy_percent")),
             "vram_total_bytes": total, "vram_used_bytes": _read(os.path.join(dev, "mem_info_vram_used")),
             "gtt_used_bytes": _read(os.path.join(dev, "mem_info_gtt_used"))}
        hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
        if hw:
            t = _read(os.path.join(hw[0], "temp1_input"))
            p = _read(os.path.join(hw[0], "power1_average"))
            d["temperature_c"] = None if t is None else t / 1000.0
            d["power_w"] = None if p is None else p / 1e6
        out.append(d)
    if out:
        return out
    return _amdsmi_devices()


def _amdsmi_devices() -> List[Dict]:
    try:
        import amdsmi  # ROCm's SMI library (driver queries only, no HIP context)
    except ImportError:
        return []
    try:
        amdsmi.amdsmi_init()
    except Exception:  # noqa: BLE001 - no driver on this host
        return []
    out = []
    try:
        for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
            d = {"index": i, "card": None, "pci_bus_id": None}
            try:
                d["pci_bus_id"] = str(amdsmi.amdsmi_get_gpu_device_bdf(h)).lower()
            except Exception:  # noqa: BLE001
                pass
            try:
                act = amdsmi.amdsmi_get_gpu_activity(h)
                d["busy_percent"] = act.get("gfx_activity")
            except Exception:  # noqa: BLE001
                d["busy_percent"] = None
            try:
                d["vram_total_bytes"] = int(amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM))
                d["vram_used_bytes"] = int(amdsmi.amdsmi_get_gpu_memory_usage(h, amdsmi.AmdSmiMemoryType.VRAM))
            except Exception:  # noqa: BLE001
                d["vram_total_bytes"] = d["vram_used_bytes"] = None
            out.append(d)
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass
    return out


# ------------------------------------------------------------------ GPU object-store publication
_pub_lock = threading.Lock()
_pub_started = False


def publish_store_stats(worker, interval_s: float = 0.0) -> None:
    """Start (once per process) a daemon thread that writes this process's GPU-store counters to
    the internal KV every `interval_s` seconds (config gpu_store_report_interval_s, default 2)."""
    global _pub_started
    cfg = getattr(worker, "config", None) or {}
    interval_s = interval_s or float(cfg.get("gpu_store_report_interval_s", 2.0))
    if interval_s <= 0:
        return
    with _pub_lock:
        if _pub_started:
            return
        _pub_started = True

    def loop():
        from ray_memory_management_amd import internal
        from ray_memory_management_amd._private import gpu_object_store as gos

        pid = os.getpid()
        while True:
            try:
                if not internal._internal_kv_initialized():
                    return
                for dev, st in gos.stats(worker).items():
                    rec = {"pid": pid, "device": int(dev), "pci_bus_id": gos.pci_bus_id(int(dev)),
                           "time": time.time(), "stats": {k: v for k, v in dict(st).items()
                                                          if isinstance(v, (int, float))}}
                    internal._internal_kv_put(f"gpu_store/{pid}/{dev}", json.dumps(rec), True, namespace=NAMESPACE)
            except Exception:  # noqa: BLE001 - the cluster is going away; stop quietly
                return
            time.sleep(interval_s)

    threading.Thread(target=loop, daemon=True, name="rmm-gpu-store-reporter").start()


def gpu_object_stores() -> List[Dict]:
    """Every published GPU-store record (latest per process and device), with its age and liveness."""
    from ray_memory_management_amd import internal

    out = []
    try:
        keys = internal._internal_kv_list("gpu_store/", namespace=NAMESPACE) or []
    except Exception:  # noqa: BLE001
        return out
    now = time.time()
    for k in keys:
        raw = internal._internal_kv_get(k, namespace=NAMESPACE)
        if not raw:
            continue
        try:
            rec = json.loads(raw)
        except ValueError:
            continue
        rec["age_s"] = round(now - float(rec.get("time", now)), 3)
        try:
            os.kill(int(rec["pid"]), 0)
            rec["alive"] = True
        except (ProcessLookupError, ValueError, KeyError):
            rec["alive"] = False
        except PermissionError:
            rec["alive"] = True
        out.append(rec)
    return sorted(out, key=lambda r: (r.get("device", 0), r.get("pid", 0)))


def prometheus_lines() -> str:
    """GPU gauges in Prometheus text format (node GPUs + live GPU object stores)."""
    lines = []

    def g(name, help_, series):
        lines.append(f"# HELP {name} {help_}\n# TYPE {name} gauge\n")
        for labels, v in series:
            if v is None:
                continue
            lab = "{" + ",".join(f'{k}="{x}"' for k, x in labels.items()) + "}" if labels else ""
            lines.append(f"{name}{lab} {float(v)}\n")

    gpus = gpu_devices()
    lab = [{"gpu": str(d["index"]), "pci_bus_id": str(d.get("pci_bus_id"))} for d in gpus]
    g("rmm_gpu_utilization_percent", "GPU busy percent (amdgpu gpu_busy_percent)",
      [(lb, d.get("busy_percent")) for lb, d in zip(lab, gpus)])
    g("rmm_gpu_vram_used_bytes", "HBM in use", [(lb, d.get("vram_used_bytes")) for lb, d in zip(lab, gpus)])
    g("rmm_gpu_vram_total_bytes", "HBM capacity", [(lb, d.get("vram_total_bytes")) for lb, d in zip(lab, gpus)])
    g("rmm_gpu_power_watts", "Average board power", [(lb, d.get("power_w")) for lb, d in zip(lab, gpus)])
    stores = [s for s in gpu_object_stores() if s.get("alive")]
    for key, help_ in (("capacity", "GPU object store capacity (bytes)"),
                       ("bytes_in_use", "GPU object store bytes in use"),
                       ("num_objects", "GPU object store objects"),
                       ("spilled_bytes_total", "GPU object store bytes spilled to host"),
                       ("restored_bytes_total", "GPU object store bytes restored from host"),
                       ("spilled_objects", "GPU objects currently spilled")):
        g(f"rmm_gpu_object_store_{key}", help_,
          [({"pid": str(s["pid"]), "device": str(s["device"]), "pci_bus_id": str(s.get("pci_bus_id"))},
            s["stats"].get(key)) for s in stores])
    return "".join(lines)
