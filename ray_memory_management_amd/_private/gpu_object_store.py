"""Python side of the HBM GPU object store (``csrc/hip/gpu_store.hip``).

``put(cuda_tensor)`` copies the tensor into this process's HBM arena with the multi-segment copy
kernel (one launch, on the caller's stream) and publishes a small *descriptor* object in the node's
shared-memory store: (nbytes, slab, offset, device, owner pid, slab hipIPC handle, PCI address,
dtype/shape). The put does NOT block the host: the descriptor is sealed by a HIP host callback
once the copy has completed, so readers in other processes see it only when the data is there.

A ``get``
  * in the owner process returns a zero-copy view (DLPack) pinned until the tensor dies (the
    owner's GpuStore defers a Delete of a pinned object to its last Release);
  * in another process whose GPU is the SAME physical device (matched by PCI address, not by the
    local index — every worker runs with its own HIP_VISIBLE_DEVICES) opens the slab once via
    hipIpcOpenMemHandle (dmabuf) and returns a zero-copy view pinned through the descriptor; the
    owner never spills, moves or frees an object whose descriptor is pinned;
  * on a DIFFERENT GPU pulls the object over xGMI: the peer slab is imported and DMA'd
    (hipMemcpyAsync device→device) into the consumer's own arena, under an HBM pull quota
    (reference: object_manager.cc Pull + pull_manager.cc UpdatePullsBasedOnAvailableMemory);
  * of an object the owner spilled restores it from the host store into local memory with the
    native pinned, side-stream, K4-decompressing restore (GpuStore.restore_foreign).

IPC mappings are reference-counted per (owner, slab handle) and closed when idle (an imported
dmabuf keeps the owner's allocation alive). CUDA tensors nested inside other values are routed
here by the serializer (each becomes its own GPU object, contained in the outer one).
Parity: no reference equivalent (the reference serializes CUDA tensors through host memory).
"""
from __future__ import annotations

import collections
import math
import os
import pickle
import struct
import threading
from typing import Dict, Optional

from ray_memory_management_amd._native import require_hip, store_ext
from ray_memory_management_amd._private import serialization as ser

_DESC = struct.Struct("<QQqQii64s16sQ")
_lock = threading.RLock()  # re-entrant: a tensor deleter may run (GC) while it is held
_IDLE_MAPPINGS = 8

_DLPACK_CODE = {}  # torch dtype -> (code, bits)


def _dl(dtype):
    import torch

    if not _DLPACK_CODE:
        _DLPACK_CODE.update({
            torch.float32: (2, 32), torch.float16: (2, 16), torch.bfloat16: (4, 16), torch.float64: (2, 64),
            torch.int8: (0, 8), torch.int16: (0, 16), torch.int32: (0, 32), torch.int64: (0, 64),
            torch.uint8: (1, 8), torch.bool: (6, 8),
        })
    return _DLPACK_CODE[dtype]


def _elem_bits(dtype) -> int:
    import torch

    if dtype in (torch.bfloat16, torch.float16):
        return 16
    if dtype == torch.float32:
        return 32
    return 0


# ---------------------------------------------------------------------------- device identity
_pci_cache: Dict[int, str] = {}


def pci_bus_id(device: int) -> str:
    """Canonical PCI address of a locally visible device ("0000:5d:00.0")."""
    s = _pci_cache.get(device)
    if s is None:
        s = _pci_cache[device] = require_hip().pci_bus_id(device)
    return s


def local_device_for_pci(pci: str) -> int:
    """Local device index of the physical GPU `pci`, or -1 if it is not visible here."""
    if os.environ.get("RMM_TEST_FORCE_PEER_COPY"):
        return -1  # test hook: treat every remote object as living on another GPU
    import torch

    for i in range(torch.cuda.device_count()):
        if pci_bus_id(i) == pci:
            return i
    return -1


def _consumer_device() -> int:
    import torch

    return torch.cuda.current_device()


# ---------------------------------------------------------------------------- per-process store
def process_store(worker, device: int):
    """The per-process GpuStore for `device` (created lazily)."""
    stores = getattr(worker, "_gpu_stores", None)
    if stores is None:
        stores = worker._gpu_stores = {}
    s = stores.get(device)
    if s is None:
        h = require_hip()
        import torch

        total = torch.cuda.get_device_properties(device).total_memory
        cfg = worker.config or {}
        cap = int(cfg.get("gpu_object_store_memory", int(total * float(cfg.get("gpu_object_store_fraction", 0.3)))))
        slab = int(cfg.get("gpu_object_store_slab_bytes", min(cap, 8 << 30)))
        # gpu_spill_prepin_bytes: page-lock that much of the host arena (the spill target) in the
        # background, so spills are straight DMAs instead of pin-on-first-use
        s = h.GpuStore(device, cap, slab, worker.store_name, bool(cfg.get("gpu_spill_compression", True)),
                       float(cfg.get("gpu_object_spilling_threshold", 0.0)),
                       int(cfg.get("gpu_spill_prepin_bytes", 0)))
        stores[device] = s
        try:  # occupancy / spill counters for the dashboard's GPU reporter (internal KV)
            from ray_memory_management_amd.dashboard.gpu_reporter import publish_store_stats

            publish_store_stats(worker)
        except Exception:  # noqa: BLE001 - reporting is best effort
            pass
    return s


def _meta_cache(worker) -> dict:
    m = getattr(worker, "_gpu_meta", None)
    if m is None:
        m = worker._gpu_meta = {}
    return m


def put_tensor(worker, oid: bytes, t) -> None:
    """Copy `t` into this process's GPU store and publish its descriptor (non-blocking)."""
    import torch

    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    g = process_store(worker, dev)
    t = t.detach()
    if not t.is_contiguous():
        t = t.contiguous()
    nbytes = t.numel() * t.element_size()
    stream = torch.cuda.current_stream(dev).cuda_stream
    g.put_segments(oid, [(t.data_ptr(), nbytes)] if nbytes else [], _elem_bits(t.dtype), stream)
    _publish_descriptor(worker, g, oid, dev, {"dtype": t.dtype, "shape": tuple(t.shape),
                                              "requires_grad": t.requires_grad}, nbytes, stream, sealed=False)


class GpuObjectHandle:
    """A GPU object this process created in place (create_object) and published (publish_created): as a
    task output or inside one it serializes as a reference to that object, with no copy."""

    __slots__ = ("oid", "shape", "dtype")

    def __init__(self, oid: bytes, shape, dtype):
        self.oid, self.shape, self.dtype = oid, tuple(shape), dtype


def create_object(worker, oid: bytes, shape, dtype, device: int) -> int:
    """Allocate an unsealed GPU object of `shape` / `dtype` and return its device address: a producer
    (a kernel writing its output buffer) writes it in place, then publish_created seals and publishes it."""
    import torch

    nbytes = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
    return int(process_store(worker, device).create(oid, nbytes, _elem_bits(dtype)))


def publish_created(worker, oid: bytes, shape, dtype, device: int, stream, synced: bool = False) -> GpuObjectHandle:
    """Seal an object from create_object once `stream`'s work so far is done (its ready event) and publish
    its descriptor; returns the handle to put in a task's output. The host descriptor is sealed by a host
    callback after that work, or at once when the caller has already synchronised `stream` (synced)."""
    import torch

    g = process_store(worker, device)
    g.seal(oid, stream)
    nbytes = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
    _publish_descriptor(worker, g, oid, device, {"dtype": dtype, "shape": tuple(shape), "requires_grad": False},
                        nbytes, stream, sealed=synced)
    from ray_memory_management_amd._private import protocol as P

    worker.send((P.GPU_OBJECT, oid))
    return GpuObjectHandle(oid, shape, dtype)


def _publish_descriptor(worker, g, oid: bytes, dev: int, meta_d: dict, nbytes: int, stream, sealed: bool) -> None:
    """Write the host-store descriptor of GPU object `oid` (location, IPC handle, meta). sealed: the data is
    complete once `stream` drains (seal now if the caller has synchronised, else on a host callback)."""
    import torch

    slab, off, n = g.locate(oid)  # location is known at allocation time: no wait for the copy
    handle = g.slab_ipc_handle(slab) if slab >= 0 else b""
    meta = pickle.dumps(meta_d, protocol=5)
    hdr = _DESC.pack(store_ext().GPU_DESC_MAGIC, nbytes, slab, off, dev, os.getpid(),
                     handle.ljust(64, b"\0")[:64], pci_bus_id(dev).encode()[:16].ljust(16, b"\0"), len(meta))
    buf = worker.store.create(oid, len(hdr) + len(meta), 0, ser.TAG_GPU, False)
    if buf is None:
        return
    mv = memoryview(buf)
    mv[:len(hdr)] = hdr
    mv[len(hdr):len(hdr) + len(meta)] = meta
    del mv
    _meta_cache(worker)[oid] = meta_d
    if sealed:  # the producer's stream has drained (the caller synchronised): no callback needed
        worker.store.seal(oid)
        buf.release()
    elif (worker.config or {}).get("gpu_async_put", True):
        buf.disown()  # the host callback seals + releases once the copy on `stream` is done
        g.seal_descriptor_async(oid, stream)
    else:
        torch.cuda.current_stream(dev).synchronize()
        worker.store.seal(oid)
        buf.release()


def _local_view(worker, g, oid, meta, dev):
    import torch

    h = require_hip()
    code, bits = _dl(meta["dtype"])
    stream = torch.cuda.current_stream(dev).cuda_stream
    cap = h.store_dlpack(g, oid, list(meta["shape"]), code, bits, stream)
    return torch.from_dlpack(cap)


# ---------------------------------------------------------------------------- IPC mappings
class _Mapping:
    __slots__ = ("base", "refs", "device")

    def __init__(self, base, device):
        self.base, self.refs, self.device = base, 0, device


_maps: "collections.OrderedDict[tuple, _Mapping]" = collections.OrderedDict()


def _map_acquire(owner, ipc: bytes, device: int) -> _Mapping:
    key = (owner, bytes(ipc), device)
    with _lock:
        m = _maps.get(key)
        if m is None:
            m = _Mapping(require_hip().ipc_open(bytes(ipc), device), device)
            _maps[key] = m
        _maps.move_to_end(key)
        m.refs += 1
        return m


def _map_release(owner, ipc: bytes, device: int):
    key = (owner, bytes(ipc), device)
    with _lock:
        m = _maps.get(key)
        if m is not None:
            m.refs -= 1
        _close_idle_locked(_IDLE_MAPPINGS)


def _close_idle_locked(keep: int):
    idle = [k for k, m in _maps.items() if m.refs <= 0]
    for k in idle[:max(0, len(idle) - keep)]:
        m = _maps.pop(k)
        try:
            require_hip().ipc_close(m.base)
        except Exception:
            pass


def close_idle_mappings(keep: int = 0) -> int:
    """Close imported slabs no live tensor uses (lets the owners' hipFree actually return HBM)."""
    with _lock:
        n = len(_maps)
        _close_idle_locked(keep)
        return n - len(_maps)


def mapping_stats() -> dict:
    with _lock:
        return {"mappings": len(_maps), "idle": sum(1 for m in _maps.values() if m.refs <= 0)}


# ---------------------------------------------------------------------------- pull quota
class _PullQuota:
    """Admission control for cross-GPU pulls: bytes of pulled replicas alive at once stay under
    `limit` (one oversized object is admitted when nothing else is in flight)."""

    def __init__(self):
        self.cv = threading.Condition()
        self.in_use = 0
        self.limit = None
        self.pulls = 0
        self.bytes_pulled = 0
        self.waits = 0

    def acquire(self, n: int, limit: int):
        with self.cv:
            self.limit = limit
            while self.in_use > 0 and self.in_use + n > limit:
                self.waits += 1
                self.cv.wait(1.0)
            self.in_use += n
            self.pulls += 1
            self.bytes_pulled += n

    def release(self, n: int):
        with self.cv:
            self.in_use -= n
            self.cv.notify_all()


_quota = _PullQuota()


def pull_stats() -> dict:
    return {"pulls": _quota.pulls, "bytes_pulled": _quota.bytes_pulled, "in_use": _quota.in_use,
            "quota_waits": _quota.waits, "limit": _quota.limit}


def _pull_limit(worker, device) -> int:
    cfg = worker.config or {}
    if "gpu_pull_quota_bytes" in cfg:
        return int(cfg["gpu_pull_quota_bytes"])
    import torch

    return int(torch.cuda.get_device_properties(device).total_memory * float(cfg.get("gpu_pull_quota_fraction", 0.25)))


def _pull_from_peer(worker, meta, nbytes, owner, ipc: bytes, off: int, pin):
    """Copy a peer GPU's object into this process's memory (DMA over xGMI), under the quota."""
    import torch

    dev = _consumer_device()
    limit = _pull_limit(worker, dev)
    _quota.acquire(nbytes, limit)
    try:
        out = torch.empty(meta["shape"], dtype=meta["dtype"], device=f"cuda:{dev}")
        if nbytes:
            m = _map_acquire(owner, ipc, dev)
            try:
                stream = torch.cuda.current_stream(dev).cuda_stream
                require_hip().memcpy_async(out.data_ptr(), m.base + off, nbytes, stream)
                torch.cuda.current_stream(dev).synchronize()
            finally:
                _map_release(owner, ipc, dev)
    except BaseException:
        _quota.release(nbytes)
        raise
    finally:
        pin.release()
    # the replica counts against the quota until it is garbage collected
    import weakref

    weakref.finalize(out, _quota.release, nbytes)
    return out


# ---------------------------------------------------------------------------- get
def get_tensor(worker, oid: bytes, _ignored=None):
    """Materialise a GPU object as a torch tensor (see module docstring)."""
    h = require_hip()
    flag_spilled = store_ext().FLAG_GPU_SPILLED
    stores = getattr(worker, "_gpu_stores", {}) or {}
    meta = _meta_cache(worker).get(oid)
    if meta is not None:  # owner fast path: no descriptor round trip, stream-ordered on the copy
        for dev, g in list(stores.items()):
            if g.contains(oid):
                t = _local_view(worker, g, oid, meta, dev)
                return t.detach().requires_grad_(True) if meta.get("requires_grad") else t
    while True:
        r = worker.store.get_raw(oid, -1)
        pin, dsize, msize, tag, is_err, flags = r
        mv = memoryview(pin)
        magic, nbytes, slab, off, dev, owner, ipc, pci, mlen = _DESC.unpack_from(mv, 0)
        meta = pickle.loads(mv[_DESC.size:_DESC.size + mlen])
        del mv
        pci = pci.rstrip(b"\0").decode()
        if owner == os.getpid() and dev in stores and stores[dev].contains(oid):
            pin.release()
            t = _local_view(worker, stores[dev], oid, meta, dev)
            break
        if flags & flag_spilled:
            t = _restore_from_host(worker, oid, meta, nbytes)
            pin.release()
            if t is None:
                continue  # owner restored concurrently: retry through the descriptor
            break
        local = local_device_for_pci(pci)
        if local >= 0:
            # same physical GPU: zero-copy through the owner's slab; pin released with the tensor
            m = _map_acquire(owner, ipc, local)
            code, bits = _dl(meta["dtype"])

            def _done(pin=pin, owner=owner, ipc=bytes(ipc), local=local):
                pin.release()
                _map_release(owner, ipc, local)

            cap = h.dlpack(m.base + off, list(meta["shape"]), code, bits, local, _done)
            if os.environ.get("RMM_SHARED_WEIGHTS_DEBUG"):
                import sys

                print(f"[gpu-store] pid {os.getpid()} get {oid.hex()[:16]}: owner {owner} slab {slab} off {off:#x} "
                      f"nbytes {nbytes} mapping base {m.base:#x} device {local}", file=sys.stderr, flush=True)
            import torch

            t = torch.from_dlpack(cap)
            break
        # another GPU: import the peer slab, DMA into our own memory (the import stays cached idle)
        t = _pull_from_peer(worker, meta, nbytes, owner, bytes(ipc), off, pin)
        break
    if meta.get("requires_grad"):
        t = t.detach().requires_grad_(True)
    return t


def _restore_from_host(worker, oid, meta, nbytes):
    """Read a spilled GPU object's host copy (written by the owner's GpuStore) into local HBM with
    the native pinned, side-stream, K4-decompressing restore."""
    import torch

    h = require_hip()
    dev = _consumer_device()
    g = process_store(worker, dev)
    out = torch.empty(meta["shape"], dtype=meta["dtype"], device=f"cuda:{dev}")
    torch.cuda.current_stream(dev).synchronize()  # `out` is allocated before the side-stream DMA
    n = g.restore_foreign(h.GpuStore.host_id(oid), out.data_ptr(), nbytes) if nbytes else 0
    if nbytes and n != nbytes:
        return None
    return out


# ---------------------------------------------------------------------------- free
def free(worker, oid: bytes):
    """FREE_GPU from the head (the object's refcount reached 0). The HBM is recycled only once no
    reader in another process pins the descriptor (it stays in the shm store, delete-pending,
    until the last reader's tensor dies); until then the free is retried by the flusher."""
    stores = getattr(worker, "_gpu_stores", None)
    if not stores:
        return
    for g in list(stores.values()):  # called from the reader thread while the owner may add stores
        if g.contains(oid):
            if worker.store.state(oid) != -1:
                with _lock:
                    _deferred(worker).add(oid)
                return
            g.delete(oid)  # native: deferred while an owner-local view pins it
            _meta_cache(worker).pop(oid, None)


def free_unescaped(worker, oid: bytes) -> bool:
    """Owner-side immediate free of a GPU object whose ref never left this process (no other
    process can have mapped it). Only once its descriptor is sealed, i.e. the put's copy has
    finished; otherwise the head's FREE_GPU path frees it later. Owner-local views still pin the
    HBM natively (GpuStore::Delete defers while pinned)."""
    for g in list((getattr(worker, "_gpu_stores", None) or {}).values()):
        if g.contains(oid):
            if worker.store.state(oid) != 2:  # kSealed
                return False
            worker.store.delete([oid])
            g.delete(oid)
            _meta_cache(worker).pop(oid, None)
            return True
    return False


def _deferred(worker) -> set:
    d = getattr(worker, "_gpu_deferred_free", None)
    if d is None:
        d = worker._gpu_deferred_free = set()
    return d


def retry_deferred(worker) -> int:
    """Free deferred objects whose descriptors are gone; returns how many remain deferred."""
    with _lock:
        pending = list(_deferred(worker))
    done = []
    for oid in pending:
        if worker.store.state(oid) == -1:
            for g in list((getattr(worker, "_gpu_stores", None) or {}).values()):
                if g.contains(oid):
                    g.delete(oid)
            _meta_cache(worker).pop(oid, None)
            done.append(oid)
    with _lock:
        d = _deferred(worker)
        for oid in done:
            d.discard(oid)
        return len(d)


def stats(worker) -> dict:
    stores = getattr(worker, "_gpu_stores", None) or {}
    out = {dev: g.stats() for dev, g in list(stores.items())}
    return out


def shutdown_process_store(worker):
    stores = getattr(worker, "_gpu_stores", None)
    with _lock:
        for k in list(_maps):
            try:
                require_hip().ipc_close(_maps[k].base)
            except Exception:
                pass
        _maps.clear()
    if stores:
        stores.clear()
    if getattr(worker, "_gpu_meta", None):
        worker._gpu_meta.clear()
    unpin_store_segment(worker)


def unpin_store_segment(worker):
    """Drop every host-registration chunk of this worker's shm segment (ingest / spill DMA) before
    the segment is unmapped at shutdown."""
    import sys

    if "ray_memory_management_amd._hip" not in sys.modules or getattr(worker, "store", None) is None:
        return
    try:
        require_hip().host_unregister_segment(worker.store.base_address())
    except Exception:
        pass
