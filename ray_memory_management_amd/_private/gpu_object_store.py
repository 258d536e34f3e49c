"""Python side of the HBM GPU object store (``csrc/hip/gpu_store.hip``).

``put(cuda_tensor)`` copies the tensor into this process's HBM arena with the multi-segment copy
kernel (one launch) and publishes a small *descriptor* object in the node's shared-memory store:
(nbytes, slab, offset, device, owner pid, slab hipIPC handle, PCI bus id, dtype/shape). A ``get``
  * in the owner process returns a zero-copy view (DLPack) pinned until the tensor dies;
  * in another process on the node opens the slab once via hipIpcOpenMemHandle (dmabuf) and
    returns a zero-copy view pinned through the descriptor (the owner never spills or moves an
    object whose descriptor is pinned — the flag protocol in shm_store.h);
  * of an object the owner spilled (LRU, under HBM pressure) restores it from the host store
    (decompressing with the K4 kernel) into local memory.
Parity: no reference equivalent (reference serializes CUDA tensors through host memory).
"""
from __future__ import annotations

import os
import pickle
import struct
import threading
from typing import Dict, Optional

from ray_memory_management_amd._native import require_hip, store_ext
from ray_memory_management_amd._private import serialization as ser

_DESC = struct.Struct("<QQqQii64s16sQ")
_lock = threading.Lock()
_ipc_cache: Dict[tuple, int] = {}

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
        s = h.GpuStore(device, cap, slab, worker.store_name, bool(cfg.get("gpu_spill_compression", True)))
        stores[device] = s
    return s


def put_tensor(worker, oid: bytes, t) -> None:
    import torch

    h = require_hip()
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    g = process_store(worker, dev)
    t = t.detach()
    if not t.is_contiguous():
        t = t.contiguous()
    nbytes = t.numel() * t.element_size()
    stream = torch.cuda.current_stream(dev).cuda_stream
    g.put_segments(oid, [(t.data_ptr(), nbytes)] if nbytes else [], _elem_bits(t.dtype), stream)
    slab, off, n = g.locate(oid)
    handle = g.slab_ipc_handle(slab) if slab >= 0 else b""
    try:
        pci = torch.cuda.get_device_properties(dev).pci_bus_id if hasattr(torch.cuda.get_device_properties(dev), "pci_bus_id") else ""
    except Exception:
        pci = ""
    meta = pickle.dumps({"dtype": t.dtype, "shape": tuple(t.shape), "requires_grad": t.requires_grad}, protocol=5)
    hdr = _DESC.pack(store_ext().GPU_DESC_MAGIC, nbytes, slab, off, dev, os.getpid(),
                     handle.ljust(64, b"\0")[:64], str(pci).encode()[:16].ljust(16, b"\0"), len(meta))
    buf = worker.store.create(oid, len(hdr) + len(meta), 0, ser.TAG_GPU, False)
    if buf is None:
        return
    mv = memoryview(buf)
    mv[:len(hdr)] = hdr
    mv[len(hdr):len(hdr) + len(meta)] = meta
    del mv
    worker.store.seal(oid)
    buf.release()


def _local_view(worker, g, oid, meta, dev):
    import torch

    h = require_hip()
    code, bits = _dl(meta["dtype"])
    stream = torch.cuda.current_stream(dev).cuda_stream
    cap = h.store_dlpack(g, oid, list(meta["shape"]), code, bits, stream)
    return torch.from_dlpack(cap)


def get_tensor(worker, oid: bytes, _ignored=None):
    """Materialise a GPU object as a torch tensor (see module docstring)."""
    import torch

    h = require_hip()
    flag_spilled = store_ext().FLAG_GPU_SPILLED
    while True:
        r = worker.store.get_raw(oid, -1)
        pin, dsize, msize, tag, is_err, flags = r
        mv = memoryview(pin)
        magic, nbytes, slab, off, dev, owner, ipc, pci, mlen = _DESC.unpack_from(mv, 0)
        meta = pickle.loads(mv[_DESC.size:_DESC.size + mlen])
        del mv
        stores = getattr(worker, "_gpu_stores", {}) or {}
        if owner == os.getpid() and dev in stores and stores[dev].contains(oid):
            pin.release()
            t = _local_view(worker, stores[dev], oid, meta, dev)
            break
        if flags & flag_spilled:
            t = _restore_from_host(worker, oid, meta, nbytes, dev)
            pin.release()
            if t is None:
                continue  # owner restored concurrently: retry through the descriptor
            break
        # zero-copy through the owner's slab; the descriptor pin is released with the tensor
        local_dev = dev if dev < torch.cuda.device_count() else 0
        key = (owner, bytes(ipc))
        with _lock:
            base = _ipc_cache.get(key)
            if base is None:
                base = h.ipc_open(bytes(ipc), local_dev)
                _ipc_cache[key] = base
        code, bits = _dl(meta["dtype"])
        cap = h.dlpack(base + off, list(meta["shape"]), code, bits, local_dev, pin.release)
        t = torch.from_dlpack(cap)
        break
    if meta.get("requires_grad"):
        t = t.detach().requires_grad_(True)
    return t


def _restore_from_host(worker, oid, meta, nbytes, dev):
    """Read a spilled GPU object's host copy (written by the owner's GpuStore) into local HBM."""
    import torch

    h = require_hip()
    hid = h.GpuStore.host_id(oid)
    r = worker.store.get_raw(hid, 0)
    if r is None:
        return None
    pin = r[0]
    mv = memoryview(pin)
    magic, total, bits, nchunks = struct.unpack_from("<QQQQ", mv, 0)
    csizes = struct.unpack_from(f"<{nchunks}Q", mv, 32)
    hdr = ((4 + nchunks) * 8 + 63) & ~63
    local_dev = dev if dev < torch.cuda.device_count() else 0
    out = torch.empty(meta["shape"], dtype=meta["dtype"], device=f"cuda:{local_dev}")
    flat = out.view(-1).view(torch.uint8) if nbytes else out
    chunk = 64 << 20
    soff = hdr
    stream = torch.cuda.current_stream(local_dev).cuda_stream
    import numpy as np

    host = np.frombuffer(mv, dtype=np.uint8)
    for c in range(nchunks):
        ln = min(chunk, total - c * chunk)
        cs = csizes[c]
        if cs:
            src = torch.from_numpy(host[soff:soff + cs]).to(f"cuda:{local_dev}")
            ws = torch.empty(h.compress_workspace(ln * 8 // bits), dtype=torch.uint8, device=f"cuda:{local_dev}")
            h.decompress(src.data_ptr(), flat.data_ptr() + c * chunk, ln * 8 // bits, bits, ws.data_ptr(), stream)
            soff += cs
        else:
            flat[c * chunk:c * chunk + ln].copy_(torch.from_numpy(host[soff:soff + ln]))
            soff += ln
    torch.cuda.current_stream(local_dev).synchronize()
    del host, mv
    pin.release()
    return out


def free(worker, oid: bytes):
    stores = getattr(worker, "_gpu_stores", None)
    if not stores:
        return
    for g in list(stores.values()):  # called from the reader thread while the owner may add stores
        if g.contains(oid):
            g.delete(oid)


def stats(worker) -> dict:
    stores = getattr(worker, "_gpu_stores", None) or {}
    return {dev: g.stats() for dev, g in list(stores.items())}


def shutdown_process_store(worker):
    stores = getattr(worker, "_gpu_stores", None)
    if stores:
        stores.clear()
    with _lock:
        _ipc_cache.clear()
