"""What bounds a GPU-store spill (csrc/hip/gpu_store.hip SpillTransfer): timings of

* the spill of a 1 GiB bf16 tensor (randn: compress ratio ~0.76; smooth: ~0.51; int noise: incompressible),
* the raw line rate: one hipMemcpy D2H of the same bytes into the registered host arena (the store's
  shared-memory segment, hipHostRegister'ed as the spill path uses it),
* the compress kernel alone on one 64 MB chunk.

Run under `rocprofv3 --kernel-trace --memory-copy-trace --stats` for the per-chunk timeline.
usage: python benchmarks/spill_probe.py [--gb 1] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import ray_memory_management_amd as ray
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    n = int(a.gb * (1 << 30)) // 2
    ray.init(num_cpus=2, num_gpus=1, object_store_memory=int(max(4.0, 3 * a.gb) * (1 << 30)),
             _system_config={"memory_monitor_interval_ms": 0})
    out = {"gb": a.gb}
    try:
        from ray_memory_management_amd._private.worker import global_worker

        g = h.GpuStore(0, int(3 * a.gb * (1 << 30)), 8 << 30, global_worker.store_name, True)
        s = torch.cuda.current_stream().cuda_stream
        data = {
            "randn": torch.randn(n, device="cuda", dtype=torch.bfloat16),
            "smooth": torch.linspace(-1, 1, n, device="cuda").to(torch.bfloat16),
            "noise": torch.randint(-32768, 32767, (n,), device="cuda", dtype=torch.int16).view(torch.bfloat16),
        }
        # warm the host pages once
        wid = os.urandom(20)
        g.put_segments(wid, [(data["randn"].data_ptr(), n * 2)], 16, s)
        torch.cuda.synchronize()
        g.spill_object(wid)
        g.delete(wid)
        for mode, name, x in [(m, nm, t) for m in ("0", "1") for nm, t in data.items()]:
            # RMM_SPILL_DEVICE_PLACE=1: chunks written by a copy kernel at a device-resident offset
            os.environ["RMM_SPILL_DEVICE_PLACE"] = mode
            name = name + ("_devplace" if mode == "1" else "")
            placed0 = g.stats().get("spills_device_placed", 0)
            ts = []
            ratio = None
            for _ in range(a.reps):
                oid = os.urandom(20)
                g.put_segments(oid, [(x.data_ptr(), n * 2)], 16, s)
                torch.cuda.synchronize()
                st0 = g.stats()
                t0 = time.perf_counter()
                assert g.spill_object(oid) > 0, g.last_error()
                ts.append(time.perf_counter() - t0)
                st1 = g.stats()
                ratio = (st1["spilled_host_bytes_total"] - st0["spilled_host_bytes_total"]) / (n * 2)
                out_t = torch.empty_like(x)
                got = g.restore_foreign(h.GpuStore.host_id(oid), out_t.data_ptr(), n * 2)
                assert got == n * 2 and torch.equal(out_t.view(torch.int16), x.view(torch.int16))
                g.delete(oid)
            out[f"spill_GBps_{name}"] = round(n * 2 / min(ts) / 1e9, 2)
            out[f"spill_ms_{name}"] = [round(t * 1e3, 2) for t in ts]
            out[f"ratio_{name}"] = round(ratio, 3)
            out[f"device_placed_{name}"] = g.stats().get("spills_device_placed", 0) - placed0
        # raw line rate into pinned host memory (same size)
        host = torch.empty(n * 2, dtype=torch.uint8).pin_memory()
        src = data["noise"].view(torch.uint8)
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            host.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
        out["d2h_pinned_GBps"] = round(n * 2 / t / 1e9, 2)
        # the same bytes written by a copy KERNEL through the pinned buffer's device mapping (CU stores over
        # PCIe instead of the DMA engine): the transfer a device-placed spill would use
        dptr = h.host_device_pointer(host.data_ptr())
        out["host_device_pointer_is_host_va"] = dptr == host.data_ptr()
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h.multi_copy([(src.data_ptr(), dptr, n * 2)], s)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
        out["d2h_kernel_write_GBps"] = round(n * 2 / t / 1e9, 2)
        assert torch.equal(host[: 1 << 20], src[: 1 << 20].cpu())
        # 64 MB chunks (the spill chunk), kernel-written
        ck = 64 << 20
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for off in range(0, n * 2 - ck + 1, ck):
            h.multi_copy([(src.data_ptr() + off, dptr + off, ck)], s)
        torch.cuda.synchronize()
        out["d2h_kernel_write_64MB_chunks_GBps"] = round((n * 2 // ck) * ck / (time.perf_counter() - t0) / 1e9, 2)
        del g
    finally:
        ray.shutdown()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
