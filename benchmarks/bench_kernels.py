"""Micro-benchmarks of the CDNA4 kernels and the GPU object store on one MI355X.

Prints one JSON line per measurement. Timed with HIP events, interleaved A/B in one process.
"""
import json
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_memory_management_amd import ops  # noqa: E402
from ray_memory_management_amd._native import require_hip, store_ext  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def out(**kw):
    print(json.dumps(kw), flush=True)


def main():
    h = require_hip()
    dev = torch.device("cuda:0")
    out(arch=h.arch(0), torch=torch.__version__)
    # --- copy bandwidth: multi_copy vs torch copy_ (1 GiB and 4 GiB)
    for gb in (1, 4):
        n = gb << 30
        a = torch.empty(n, dtype=torch.uint8, device=dev).fill_(1)
        b = torch.empty_like(a)
        t_mc = timeit(lambda: ops.multi_copy([(a, b)]))
        t_tc = timeit(lambda: b.copy_(a))
        out(kernel="multi_copy", bytes=n, ms=t_mc * 1e3, GBps_rw=2 * n / t_mc / 1e9, torch_copy_GBps_rw=2 * n / t_tc / 1e9)
        del a, b
    # --- many small segments (pack of 256 tensors of 1 MiB)
    srcs = [torch.empty(1 << 20, dtype=torch.uint8, device=dev) for _ in range(256)]
    dsts = [torch.empty_like(s) for s in srcs]
    pairs = list(zip(srcs, dsts))
    t_mc = timeit(lambda: ops.multi_copy(pairs))
    t_loop = timeit(lambda: [d.copy_(s) for s, d in pairs])
    out(kernel="multi_copy_256x1MiB", ms=t_mc * 1e3, loop_copy_ms=t_loop * 1e3, speedup=t_loop / t_mc)
    # --- gather rows (PPO minibatch of 84x84x4 uint8 frames)
    frames = torch.randint(0, 255, (65536, 4, 84, 84), dtype=torch.uint8, device=dev)
    idx = torch.randperm(65536, device=dev)[:16384]
    t_g = timeit(lambda: ops.gather_rows(frames, idx))
    t_t = timeit(lambda: frames[idx])
    nbytes = idx.numel() * frames[0].numel()
    out(kernel="gather_rows", rows=idx.numel(), ms=t_g * 1e3, GBps_rw=2 * nbytes / t_g / 1e9, torch_index_ms=t_t * 1e3)
    del frames
    # --- GAE
    for T, B in ((256, 1024), (2048, 4096)):
        r, v = torch.randn(T, B, device=dev), torch.randn(T, B, device=dev)
        d = (torch.rand(T, B, device=dev) < 0.01).float()
        lv = torch.randn(B, device=dev)
        t_k = timeit(lambda: ops.gae(r, v, d, lv))
        out(kernel="gae", T=T, B=B, ms=t_k * 1e3, GBps=(5 * T * B * 4) / t_k / 1e9)
    # --- compress/decompress bf16 (spill path)
    n = 256 << 20
    x = (torch.randn(n, device=dev) * 0.02).to(torch.bfloat16)
    c = ops.compress(x)
    t_c = timeit(lambda: ops.compress(x), iters=5)
    t_d = timeit(lambda: ops.decompress(c, n, torch.bfloat16), iters=5)
    out(kernel="compress_bf16", bytes=2 * n, ratio=c.numel() / (2 * n), compress_GBps=2 * n / t_c / 1e9,
        decompress_GBps=2 * n / t_d / 1e9)
    del x, c
    # --- GPU object store put/get
    name = "/rmm-bench-" + uuid.uuid4().hex[:8]
    host = store_ext().ObjectStore.create_segment(name, 8 << 30, "/tmp", 0.8, 1 << 30, True)
    g = h.GpuStore(0, 64 << 30, 16 << 30, name, True)
    s = torch.cuda.current_stream().cuda_stream
    for gb in (1, 4, 16):
        nel = (gb << 30) // 2
        t = torch.randn(nel, device=dev, dtype=torch.bfloat16)
        ids = []

        def put_get():
            oid = os.urandom(20)
            g.put_segments(oid, [(t.data_ptr(), nel * 2)], 16, s)
            v = torch.from_dlpack(h.store_dlpack(g, oid, [nel], 4, 16, s))
            ids.append(oid)
            return v

        put_get()
        torch.cuda.synchronize()
        for oid in ids:
            g.delete(oid)
        ids.clear()
        iters = 5
        dt = 0.0
        for _ in range(iters):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v = put_get()
            torch.cuda.synchronize()
            dt += (time.perf_counter() - t0) / iters
            del v
            g.delete(ids.pop())
        out(bench="gpu_put_get", GB=gb, ms=dt * 1e3, GBps=(gb << 30) / dt / 1e9)
        del t
    # spill/restore throughput
    nel = (2 << 30) // 2
    t = (torch.randn(nel, device=dev) * 0.02).to(torch.bfloat16)
    oid = os.urandom(20)
    g.put_segments(oid, [(t.data_ptr(), nel * 2)], 16, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.spill_object(oid)
    t1 = time.perf_counter()
    v = torch.from_dlpack(h.store_dlpack(g, oid, [nel], 4, 16, s))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ok = bool(torch.equal(v, t))
    st = g.stats()
    out(bench="gpu_spill_restore", GB=2, spill_GBps=(2 << 30) / (t1 - t0) / 1e9, restore_GBps=(2 << 30) / (t2 - t1) / 1e9,
        host_ratio=st["spilled_host_bytes_total"] / max(1, st["spilled_bytes_total"]), exact=ok)
    del v
    g.delete(oid)
    del g, host


if __name__ == "__main__":
    main()
