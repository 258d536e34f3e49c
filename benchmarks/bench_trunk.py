"""Microbenchmark of the K10 fused Nature-CNN trunk kernels (csrc/hip/conv_kernels.hip) with the
profiling phase masks: prints µs per launch (graph-replayed: GPU time, not host launch rate) for fwd
(B=500 SGD minibatch, B=50 rollout step) and bwd (B=500), each phase skipped in turn to attribute time.
fwd dbg bits: 1 conv1 MFMA, 2 conv2 MFMA, 8 weight staging, 16 h1 store, 32 frame loads, 64 h2 store,
128 return at once (launch + dispatch floor). bwd bits: 1 dW2, 2 dh1, 4 dW1, 8 P0 loads, 16 partial
stores, 32 st zeroing, 64 return at once, 128 skip the reduce launch, 256 all LDS zeroing, 512 W2 staging,
1024 the bias-gradient epilogue. Usage: python benchmarks/bench_trunk.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ray_memory_management_amd._native import require_hip  # noqa: E402


def timeit(fn, iters=200):
    """µs per call on the GPU: `iters` calls captured in one HIP graph and replayed (eager launches
    from Python cost more host time than these kernels take, which would time the host instead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters) * 1e3


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="'bwd' or 'fwd': time one kernel config (for PMC runs)")
    ap.add_argument("--B", type=int, default=500)
    ap.add_argument("--dbg", type=int, default=0)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    h = require_hip()
    dev = torch.device("cuda:0")
    obs = torch.randint(0, 256, (5000, 4, 84, 84), dtype=torch.uint8, device=dev)
    w1 = (torch.randn(16, 4, 8, 8, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w2 = (torch.randn(32, 16, 4, 4, device=dev) * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b1 = torch.zeros(16, dtype=torch.bfloat16, device=dev)
    b2 = torch.zeros(32, dtype=torch.bfloat16, device=dev)
    out = {}
    if a.only:
        B = a.B
        idx = torch.randperm(5000, device=dev)[:B].contiguous()
        h1 = torch.zeros(B, 441, 16, dtype=torch.bfloat16, device=dev)
        h2 = torch.zeros(B, 3872, dtype=torch.bfloat16, device=dev)
        if a.only == "fwd":
            t = timeit(lambda: h.nature_trunk_fwd(
                obs.data_ptr(), idx.data_ptr(), 0, 1, B, w1.data_ptr(), list(w1.stride()), b1.data_ptr(),
                w2.data_ptr(), list(w2.stride()), b2.data_ptr(), h1.data_ptr(), h2.data_ptr(), torch.cuda.current_stream().cuda_stream, dbg=a.dbg), a.iters)
        else:
            dh2 = torch.randn(B, 3872, device=dev).to(torch.bfloat16)
            part = torch.empty(h.nature_trunk_partial_floats(B), dtype=torch.float32, device=dev)
            dw1, dw2 = torch.empty_like(w1), torch.empty_like(w2)
            db1, db2 = torch.empty_like(b1), torch.empty_like(b2)
            t = timeit(lambda: h.nature_trunk_bwd(
                obs.data_ptr(), idx.data_ptr(), 0, 1, B, w2.data_ptr(), list(w2.stride()), h1.data_ptr(),
                h2.data_ptr(), dh2.data_ptr(), part.data_ptr(), dw1.data_ptr(), list(w1.stride()), db1.data_ptr(),
                dw2.data_ptr(), db2.data_ptr(), torch.cuda.current_stream().cuda_stream, dbg=a.dbg), a.iters)
        print(json.dumps({f"{a.only}_B{B}_dbg{a.dbg}": round(t, 1),
                          "cus": torch.cuda.get_device_properties(0).multi_processor_count}))
        return
    for B in (500, 50):
        idx = torch.randperm(5000, device=dev)[:B].contiguous()
        h1 = torch.empty(B, 441, 16, dtype=torch.bfloat16, device=dev)
        h2 = torch.empty(B, 3872, dtype=torch.bfloat16, device=dev)
        for dbg in (0, 1, 2, 3, 7, 8, 16, 32, 64, 120, 127, 128):
            out[f"fwd_B{B}_dbg{dbg}"] = round(timeit(lambda: h.nature_trunk_fwd(
                obs.data_ptr(), idx.data_ptr(), 0, 1, B, w1.data_ptr(), list(w1.stride()), b1.data_ptr(),
                w2.data_ptr(), list(w2.stride()), b2.data_ptr(), h1.data_ptr(), h2.data_ptr(), torch.cuda.current_stream().cuda_stream, dbg=dbg)), 1)
        if B == 500:
            dh2 = torch.randn(B, 3872, device=dev).to(torch.bfloat16)
            part = torch.empty(h.nature_trunk_partial_floats(B), dtype=torch.float32, device=dev)
            dw1, dw2 = torch.empty_like(w1), torch.empty_like(w2)
            db1, db2 = torch.empty_like(b1), torch.empty_like(b2)
            for dbg in (0, 1, 2, 4, 7, 8, 15, 16, 31, 63, 64, 128, 128 + 31, 128 + 64, 159 + 256, 159 + 512,
                        159 + 1024, 159 + 256 + 512 + 1024):
                out[f"bwd_B{B}_dbg{dbg}"] = round(timeit(lambda: h.nature_trunk_bwd(
                    obs.data_ptr(), idx.data_ptr(), 0, 1, B, w2.data_ptr(), list(w2.stride()), h1.data_ptr(),
                    h2.data_ptr(), dh2.data_ptr(), part.data_ptr(), dw1.data_ptr(), list(w1.stride()), db1.data_ptr(),
                    dw2.data_ptr(), db2.data_ptr(), torch.cuda.current_stream().cuda_stream, dbg=dbg)), 1)
    # latency vs throughput: backward at growing B (G = min(B, 256) workgroups)
    for B in (1, 16, 64, 256):
        idx = torch.randperm(5000, device=dev)[:B].contiguous()
        h1 = torch.zeros(B, 441, 16, dtype=torch.bfloat16, device=dev)
        h2 = torch.zeros(B, 3872, dtype=torch.bfloat16, device=dev)
        dh2 = torch.randn(B, 3872, device=dev).to(torch.bfloat16)
        part = torch.empty(h.nature_trunk_partial_floats(B), dtype=torch.float32, device=dev)
        dw1, dw2 = torch.empty_like(w1), torch.empty_like(w2)
        db1, db2 = torch.empty_like(b1), torch.empty_like(b2)
        for dbg in (0, 15, 31, 128 + 31, 159 + 256 + 512 + 1024):
            out[f"bwd_B{B}_dbg{dbg}"] = round(timeit(lambda: h.nature_trunk_bwd(
                obs.data_ptr(), idx.data_ptr(), 0, 1, B, w2.data_ptr(), list(w2.stride()), h1.data_ptr(),
                h2.data_ptr(), dh2.data_ptr(), part.data_ptr(), dw1.data_ptr(), list(w1.stride()), db1.data_ptr(),
                dw2.data_ptr(), db2.data_ptr(), torch.cuda.current_stream().cuda_stream, dbg=dbg)), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
