"""Microbenchmark of K12 (fused dense-tail backward, csrc/hip/dense_kernels.hip) and K13 (dense
forward) at the PPO minibatch shape: M = 500 rows, K = 3872 (Nature-CNN flatten), hidden 256,
A+1 = 5 heads. Prints µs per call as one JSON line.
Usage: python benchmarks/bench_dense.py [--M 500]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ray_memory_management_amd._native import require_hip  # noqa: E402


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=500)
    ap.add_argument("--K", type=int, default=3872)
    ap.add_argument("--A1", type=int, default=5)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    h = require_hip()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    bf = torch.bfloat16
    M, K, A1 = a.M, a.K, a.A1
    x = torch.randn(M, K, device=dev).to(bf)
    w = (torch.randn(256, K, device=dev) * 0.02).to(bf)
    b = torch.zeros(256, device=dev).to(bf)
    wh = (torch.randn(A1, 256, device=dev) * 0.05).to(bf)
    y = torch.relu(torch.randn(M, 256, device=dev)).to(bf)
    dz = torch.randn(M, A1, device=dev).to(bf)
    dx, dw = torch.empty_like(x), torch.empty_like(w)
    db, dwh, dbh = torch.empty(256, device=dev, dtype=bf), torch.empty_like(wh), torch.empty(A1, device=dev, dtype=bf)
    scratch = torch.empty(M, 256, device=dev, dtype=bf)
    hid = torch.empty(M, 256, device=dev, dtype=bf)
    out = {
        "k12_us": round(timeit(lambda: h.dense_heads_bwd(dz.data_ptr(), A1, wh.data_ptr(), y.data_ptr(), x.data_ptr(),
                                                         w.data_ptr(), M, K, dx.data_ptr(), dw.data_ptr(),
                                                         db.data_ptr(), dwh.data_ptr(), dbh.data_ptr(),
                                                         scratch.data_ptr(), st), a.iters), 2),
        "k13_us": round(timeit(lambda: h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, 256,
                                                        hid.data_ptr(), st), a.iters), 2),
        "M": M, "K": K, "A1": A1, "k12_version": 2,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
