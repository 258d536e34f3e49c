"""HBM -> HBM copy throughput of K1 multi_copy (the GPU object store's put path) vs hipMemcpyAsync and
torch's copy_, for one large segment. Prints copy GB/s (bytes copied / s; HBM traffic is 2x).
RMM_COPY_VARIANT selects the K1 inner loop (csrc/hip/kernels.hip: copy_range). Usage:
python benchmarks/bench_copy.py [GiB]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ray_memory_management_amd._native import require_hip  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(gib * (1 << 30))
    h = require_hip()
    src = torch.empty(n, dtype=torch.uint8, device="cuda").random_(0, 255)
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream().cuda_stream
    out = {"GiB": gib, "variant": int(os.environ.get("RMM_COPY_VARIANT", "2"))}
    t = timeit(lambda: h.multi_copy([(src.data_ptr(), dst.data_ptr(), n)], st))
    out["k1_GBps"] = round(n / t / 1e9, 1)
    assert torch.equal(src[: 1 << 20], dst[: 1 << 20]) and torch.equal(src[-(1 << 20):], dst[-(1 << 20):])
    t = timeit(lambda: h.memcpy_async(dst.data_ptr(), src.data_ptr(), n, st))
    out["hipMemcpyAsync_GBps"] = round(n / t / 1e9, 1)
    t = timeit(lambda: dst.copy_(src))
    out["torch_copy_GBps"] = round(n / t / 1e9, 1)
    # the HBM's one-directional rates for reference: a copy moves 2n bytes (n read + n written)
    t = timeit(lambda: dst.view(torch.int64).fill_(7))
    out["write_only_GBps"] = round(n / t / 1e9, 1)
    t = timeit(lambda: src.view(torch.int64).sum())
    out["read_only_GBps"] = round(n / t / 1e9, 1)
    out["k1_traffic_TBps"] = round(2 * out["k1_GBps"] / 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
