"""K10 rollout trunk in push mode (K19 folded in) at the hybrid worker's batch: how much of the launch is
the PCIe read of the envs' newest frames. Times nature_trunk_fwd_push with the new frames in (a)
device-mapped pinned host memory (zero-copy, the rollout default), (b) HBM, and (c) a 353 KB H2D DMA
copy on its own. Usage: python benchmarks/bench_push.py [B]"""
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
    return round(s.elapsed_time(e) / iters * 1e3, 2)


def main(B: int = 50):
    h = require_hip()
    dev = torch.device("cuda:0")
    stack = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=dev)
    new_host = torch.randint(0, 256, (B, 84, 84), dtype=torch.uint8).pin_memory()
    new_dev = new_host.to(dev)
    mapped = int(h.host_device_pointer(new_host.data_ptr()))
    w1 = (torch.randn(16, 4, 8, 8, device=dev) * 0.05).to(torch.bfloat16)
    b1 = torch.zeros(16, device=dev, dtype=torch.bfloat16)
    w2 = (torch.randn(32, 16, 4, 4, device=dev) * 0.05).to(torch.bfloat16)
    b2 = torch.zeros(32, device=dev, dtype=torch.bfloat16)
    h2 = torch.empty(B, 3872, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream

    def push(src):
        return lambda: h.nature_trunk_fwd_push(stack.data_ptr(), src, 0, 0, B, w1.data_ptr(), list(w1.stride()),
                                               b1.data_ptr(), w2.data_ptr(), list(w2.stride()), b2.data_ptr(),
                                               h2.data_ptr(), st)

    out = {"B": B, "push_mapped_host_us": timeit(push(mapped)), "push_hbm_us": timeit(push(new_dev.data_ptr())),
           "h2d_dma_us": timeit(lambda: new_dev.copy_(new_host, non_blocking=True))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
