"""K13 timing for the PPO dense layer (x[M,3872] · W[256,3872]ᵀ + b, ReLU), per M: mean µs per
launch over HIP-graph replays of 50 back-to-back launches.

Round 2 tried a split-K variant (MT x 64 tiles, K slices, fp32 partials): with the last slice
summing in-kernel it was 4x slower (agent-scope release/acquire = L2 write-back/invalidate across
XCDs), with a separate reduce launch 1.1-1.7x slower than K13 at M = 12..500 — K13's remaining cost
is the uncoalesced 16-row fragment loads, which an LDS-staged tile would fix."""
import os
import sys

import torch

sys.path.insert(0, ".")
from ray_memory_management_amd._native import require_hip  # noqa: E402


def main():
    h = require_hip()
    K, N = 3872, 256
    tag = "K13"
    for M in (12, 25, 50, 500):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, y.data_ptr(), st)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        reps = 50
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, y.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"{tag} M={M}: {e0.elapsed_time(e1) / (10 * reps) * 1e3:.2f} us", flush=True)


if __name__ == "__main__":
    main()
