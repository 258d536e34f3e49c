"""K6 flat-Adam microbenchmark (one MI355X): us per launch of `adam_flat` at the PPO learner's
parameter count, HIP-graph replays of 50 launches, for several grid caps, next to a plain
device copy of the same bytes (the HBM / Infinity-Cache floor) and a tiny launch (the
kernel-boundary floor). Usage: python benchmarks/bench_adam.py [n_params]"""
import json
import sys

import torch

from ray_memory_management_amd._native import require_hip


def _time_graph(fn, reps=50, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    h = require_hip()
    dev = torch.device("cuda:0")
    master = torch.randn(n, device=dev)
    m1 = torch.zeros(n, device=dev)
    m2 = torch.zeros(n, device=dev)
    grad = torch.randn(n, device=dev).to(torch.bfloat16)
    wbf = torch.empty(n, dtype=torch.bfloat16, device=dev)
    hp = torch.tensor([5e-5, 0.9, 0.999, 1e-8, 0.0, 1.0], device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    done = torch.zeros(h.bump_done_words(), dtype=torch.int32, device=dev)

    def adam(nn=n, mb=0, bump=True):
        st = torch.cuda.current_stream().cuda_stream
        h.adam_flat(master.data_ptr(), m1.data_ptr(), m2.data_ptr(), grad.data_ptr(), True, wbf.data_ptr(),
                    hp.data_ptr(), 1.0, nn, st, step_ctr=ctr.data_ptr() + 8, bump=ctr.data_ptr() if bump else 0,
                    nbump=2 if bump else 0, done=done.data_ptr() if bump else 0, max_blocks=mb)

    out = {"n_params": n, "bytes_per_launch": 28 * n}
    for mb in (0, 256, 512, 1024, 2048):
        out[f"adam_us_maxblocks{mb}"] = round(_time_graph(lambda mb=mb: adam(mb=mb)), 2)
    out["adam_us_n256"] = round(_time_graph(lambda: adam(nn=256)), 2)
    # the step-counter bump of the last workgroup (two relaxed agent-scope tickets) vs none
    out["adam_us_nobump"] = round(_time_graph(lambda: adam(bump=False)), 2)
    out["adam_us_n256_nobump"] = round(_time_graph(lambda: adam(nn=256, bump=False)), 2)
    src1 = torch.empty(256, dtype=torch.uint8, device=dev)
    dst1 = torch.empty_like(src1)
    out["copy_us_256B"] = round(_time_graph(lambda: dst1.copy_(src1)), 2)
    src = torch.empty(14 * n, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    out["copy_us_same_bytes"] = round(_time_graph(lambda: dst.copy_(src)), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
