"""Cost of forking work onto a second HIP stream and joining it back, inside a captured graph and
eagerly (the pattern of an all-reduce overlapped with backward on a comm stream).

Each step is kernel A → [fork: kernel C on the side stream] → kernel B → [join] on 1 MI355X; the
script prints µs per step for: no fork, fork inside one graph per step, fork inside a graph of 50
steps, eager fork/join with events. Usage: python benchmarks/stream_fork_cost.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(1 << 20, device=dev)
    y = torch.randn(1 << 20, device=dev)
    z = torch.randn(1 << 16, device=dev)
    side = torch.cuda.Stream(dev)

    def step(fork: bool):
        x.mul_(1.0001)          # A
        if fork:
            cur = torch.cuda.current_stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                z.add_(1.0)     # C
        y.mul_(0.9999)          # B
        if fork:
            torch.cuda.current_stream(dev).wait_stream(side)

    def timed(fn, iters=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    out = {}
    s = torch.cuda.Stream(dev)
    for fork in (False, True):
        for reps in (1, 50):
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                step(fork)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    step(fork)
            out[f"graph_fork{int(fork)}_steps{reps}_us_per_step"] = round(timed(g.replay, 200 // reps + 5) / reps, 2)
        out[f"eager_fork{int(fork)}_us_per_step"] = round(timed(lambda: step(fork)), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
