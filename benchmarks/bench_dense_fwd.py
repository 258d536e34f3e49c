"""K13 vs K13s timing for the PPO dense layer (x[M,3872] · W[256,3872]ᵀ + b, ReLU), per M: mean µs
per launch over HIP-graph replays of 50 back-to-back launches, plus the consumer side: K15 (SGD step,
M = 500) and K16 (rollout, M = 12 / 25) reading bf16 hidden vs summing the K13s partials.

Round 2 tried a split-K variant with the reduction in-kernel (agent-scope release/acquire = L2
write-back across XCDs: 4x slower) or in a separate reduce launch (1.1-1.7x slower than K13). K13s
moves the reduction into the consumer's prologue (no extra boundary). RMM_K13S_S=<S> overrides the
slice count (read once per process). Usage: python benchmarks/bench_dense_fwd.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_memory_management_amd._native import require_hip  # noqa: E402


def _time(fn, reps=50, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / (iters * reps) * 1e3, 2)


def main():
    h = require_hip()
    K, N, A1 = 3872, 256, 5
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    out = {"S_override": os.environ.get("RMM_K13S_S")}
    for M in (12, 13, 25, 50, 500):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        S = h.dense_fwd_part_slices(M, K, N)
        part = torch.empty(S * M * N, device="cuda", dtype=torch.float32)
        r = {"S": S}
        r["k13_us"] = _time(lambda: h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, y.data_ptr(),
                                                     st()))
        r["k13s_us"] = _time(lambda: h.dense_fwd_part(x.data_ptr(), w.data_ptr(), M, K, N, part.data_ptr(), S, st()))
        wh = (torch.randn(A1, N, device="cuda") * 0.05).to(torch.bfloat16)
        bh = torch.zeros(A1, device="cuda", dtype=torch.bfloat16)
        if M == 500:
            cols = torch.randn(M, A1 - 1 + 4, device="cuda")
            cols[:, A1 - 1 + 3] = torch.randint(0, A1 - 1, (M,), device="cuda").float()
            coef = torch.tensor([0.1, 10.0, 1.0, 0.01, 0.2], device="cuda")
            acc = torch.zeros(6, device="cuda")
            one = torch.ones(1, device="cuda")
            dz = torch.empty(M, A1, device="cuda", dtype=torch.bfloat16)
            dpre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            hid2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            r["k15_us"] = _time(lambda: h.dense_heads_ppo(y.data_ptr(), wh.data_ptr(), bh.data_ptr(), cols.data_ptr(),
                                                          coef.data_ptr(), acc.data_ptr(), one.data_ptr(), M, A1,
                                                          dz.data_ptr(), dpre.data_ptr(), st()))
            r["k15_part_us"] = _time(lambda: h.dense_heads_ppo(
                0, wh.data_ptr(), bh.data_ptr(), cols.data_ptr(), coef.data_ptr(), acc.data_ptr(), one.data_ptr(), M,
                A1, dz.data_ptr(), dpre.data_ptr(), st(), hpart=part.data_ptr(), S=S, hb=b.data_ptr(),
                hid_out=hid2.data_ptr()))
        else:
            t = torch.zeros(1, dtype=torch.int64, device="cuda")
            act = torch.empty(4 * M, dtype=torch.int64, device="cuda")
            logp = torch.empty(4 * M, device="cuda")
            vf = torch.empty(4 * M, device="cuda")
            lout = torch.empty(4 * M * (A1 - 1), device="cuda")
            an = torch.empty(M, dtype=torch.int64, device="cuda")
            r["k16_us"] = _time(lambda: h.dense_heads_sample(y.data_ptr(), wh.data_ptr(), bh.data_ptr(), t.data_ptr(),
                                                             t.data_ptr(), 7, act.data_ptr(), logp.data_ptr(),
                                                             vf.data_ptr(), lout.data_ptr(), an.data_ptr(), M, A1, st()))
            r["k16_part_us"] = _time(lambda: h.dense_heads_sample(
                0, wh.data_ptr(), bh.data_ptr(), t.data_ptr(), t.data_ptr(), 7, act.data_ptr(), logp.data_ptr(),
                vf.data_ptr(), lout.data_ptr(), an.data_ptr(), M, A1, st(), hpart=part.data_ptr(), S=S,
                hb=b.data_ptr()))
        # numerics: partial path hidden vs K13's
        h.dense_fwd_part(x.data_ptr(), w.data_ptr(), M, K, N, part.data_ptr(), S, st())
        ref = torch.relu(x.float() @ w.float().t() + b.float())
        got = torch.relu(part.view(S, M, N).sum(0) + b.float())
        r["max_abs_err_vs_fp32"] = float((got - ref).abs().max())
        r["k13_max_abs_err_vs_fp32"] = float((y.float() - ref).abs().max())
        out[f"M{M}"] = r
        print(json.dumps({f"M{M}": r}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
