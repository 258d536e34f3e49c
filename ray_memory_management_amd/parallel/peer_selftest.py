"""Multi-process self-test and micro-benchmark of PeerComm (csrc/hip/peer_allreduce.hip).

``python -m ray_memory_management_amd.parallel.peer_selftest --world 2 --out DIR`` starts `world`
rank processes (all on GPU 0 when there is one GPU: the 1-GPU rehearsal; rank r on GPU r otherwise),
rendezvoused through a FileStore. Every rank builds every rank's inputs from the same seeds, so it
checks its result against the exact reference: the fp32 sum of the per-rank buffers in rank order,
rounded once to the buffer's dtype. Each rank writes ``DIR/rank<r>.json``; the parent prints one
JSON summary and exits non-zero on any mismatch.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time


def _inputs(n, dtype, world, seed, device):
    import torch

    out = []
    for r in range(world):
        g = torch.Generator().manual_seed(seed * 1000 + r)
        out.append((torch.randn(n, generator=g) * (1 + r)).to(dtype).to(device))
    return out


def _ref(xs):
    acc = xs[0].float().clone()
    for x in xs[1:]:
        acc = acc + x.float()
    return acc.to(xs[0].dtype)


def _sweep(rank, world, store, d, dev, iters):
    """µs per all-reduce over payload sizes x workgroup counts (eager back-to-back and 25 per graph)."""
    import torch

    from ray_memory_management_amd.parallel.comm import PeerComm

    out = []
    for nb in (8, 32, 64, 128, 256):
        # short flag timeout: on ONE shared GPU the ranks' kernels (world x nb workgroups) are not
        # guaranteed to be co-resident, and a configuration that cannot be is recorded, not fatal
        comm = PeerComm(store, rank, world, key=f"sw{nb}", device=dev, cap_bytes=16 << 20, nblocks=nb, zero1_blocks=0,
                        timeout_s=5.0)
        failed = None
        for nbytes in (4 << 10, 64 << 10, 1354858, 8 << 20):
            for algo in ((1, 2) if world > 2 else (1,)):
                comm.algo = algo
                x = torch.zeros(nbytes // 2, dtype=torch.bfloat16, device=d)
                for _ in range(5):
                    comm.allreduce(x)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    comm.allreduce(x)
                torch.cuda.synchronize()
                eager = (time.perf_counter() - t0) / iters * 1e6
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(25):
                        comm.allreduce(x)
                g.replay()
                torch.cuda.synchronize()
                reps = max(1, iters // 25)
                t0 = time.perf_counter()
                for _ in range(reps):
                    g.replay()
                torch.cuda.synchronize()
                graph = (time.perf_counter() - t0) / (reps * 25) * 1e6
                try:
                    comm.check()
                except RuntimeError as e:
                    failed = str(e)[:200]
                out.append({"nblocks": nb, "bytes": nbytes, "algo": algo, "us_eager": round(eager, 2),
                            "us_graph": round(graph, 2), **({"error": failed} if failed else {})})
                if failed:
                    break
            if failed:
                break
        store.add(f"sw{nb}/done", 1)
        while int(store.add(f"sw{nb}/done", 0)) < world:
            time.sleep(0.001)
        comm.close()
    return out


def _zero1_cases(rank, world, comm, d, res):
    """PeerComm.allreduce_adam_on (ZeRO-1: reduce-scatter + Adam + all-gather in one launch) against the
    unfused path: the fp32 sum in rank order (rounded once for bf16 gradients) -> K6 adam_flat on the
    same state. Masters and weight planes must match bit for bit on every rank; the moments after
    replicate_moments; the step counters advance once per step (ticket and parity forms)."""
    import torch

    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    st = torch.cuda.current_stream(d)

    def state(n, seed):
        g = torch.Generator().manual_seed(seed)
        master = (torch.randn(n, generator=g) * 0.1).to(d)
        m1 = (torch.randn(n, generator=g) * 1e-3).to(d)
        m2 = (torch.rand(n, generator=g) * 1e-5).to(d)
        return master, m1, m2

    def planes(n):
        return (torch.empty(n, dtype=torch.bfloat16, device=d), torch.empty(n, dtype=torch.bfloat16, device=d))

    hp = torch.tensor([3e-4, 0.9, 0.999, 1e-8, 0.0, 1.0], device=d)

    def run(name, n, gdt, seed, steps=2, split=True, parity=False, graph=False):
        master, m1, m2 = state(n, seed)
        rmaster, rm1, rm2 = master.clone(), m1.clone(), m2.clone()
        whi, wlo = planes(n)
        rhi, rlo = planes(n)
        ctr = torch.tensor([5, 7], dtype=torch.int64, device=d)
        ctr2 = ctr.clone()
        rctr = ctr.clone()
        done = torch.zeros(h.bump_done_words(), dtype=torch.int32, device=d)
        rdone = torch.zeros_like(done)
        grads = []
        for k in range(steps):
            xs = _inputs(n, gdt, world, seed * 100 + k, d)
            grads.append(xs)
        gbuf = torch.empty(n, dtype=gdt, device=d)
        scale = 1.0 / world
        cur = [ctr, ctr2]

        def step(k):
            c = cur[k % 2] if parity else ctr
            kw = dict(master=master.data_ptr(), m1=m1.data_ptr(), m2=m2.data_ptr(), whi=whi.data_ptr(),
                      wlo=wlo.data_ptr() if split else 0, hp=hp.data_ptr(), grad_scale=scale,
                      step_ctr=c.data_ptr() + 8, bump=c.data_ptr(), nbump=2)
            if parity:
                kw["bump_next"] = cur[(k + 1) % 2].data_ptr()
            else:
                kw["done"] = done.data_ptr()
            comm.allreduce_adam_on(gbuf, torch.cuda.current_stream(d), **kw)  # the capture stream under a graph

        if graph:  # capture `steps` fused steps (gradients copied in per step from a staging list)
            srcs = [torch.empty(n, dtype=gdt, device=d) for _ in range(steps)]
            for k in range(steps):
                srcs[k].copy_(grads[k][rank])
            gr = torch.cuda.CUDAGraph()
            # warm-up and capture would both step the state: capture on copies, replay on the real state
            saved = [t.clone() for t in (master, m1, m2, ctr, ctr2)]
            s0 = torch.cuda.Stream(d)
            s0.wait_stream(st)
            with torch.cuda.stream(s0):
                gbuf.copy_(srcs[0])
                step(0)
            st.wait_stream(s0)
            torch.cuda.synchronize()
            with torch.cuda.graph(gr):
                for k in range(steps):
                    gbuf.copy_(srcs[k])
                    step(k)
            for t, v in zip((master, m1, m2, ctr, ctr2), saved):
                t.copy_(v)
            torch.cuda.synchronize()
            gr.replay()
        else:
            for k in range(steps):
                gbuf.copy_(grads[k][rank])
                step(k)
        torch.cuda.synchronize()
        comm.check()
        for k in range(steps):  # reference: all-reduce (rank order, rounded once) -> K6
            gsum = _ref(grads[k])
            h.adam_flat(rmaster.data_ptr(), rm1.data_ptr(), rm2.data_ptr(), gsum.data_ptr(), gdt == torch.bfloat16,
                        rhi.data_ptr(), hp.data_ptr(), scale, n, st.cuda_stream, step_ctr=rctr.data_ptr() + 8,
                        bump=rctr.data_ptr(), nbump=2, done=rdone.data_ptr(), wlo=rlo.data_ptr() if split else 0)
        comm.replicate_moments(gdt, n, m1.data_ptr(), m2.data_ptr())
        torch.cuda.synchronize()
        comm.check()
        want_ctr = rctr if not parity else rctr
        got_ctr = cur[steps % 2] if parity else ctr
        ok = {"master": torch.equal(master, rmaster), "whi": torch.equal(whi, rhi),
              "wlo": (not split) or torch.equal(wlo, rlo), "m1": torch.equal(m1, rm1), "m2": torch.equal(m2, rm2),
              "ctr": torch.equal(got_ctr, want_ctr)}
        res["cases"][name] = {"ok": all(ok.values()), "n": n, "parts": ok,
                              "max_abs_err": float((master - rmaster).abs().max())}

    run("zero1_fp32_chunked", 300007, torch.float32, 11)          # 2 launches at a 1 MB cap
    run("zero1_bf16_nolo", 100003, torch.bfloat16, 12, split=False)
    run("zero1_fp32_parity", 4099, torch.float32, 13, steps=3, parity=True)
    run("zero1_fp32_graph", 65541, torch.float32, 14, steps=3, parity=True, graph=True)
    run("zero1_tiny", 6, torch.float32, 15)

    # timing on the fp32 PPO bucket (x3 learner, 1,005,109 params): all-reduce -> K6 vs the fused launch
    n = 1_005_109
    master, m1, m2 = state(n, 21)
    whi, wlo = planes(n)
    ctr = torch.zeros(2, dtype=torch.int64, device=d)
    done = torch.zeros(h.bump_done_words(), dtype=torch.int32, device=d)
    gbuf = _inputs(n, torch.float32, world, 22, d)[rank]
    kw = dict(master=master.data_ptr(), m1=m1.data_ptr(), m2=m2.data_ptr(), whi=whi.data_ptr(), wlo=wlo.data_ptr(),
              hp=hp.data_ptr(), grad_scale=1.0 / world, step_ctr=ctr.data_ptr() + 8, bump=ctr.data_ptr(), nbump=2,
              done=done.data_ptr())

    def unfused():
        comm.allreduce(gbuf)
        h.adam_flat(master.data_ptr(), m1.data_ptr(), m2.data_ptr(), gbuf.data_ptr(), False, whi.data_ptr(),
                    hp.data_ptr(), 1.0 / world, n, st.cuda_stream, step_ctr=ctr.data_ptr() + 8, bump=ctr.data_ptr(),
                    nbump=2, done=done.data_ptr(), wlo=wlo.data_ptr())

    def fused():
        comm.allreduce_adam_on(gbuf, torch.cuda.current_stream(d), **kw)

    for name, fn in (("unfused", unfused), ("zero1", fused)):
        for _ in range(5):
            fn()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            gr.replay()
        torch.cuda.synchronize()
        res[f"ppo_bucket_fp32_us_{name}"] = round((time.perf_counter() - t0) / 100 * 1e6, 2)
    comm.check()


def _rank_main(rank, world, path, out_dir, bench_iters, sweep=False):
    import torch
    import torch.distributed as dist

    from ray_memory_management_amd.parallel.comm import PeerComm

    ndev = torch.cuda.device_count()
    dev = rank if ndev >= world else 0
    torch.cuda.set_device(dev)
    d = torch.device("cuda", dev)
    store = dist.FileStore(path, world)
    if sweep:
        res = {"rank": rank, "device": dev, "sweep": _sweep(rank, world, store, d, dev, bench_iters), "ok": True}
        with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        return
    res = {"rank": rank, "device": dev, "cases": {}}
    comm = PeerComm(store, rank, world, key="t", device=dev, cap_bytes=1 << 20)
    res["uncached_signals"] = bool(comm._c.uncached_signals)
    res["alloc_attempts"] = int(comm._c.alloc_attempts)

    def case(name, n, dtype, seed, algo=0):
        xs = _inputs(n, dtype, world, seed, d)
        comm.algo = algo
        x = xs[rank].clone()
        comm.allreduce(x)
        torch.cuda.synchronize()
        comm.check()
        ref = _ref(xs)
        ok = bool(torch.equal(x, ref))
        res["cases"][name] = {"ok": ok, "n": n, "max_abs_err": float((x.float() - ref.float()).abs().max())}
        comm.algo = 0

    case("bf16_odd_oneshot", 677429, torch.bfloat16, 1)
    case("bf16_chunked_3MB", 1_500_001, torch.bfloat16, 2)       # 3 launches at a 1 MB cap
    case("fp32_tiny", 6, torch.float32, 3)
    case("bf16_twoshot", 100003, torch.bfloat16, 4, algo=2)
    case("fp32_twoshot_chunked", 300007, torch.float32, 5, algo=2)
    case("bf16_oneshot_forced", 4097, torch.bfloat16, 6, algo=1)

    _zero1_cases(rank, world, comm, d, res)

    # broadcast (all-reduce against zeros) from the last rank
    g = torch.Generator().manual_seed(77)
    src = torch.randn(12345, generator=g).to(d)
    b = src.clone() if rank == world - 1 else torch.full_like(src, 3.0)
    comm.broadcast(b, src=world - 1)
    torch.cuda.synchronize()
    res["cases"]["broadcast_fp32"] = {"ok": bool(torch.equal(b, src)), "n": 12345}
    src64 = (torch.randn(777, generator=g, dtype=torch.float64) * 1e-300).to(d)  # not fp32-representable
    b64 = src64.clone() if rank == 0 else torch.full_like(src64, 5.0)
    comm.broadcast(b64, src=0)
    i64 = torch.randint(-2**62, 2**62, (33,), generator=g, dtype=torch.int64).to(d)
    bi = i64.clone() if rank == 0 else torch.zeros_like(i64)
    comm.broadcast(bi, src=0)
    s0 = torch.tensor(-(2**61) - 7, dtype=torch.int64, device=d)  # 0-dim, 8-byte dtype
    b0 = s0.clone() if rank == 0 else torch.zeros_like(s0)
    comm.broadcast(b0, src=0)
    torch.cuda.synchronize()
    res["cases"]["broadcast_bytes_f64_i64"] = {"ok": bool(torch.equal(b64, src64)) and bool(torch.equal(bi, i64))
                                               and b0.dim() == 0 and bool(torch.equal(b0, s0)), "n": 818}

    # graph capture: 3 all-reduces inside one graph, replayed with fresh inputs
    n = 65536 + 3
    srcs = [torch.empty(n, dtype=torch.bfloat16, device=d) for _ in range(3)]
    outs = [torch.empty_like(s) for s in srcs]
    work = [torch.empty_like(s) for s in srcs]
    for s in srcs:
        s.zero_()
    s0 = torch.cuda.Stream(d)
    s0.wait_stream(torch.cuda.current_stream(d))
    with torch.cuda.stream(s0):  # warm-up outside capture (same launch sequence on every rank)
        for i in range(3):
            work[i].copy_(srcs[i])
            comm.allreduce(work[i])
            outs[i].copy_(work[i])
    torch.cuda.current_stream(d).wait_stream(s0)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for i in range(3):
            work[i].copy_(srcs[i])
            comm.allreduce(work[i])
            outs[i].copy_(work[i])
    gok = True
    for rep in range(4):
        refs = []
        for i in range(3):
            xs = _inputs(n, torch.bfloat16, world, 100 + rep * 10 + i, d)
            srcs[i].copy_(xs[rank])
            refs.append(_ref(xs))
        graph.replay()
        torch.cuda.synchronize()
        comm.check()
        gok = gok and all(bool(torch.equal(o, r)) for o, r in zip(outs, refs))
    res["cases"]["graph_replay"] = {"ok": gok, "n": n, "replays": 4}

    # timing: the PPO gradient bucket (677429 bf16 = 1.35 MB), eager back-to-back and in one graph
    x = _inputs(677429, torch.bfloat16, world, 9, d)[rank]
    store.add("bench", 1)
    while int(store.add("bench", 0)) < world:
        time.sleep(0.001)
    for _ in range(5):
        comm.allreduce(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(bench_iters):
        comm.allreduce(x)
    torch.cuda.synchronize()
    res["bucket_us_eager"] = (time.perf_counter() - t0) / bench_iters * 1e6
    gb = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gb):
        for _ in range(25):
            comm.allreduce(x)
    gb.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(max(1, bench_iters // 25)):
        gb.replay()
    torch.cuda.synchronize()
    res["bucket_us_graph"] = (time.perf_counter() - t0) / (max(1, bench_iters // 25) * 25) * 1e6
    comm.check()

    # bounded wait: a communicator whose peer never launches reports an error instead of hanging
    dead = PeerComm(store, rank, world, key="dead", device=dev, cap_bytes=1 << 16, timeout_s=0.5, zero1_blocks=0)
    if rank == 0:
        y = torch.ones(1000, device=d)
        t0 = time.perf_counter()
        dead.allreduce(y)
        torch.cuda.synchronize()
        t_first = time.perf_counter() - t0
        try:
            dead.check()
            raised = False
        except RuntimeError:
            raised = True
        t0 = time.perf_counter()
        dead.allreduce(y)  # the device error word short-circuits every later launch
        torch.cuda.synchronize()
        t_second = time.perf_counter() - t0
        res["cases"]["timeout_reported"] = {"ok": raised and t_first < 5.0 and t_second < 0.25,
                                            "first_s": t_first, "second_s": t_second}
    store.add("done", 1)
    while int(store.add("done", 0)) < world:
        time.sleep(0.002)
    dead.close()
    comm.close()
    res["ok"] = all(c["ok"] for c in res["cases"].values())
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--out", default="/tmp/peer_selftest")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--store", default="")
    ap.add_argument("--sweep", action="store_true", help="timing sweep over sizes x workgroup counts")
    a = ap.parse_args()
    if a.rank >= 0:
        _rank_main(a.rank, a.world, a.store, a.out, a.iters, a.sweep)
        return
    os.makedirs(a.out, exist_ok=True)
    store = os.path.join(a.out, f"store-{os.getpid()}")
    if os.path.exists(store):
        os.unlink(store)
    procs = [subprocess.Popen([sys.executable, "-m", "ray_memory_management_amd.parallel.peer_selftest", "--world",
                               str(a.world), "--out", a.out, "--iters", str(a.iters), "--rank", str(r), "--store",
                               store] + (["--sweep"] if a.sweep else [])) for r in range(a.world)]
    rcs = [p.wait() for p in procs]
    results = []
    for r in range(a.world):
        try:
            with open(os.path.join(a.out, f"rank{r}.json")) as f:
                results.append(json.load(f))
        except OSError:
            results.append({"rank": r, "ok": False, "error": "no result"})
    summary = {"world": a.world, "rcs": rcs, "ok": all(rc == 0 for rc in rcs) and all(r.get("ok") for r in results),
               "ranks": results}
    print(json.dumps(summary))
    sys.exit(0 if summary["ok"] else 1)


if __name__ == "__main__":
    main()
