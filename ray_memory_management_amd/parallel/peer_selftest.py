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
        comm = PeerComm(store, rank, world, key=f"sw{nb}", device=dev, cap_bytes=16 << 20, nblocks=nb,
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

    # broadcast (all-reduce against zeros) from the last rank
    g = torch.Generator().manual_seed(77)
    src = torch.randn(12345, generator=g).to(d)
    b = src.clone() if rank == world - 1 else torch.full_like(src, 3.0)
    comm.broadcast(b, src=world - 1)
    torch.cuda.synchronize()
    res["cases"]["broadcast_fp32"] = {"ok": bool(torch.equal(b, src)), "n": 12345}

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
    dead = PeerComm(store, rank, world, key="dead", device=dev, cap_bytes=1 << 16, timeout_s=0.5)
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
