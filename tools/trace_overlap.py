"""Concurrency in a rocprofv3 kernel trace: for every process, how much of each kernel of interest
(`--kernel`, a substring, default the ZeRO-1 peer launch) ran at the same time as kernels matching
`--beside` (default the x3 trunk backward), and on how many distinct queues / streams.

usage: python tools/trace_overlap.py <rocprofv3 output dir> [--kernel k_peer_zero1] [--beside conv2_bwd,conv1_wgrad]
Reads every *kernel_trace.csv below the directory (one per process).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
from collections import defaultdict


def _rows(path):
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            yield r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_peer_zero1")
    ap.add_argument("--beside", default="k_conv2_bwd_x3,k_conv1_wgrad_x3")
    a = ap.parse_args()
    beside = [b for b in a.beside.split(",") if b]
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    per_pid = defaultdict(list)
    for p in files:
        for r in _rows(p):
            name = r.get("Kernel_Name", "")
            pid = r.get("Process_Id") or os.path.basename(os.path.dirname(p))
            per_pid[pid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name,
                                 r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    print(f"# {len(files)} trace file(s); kernel '{a.kernel}' vs {beside}")
    print(f"{'pid':>10} {'launches':>8} {'mean_us':>8} {'overlapped':>10} {'overlap_us':>10} {'queues':>6}  kernels beside")
    for pid, ks in sorted(per_pid.items()):
        mine = [k for k in ks if a.kernel in k[2]]
        if not mine:
            continue
        other = [k for k in ks if any(b in k[2] for b in beside)]
        ov_n, ov_t = 0, 0
        seen = set()
        for s, e, _, q, _ in mine:
            best = 0
            for s2, e2, n2, q2, _ in other:
                o = min(e, e2) - max(s, s2)
                if o > 0:
                    best += o
                    seen.add(n2.split("(")[0][-40:])
            if best > 0:
                ov_n += 1
                ov_t += best
        queues = {k[3] for k in mine} | {k[3] for k in other}
        mean = sum(e - s for s, e, *_ in mine) / len(mine) / 1e3
        print(f"{pid:>10} {len(mine):>8} {mean:>8.1f} {ov_n:>10} {ov_t / 1e3:>10.1f} {len(queues):>6}  {sorted(seen)}")


if __name__ == "__main__":
    main()
