"""Per-SGD-step timeline from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

An SGD step of the fused PPO learner is the kernel run k_trunk_fwd → k_dense_fwd → k_heads_ppo →
k_dense_heads_bwd2 → k_trunk_bwd → k_trunk_reduce → k_adam_flat inside one graph replay. For every
step found in the trace this prints the wall span (first start → last end), the summed kernel time
and the idle gaps between kernels, then the medians, and the same for rollout steps
(k_frame_push / k_synth_env_step → k_trunk_fwd → k_dense_fwd → k_heads_sample).

Usage: python benchmarks/step_timeline.py <dir-or-kernel_trace.csv>
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys

SGD = ["k_trunk_fwd", "k_dense_fwd", "k_heads_ppo", "k_dense_heads_bwd2", "k_trunk_bwd", "k_trunk_reduce",
       "k_adam_flat"]
ROLL = ["k_trunk_fwd", "k_dense_fwd", "k_heads_sample"]


def _short(name: str) -> str:
    base = name.split("(")[0]
    base = base.split("<")[0] if "<" in base and "::" not in base.split("<")[0][-3:] else base
    return base.split("::")[-1].split("<")[0]


def load(path: str):
    if os.path.isdir(path):
        files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not files:
            raise SystemExit(f"no *kernel_trace.csv under {path}")
        path = files[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]),
                     int(r.get("Queue_Id", 0) or 0)))
    rows.sort()
    return rows


def find_runs(rows, pattern):
    out = []
    names = [r[2] for r in rows]
    i = 0
    while i + len(pattern) <= len(rows):
        if names[i:i + len(pattern)] == pattern:
            seg = rows[i:i + len(pattern)]
            span = seg[-1][1] - seg[0][0]
            busy = sum(e - s for s, e, _, _ in seg)
            per = [(n, (e - s) / 1e3) for s, e, n, _ in seg]
            gaps = [(seg[k + 1][0] - seg[k][1]) / 1e3 for k in range(len(seg) - 1)]
            out.append((span / 1e3, busy / 1e3, per, gaps))
            i += len(pattern)
        else:
            i += 1
    return out


def report(title, runs):
    if not runs:
        print(f"{title}: none found")
        return
    span = statistics.median(r[0] for r in runs)
    busy = statistics.median(r[1] for r in runs)
    print(f"{title}: {len(runs)} steps, median span {span:.1f} us, kernel busy {busy:.1f} us, "
          f"gaps {span - busy:.1f} us")
    k = len(runs[0][2])
    for j in range(k):
        name = runs[0][2][j][0]
        med = statistics.median(r[2][j][1] for r in runs)
        gap = statistics.median(r[3][j] for r in runs) if j < k - 1 else 0.0
        print(f"   {name:<22} {med:7.1f} us   gap after {gap:5.1f} us")


def main():
    rows = load(sys.argv[1])
    report("SGD step", find_runs(rows, SGD))
    report("rollout inference", find_runs(rows, ROLL))


if __name__ == "__main__":
    main()
