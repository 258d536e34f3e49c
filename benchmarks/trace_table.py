"""Per-kernel, per-launch-shape duration table from a rocprofv3 --kernel-trace CSV run.

    python benchmarks/trace_table.py <rocprofv3 -d dir> [--top 25] [--match substr]

Launches of one kernel with different grids (e.g. the SGD step's B=500 trunk forward vs the rollout's
B=50) are separate rows: total ms, calls, mean and median us, grid / workgroup size, LDS bytes, VGPRs."""
import argparse
import collections
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    rows = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if a.match and a.match not in k:
                continue
            k = k.replace("(anonymous namespace)::", "")
            key = (k.split("(")[0].replace("rmm::hip::", "")[:56], r["Grid_Size_X"], r["Workgroup_Size_X"],
                   r["LDS_Block_Size"], r["VGPR_Count"])
            rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'tot ms':>7} {'calls':>6} {'mean us':>8} {'med us':>7} {'grid':>8} {'wg':>4} {'lds':>7} {'vgpr':>4}  kernel")
    for (k, grid, wg, lds, vgpr), d in sorted(rows.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"{sum(d) / 1e3:7.2f} {len(d):6d} {sum(d) / len(d):8.1f} {statistics.median(d):7.1f} {grid:>8} {wg:>4} "
              f"{lds:>7} {vgpr:>4}  {k}")


if __name__ == "__main__":
    main()
