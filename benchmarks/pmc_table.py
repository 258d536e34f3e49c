"""Per-kernel PMC counters (per-dispatch averages) from one or more rocprofv3 --pmc runs.

    python benchmarks/pmc_table.py <dir> [<dir> ...] [--match substr]

Each dir is a rocprofv3 ``-d`` output with a counter_collection CSV; kernels are matched by name
across runs. Derived columns: wait% = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (wave time stalled on
s_waitcnt), vmem% / lds% = SQ_ACTIVE_INST_VMEM / _LDS per wave cycle, mfma% = MFMA-busy cycles per
SIMD-cycle of the kernel's busy time."""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("rmm::hip::", "")[:52] + f" g{r.get('Grid_Size', '')}"
                if a.match and a.match not in r["Kernel_Name"]:
                    continue
                c = r["Counter_Name"]
                cnt[k][c] += float(r["Counter_Value"])
                disp[k][c].add(r["Dispatch_Id"])
    for k in sorted(cnt):
        c = {n: v / max(1, len(disp[k][n])) for n, v in cnt[k].items()}
        wc = c.get("SQ_WAVE_CYCLES")
        der = {}
        if wc:
            for n, lab in (("SQ_WAIT_INST_ANY", "wait%"), ("SQ_WAIT_ANY", "waitany%"), ("SQ_ACTIVE_INST_VMEM", "vmem%"),
                           ("SQ_ACTIVE_INST_LDS", "lds%"), ("SQ_WAIT_INST_LDS", "waitlds%")):
                if n in c:
                    der[lab] = 100.0 * c[n] / wc
        if c.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            der["mfma%"] = 100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["SQ_BUSY_CYCLES"] * 4 * 256 / 8)
        if c.get("TCP_TCC_READ_REQ_sum"):
            der["l2lat_cyc"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / c["TCP_TCC_READ_REQ_sum"]
        print(k)
        print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
        print("   derived: " + "  ".join(f"{n}={v:.1f}" for n, v in der.items()))


if __name__ == "__main__":
    main()
