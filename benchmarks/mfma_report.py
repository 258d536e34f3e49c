"""Per-kernel MFMA utilisation report from one rocprofv3 run with --pmc (MFMA counters) and
--kernel-trace (durations), csv output. For every kernel: mean duration, achieved bf16 MFMA
TFLOP/s (SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / duration), that as % of the 2.5 PF dense bf16 peak,
MFMA-busy % (SQ_VALU_MFMA_BUSY_CYCLES over the kernel's duration x 1024 SIMDs x 2.4 GHz), waves.
Usage: python benchmarks/mfma_report.py <rocprof output dir> [top_n]"""
import collections
import csv
import glob
import os
import sys

SIMDS = 256 * 4


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    rows = []
    for k, ds in dur.items():
        n = len(disp.get(k, ())) or 1
        c = {name: v / n for name, v in cnt.get(k, {}).items()}
        t = sum(ds) / len(ds)
        flops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        rows.append((sum(ds), k, len(ds), t, flops / t / 1e3 if t else 0.0,
                     100.0 * busy / (t * 2.4 * SIMDS) if t else 0.0, c.get("SQ_WAVES", 0.0)))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"{'total ms':>9} {'pct':>6} {'calls':>6} {'avg us':>8} {'TFLOP/s':>8} {'%peak':>6} {'MFMAbusy%':>9} "
          f"{'waves':>7}  kernel")
    for s, k, n, t, tf, mb, w in rows[:top]:
        print(f"{s / 1e6:9.2f} {100 * s / tot:6.1f} {n:6d} {t / 1e3:8.1f} {tf:8.1f} {100 * tf / 2500:6.1f} {mb:9.1f} "
              f"{w:7.0f}  {k.split('(')[0][:70]}")


if __name__ == "__main__":
    main()
