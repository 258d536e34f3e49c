"""Per-kernel roofline table from several rocprofv3 runs of the same program (one PMC group per run,
each with --kernel-trace): duration, HBM bytes (FETCH_SIZE / WRITE_SIZE, KiB per dispatch), achieved
GB/s and % of the 8 TB/s HBM3E peak, bf16 MFMA TFLOP/s and MFMA-busy %, VALU / LDS instruction
counts and LDS bank-conflict cycles per dispatch.

    python benchmarks/roofline_report.py <dir> [<dir> ...] [--top 25] [--match substr]

Each dir is a rocprofv3 ``-d`` output; kernels are matched across runs by name. Durations come from
the FIRST dir (a --kernel-trace-only run: the counter runs serialise dispatches, so their
kernel-trace durations are inflated and only their counter values are used)."""
import argparse
import collections
import csv
import glob
import os

SIMDS = 256 * 4
CLK_GHZ = 2.4
HBM_GBPS = 8000.0
MFMA_PEAK_TF = 2500.0


def load(d):
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
    per = {k: {n: v / max(1, len(disp[k])) for n, v in c.items()} for k, c in cnt.items()}
    return dur, per


def short(k):
    return k.split("(")[0].replace("rmm::hip::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    durs, ctrs = {}, collections.defaultdict(dict)
    for i, d in enumerate(a.dirs):
        dur, per = load(d)
        if i == 0:  # the trace-only run: reference durations
            durs = dur
        for k, c in per.items():
            ctrs[k].update(c)
    rows = []
    for k, ds in durs.items():
        if a.match and a.match not in k:
            continue
        t_us = sum(ds) / len(ds) / 1e3
        c = ctrs.get(k, {})
        rd = c.get("FETCH_SIZE")
        wr = c.get("WRITE_SIZE")
        byts = None if rd is None and wr is None else 1024.0 * ((rd or 0.0) + (wr or 0.0))
        gbps = byts / (t_us * 1e3) if byts is not None and t_us else None
        tf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / (t_us * 1e6) if t_us else 0.0
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mb = None if busy is None else 100.0 * busy / (t_us * 1e3 * CLK_GHZ * SIMDS)
        rows.append(dict(total=sum(ds) / 1e6, k=k, n=len(ds), t=t_us, rd=rd, wr=wr, gbps=gbps, tf=tf, mb=mb,
                         valu=c.get("SQ_INSTS_VALU"), lds=c.get("SQ_INSTS_LDS"),
                         bank=c.get("SQ_LDS_BANK_CONFLICT"), waves=c.get("SQ_WAVES")))
    rows.sort(key=lambda r: -r["total"])

    def f(v, fmt):
        return "-" if v is None else format(v, fmt)

    print(f"{'tot ms':>7} {'calls':>6} {'avg us':>7} {'rd KiB':>8} {'wr KiB':>8} {'GB/s':>7} {'%HBM':>5} "
          f"{'TF/s':>6} {'MFMA%':>6} {'VALU/d':>9} {'LDS/d':>8} {'bankcf':>8} {'waves':>6}  kernel")
    for r in rows[:a.top]:
        print(f"{r['total']:7.2f} {r['n']:6d} {r['t']:7.1f} {f(r['rd'], '8.0f')} {f(r['wr'], '8.0f')} "
              f"{f(r['gbps'], '7.0f')} {f(None if r['gbps'] is None else 100 * r['gbps'] / HBM_GBPS, '5.1f')} "
              f"{r['tf']:6.1f} {f(r['mb'], '6.1f')} {f(r['valu'], '9.0f')} {f(r['lds'], '8.0f')} "
              f"{f(r['bank'], '8.0f')} {f(r['waves'], '6.0f')}  {short(r['k'])}")


if __name__ == "__main__":
    main()
