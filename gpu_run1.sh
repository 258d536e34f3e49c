set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc3 gpurun_out/pmc4
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA -d gpurun_out/pmc3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-putget > gpurun_out/pmc3.log 2>&1; echo "pmc3 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH -d gpurun_out/pmc4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-putget > gpurun_out/pmc4.log 2>&1; echo "pmc4 rc=$?"
python3 - <<'PY'
import csv, collections, glob
for d in ("pmc3", "pmc4"):
    fs = glob.glob(f"gpurun_out/{d}/*counter_collection.csv")
    if not fs: print(d, "missing"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "dense" in k or "trunk_bwd" in k:
            agg[k[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        print(d, k, {c: round(sum(v) / len(v)) for c, v in dd.items()})
PY
rm -rf gpurun_out/pmc3 gpurun_out/pmc4
