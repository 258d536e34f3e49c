# K10 phase attribution (dbg masks) + one PMC pass of the trunk backward / forward (LDS / MFMA / waits).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u benchmarks/bench_trunk.py > gpurun_out/bench_trunk_r3.txt 2>&1 || { tail -5 gpurun_out/bench_trunk_r3.txt; exit 1; }
cat gpurun_out/bench_trunk_r3.txt
for k in bwd fwd; do
rm -rf gpurun_out/pmc_$k
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/pmc_$k -o run -- python3 benchmarks/bench_trunk.py --only $k --iters 20 > gpurun_out/pmc_$k.log 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_$k.log; exit 1; }
python3 benchmarks/pmc_summary.py gpurun_out/pmc_$k 2>&1 | head -20
done
