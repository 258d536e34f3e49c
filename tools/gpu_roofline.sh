# Per-kernel roofline of the fused PPO loop (bench.py --mode fused: learner SGD steps + rollout kernels
# in one process) on one MI355X: (1) kernel-trace durations, (2) FETCH_SIZE pass, (3) WRITE_SIZE pass,
# (4) MFMA/VALU pass, (5) LDS pass — one PMC group per run, each with --kernel-trace only; then
# benchmarks/roofline_report.py joins them by kernel name.
#   gpurun -- 'OUT=gpurun_out/roof BENCH_ARGS="--dtype fp32" bash tools/gpu_roofline.sh'
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/roof}
B="--mode fused --no-putget ${BENCH_ARGS:-}"
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B --steps 5 --warmup 2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
echo trace-ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py $B --steps 2 --warmup 1 > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $O/fetch.log; exit 1; }
echo fetch-ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py $B --steps 2 --warmup 1 > $O/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $O/write.log; exit 1; }
echo write-ok
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/mfma -o run -- python3 bench.py $B --steps 2 --warmup 1 > $O/mfma.log 2>&1 || { echo MFMA_FAIL; tail -5 $O/mfma.log; exit 1; }
echo mfma-ok
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O/lds -o run -- python3 bench.py $B --steps 2 --warmup 1 > $O/lds.log 2>&1 || { echo LDS_FAIL; tail -5 $O/lds.log; exit 1; }
python3 benchmarks/roofline_report.py $O/trace $O/fetch $O/write $O/mfma $O/lds --top 30 > $O/roofline.txt 2>&1
cat $O/roofline.txt
tail -1 $O/trace.log
rm -f $(find $O -name "*.db")
