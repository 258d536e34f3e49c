# Stall attribution for the fused PPO loop's kernels on one MI355X: one PMC group per run (each within
# the per-block counter limits), --kernel-trace only; benchmarks/pmc_table.py prints per-dispatch
# averages per kernel.   gpurun -- 'OUT=gpurun_out/stalls bash tools/gpu_stalls.sh'
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/stalls}
B="--mode fused --no-putget ${BENCH_ARGS:-} --steps 2 --warmup 1"
rm -rf $O && mkdir -p $O
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o run -- python3 bench.py $B > $O/$n.log 2>&1 || { echo "PASS_FAIL $n"; tail -5 $O/$n.log; exit 1; }
  echo "pass-ok $n"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM
pass b SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LEVEL_WAVES SQ_INSTS_SALU
pass c TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum
python3 benchmarks/pmc_table.py $O/a $O/b $O/c --match "${MATCH:-x3::}" > $O/table.txt 2>&1
cat $O/table.txt
rm -f $(find $O -name "*.db")
