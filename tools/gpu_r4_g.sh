# Round 4 (g): K10 bias prefetch + reduce variant: tests, phase timing; LDS bank-conflict attribution per
# K10 phase (PMC); K13s configuration sweep on the fused loop.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 || { tail -40 gpurun_out/pytest_g.log; exit 1; }
tail -1 gpurun_out/pytest_g.log
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_g.json 2> gpurun_out/trunk_phases_g.err || { tail -5 gpurun_out/trunk_phases_g.err; exit 1; }
cat gpurun_out/trunk_phases_g.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in bwd fwd; do
  for d in 0 1 2 4 8 16 32; do
    rm -rf gpurun_out/pmc_$k$d
    timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_$k$d -o run -- python3 benchmarks/bench_trunk.py --only $k --dbg $d --iters 20 > gpurun_out/pmc_$k$d.log 2>&1 || { echo PMC_FAIL $k $d; tail -5 gpurun_out/pmc_$k$d.log; exit 1; }
    echo "$k dbg=$d $(python3 benchmarks/roofline_report.py gpurun_out/pmc_$k$d gpurun_out/pmc_$k$d --match trunk --top 2 | tail -2 | tr -s ' ' | cut -c1-160)"
    rm -f $(find gpurun_out/pmc_$k$d -name "*.db")
  done
done
cd "$GRAFT_REPO_ROOT"
for c in 0 1 2 3 4 5 6; do
  RMM_K13S_CFG=$c timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/k13s_$c.log 2>&1 || { tail -5 gpurun_out/k13s_$c.log; exit 1; }
  echo "K13S_CFG=$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k13s_$c.log)"
done
