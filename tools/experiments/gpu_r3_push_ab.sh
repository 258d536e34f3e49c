# K10 push mode + single-workgroup K16: GPU tests, then runtime bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/push_tests.log 2>&1; rc=$?; tail -3 gpurun_out/push_tests.log; grep -E "FAILED|Error" gpurun_out/push_tests.log | head; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do
  if [ $v = old ]; then export RMM_NO_FOLD_PUSH=1 RMM_K16_MULTI=1; else unset RMM_NO_FOLD_PUSH RMM_K16_MULTI; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/push_rt_$v.log 2>&1 || { tail -5 gpurun_out/push_rt_$v.log; exit 1; }
  echo "runtime $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/push_rt_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/push_rt_$v.log)"
done
unset RMM_NO_FOLD_PUSH RMM_K16_MULTI
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/rollprof2; mkdir -p gpurun_out/rollprof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rollprof2 -o roll -- python3 benchmarks/hybrid_step_trace.py graph double > gpurun_out/rollprof2/run.log 2>&1 || { tail -20 gpurun_out/rollprof2/run.log; exit 1; }
f=$(find gpurun_out/rollprof2 -name "*kernel_stats.csv" | head -1); python3 benchmarks/summarize_prof.py "$f" 8; rm -f $(find gpurun_out/rollprof2 -name "*.db")
