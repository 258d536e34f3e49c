# Zero-copy shared learner weights: GPU tests, then runtime A/B vs a copy per iteration.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sw_pytest.log; grep -E "FAILED|Error" gpurun_out/sw_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in 0 1; do
    RMM_NO_SHARED_WEIGHTS=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/shw_$v.log 2>&1 || { tail -5 gpurun_out/shw_$v.log; exit 1; }
    echo "runtime NO_SHARED=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/shw_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/shw_$v.log)"
  done
done
RMM_NO_SHARED_WEIGHTS=0 timeout -k 10 200 python -u benchmarks/ppo_phase_probe.py 1 > gpurun_out/shw_phase.log 2>&1 && tail -1 gpurun_out/shw_phase.log
