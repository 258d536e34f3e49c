# Fused Adam epilogues (K12 / K10 trunk reduce) on a gpurun box: learner GPU tests, then fused-loop and
# runtime PPO A/B against the separate K6 launch (RMM_FUSED_ADAM unset). Each GPU step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_fused_adam.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fused_adam.log; grep -E "FAILED|Error" gpurun_out/pytest_fused_adam.log | head -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    RMM_NO_FUSED_ADAM=$([ $v = 1 ] && echo 1 || echo "") timeout -k 10 120 python -u bench.py --mode fused --steps 20 --warmup 3 > gpurun_out/fa_fused_$v.log 2>&1 || { tail -5 gpurun_out/fa_fused_$v.log; exit 1; }
    echo "fused NO_FUSED_ADAM=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fa_fused_$v.log)"
  done
done
for i in 1 2; do
  for v in 1 0; do
    RMM_NO_FUSED_ADAM=$([ $v = 1 ] && echo 1 || echo "") timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/fa_rt_$v.log 2>&1 || { tail -5 gpurun_out/fa_rt_$v.log; exit 1; }
    echo "runtime NO_FUSED_ADAM=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fa_rt_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/fa_rt_$v.log)"
  done
done
