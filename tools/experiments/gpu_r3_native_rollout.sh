# Native hybrid rollout loop (csrc/hip/rollout_loop.cc) + native synthetic env: GPU tests of the hybrid
# worker, then runtime PPO A/B against the Python loop (RMM_NO_NATIVE_ROLLOUT=1), group streams on/off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -v --timeout 200 --timeout-method thread -k "hybrid or native or k19" > gpurun_out/pytest_native_rollout.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_native_rollout.log; grep -E "FAILED|Error" gpurun_out/pytest_native_rollout.log | head -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    RMM_NO_NATIVE_ROLLOUT=$([ $v = 1 ] && echo 1 || echo "") timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/nr_rt_$v.log 2>&1 || { tail -5 gpurun_out/nr_rt_$v.log; exit 1; }
    echo "runtime NO_NATIVE_ROLLOUT=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nr_rt_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/nr_rt_$v.log)"
  done
done
for gs in 1; do
  RMM_GROUP_STREAMS=$gs timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/nr_gs_$gs.log 2>&1 || { tail -5 gpurun_out/nr_gs_$gs.log; exit 1; }
  echo "runtime native GROUP_STREAMS=$gs $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nr_gs_$gs.log)"
done
timeout -k 10 200 python -u benchmarks/ppo_phase_probe.py > gpurun_out/nr_phase.log 2>&1 || { tail -5 gpurun_out/nr_phase.log; exit 1; }
tail -1 gpurun_out/nr_phase.log
