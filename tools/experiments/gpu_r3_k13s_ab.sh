# K13s in the learner / rollout: GPU tests, then fused loop + runtime bench A/B (RMM_NO_K13S=1 = K13)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py tests/test_hip_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/k13s_tests.log 2>&1; rc=$?; tail -3 gpurun_out/k13s_tests.log; grep -E "FAILED|Error" gpurun_out/k13s_tests.log | head; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export RMM_NO_K13S=1; else unset RMM_NO_K13S; fi
  timeout -k 10 300 python -u bench.py --mode fused --steps 20 --warmup 5 > gpurun_out/k13s_fused_$v.log 2>&1 || { tail -5 gpurun_out/k13s_fused_$v.log; exit 1; }
  echo "fused NO_K13S=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k13s_fused_$v.log)"
done
for v in 1 0; do
  if [ $v = 1 ]; then export RMM_NO_K13S=1; else unset RMM_NO_K13S; fi
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/k13s_rt_$v.log 2>&1 || { tail -5 gpurun_out/k13s_rt_$v.log; exit 1; }
  echo "runtime NO_K13S=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k13s_rt_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/k13s_rt_$v.log)"
done
