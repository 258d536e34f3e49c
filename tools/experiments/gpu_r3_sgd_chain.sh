# SGD steps chained in one HIP graph (world of one) vs one graph per step (RMM_SGD_CHAIN=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/chain_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/chain_pytest.log; grep -E "FAILED|Error" gpurun_out/chain_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in 1 25 100; do
    RMM_SGD_CHAIN=$c timeout -k 10 120 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget > gpurun_out/chain_f_$c.log 2>&1 || { tail -5 gpurun_out/chain_f_$c.log; exit 1; }
    echo "fused chain=$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/chain_f_$c.log)"
  done
done
for rep in 1 2; do
  for c in 1 25; do
    RMM_SGD_CHAIN=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/chain_r_$c.log 2>&1 || { tail -5 gpurun_out/chain_r_$c.log; exit 1; }
    echo "runtime chain=$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/chain_r_$c.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/chain_r_$c.log)"
  done
done
