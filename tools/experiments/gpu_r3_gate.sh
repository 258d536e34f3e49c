# rollout step gate: tests, probe, runtime bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gate_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gate_tests.log; grep -E "FAILED|Error" gpurun_out/gate_tests.log | head; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  RMM_ROLLOUT_GATE=$v timeout -k 10 240 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/gate_probe_$v.log 2>&1 || { tail -5 gpurun_out/gate_probe_$v.log; exit 1; }
  echo "GATE=$v"; grep "n=" gpurun_out/gate_probe_$v.log | grep "graphs=True"
done
for i in 1 2 3; do for v in 0 1; do
  RMM_ROLLOUT_GATE=$v timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/gate_rt_$v.log 2>&1 || { tail -5 gpurun_out/gate_rt_$v.log; exit 1; }
  echo "runtime GATE=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gate_rt_$v.log)"
  RMM_ROLLOUT_DOUBLE_BUFFER=0 RMM_ROLLOUT_GATE=$v timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/gate_rt1_$v.log 2>&1 || { tail -5 gpurun_out/gate_rt1_$v.log; exit 1; }
  echo "runtime single-group GATE=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gate_rt1_$v.log)"
done; done
