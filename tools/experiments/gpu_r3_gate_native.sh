# Native rollout loop with / without the device step gate (step t+1 launched before step t's env step).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -q --timeout 200 --timeout-method thread -k "gate or native" > gpurun_out/gn_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/gn_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for gt in 1 0; do
    RMM_ROLLOUT_GATE=$gt timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/gn_${gt}.log 2>&1 || { tail -5 gpurun_out/gn_${gt}.log; exit 1; }
    echo "gate=$gt $(tail -1 gpurun_out/gn_${gt}.log)"
  done
done
for rep in 1 2; do
  for gt in 1 0; do
    RMM_ROLLOUT_GATE=$gt timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/gn_rt_$gt.log 2>&1 || { tail -5 gpurun_out/gn_rt_$gt.log; exit 1; }
    echo "runtime gate=$gt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gn_rt_$gt.log)"
  done
done
