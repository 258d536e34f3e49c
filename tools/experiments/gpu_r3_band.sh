# K10 rollout band mode: GPU tests, isolated worker probe and runtime A/B vs the per-frame push.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/band_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/band_pytest.log; grep -E "FAILED|Error" gpurun_out/band_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  RMM_BAND_PUSH=$([ $v = 1 ] && echo 0 || echo 1) timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/band_p$v.log 2>&1 || { tail -5 gpurun_out/band_p$v.log; exit 1; }
  echo "NO_BAND=$v $(tail -1 gpurun_out/band_p$v.log)"
done
for rep in 1 2; do
  for v in 0 1; do
    RMM_BAND_PUSH=$([ $v = 1 ] && echo 0 || echo 1) timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/band_r$v.log 2>&1 || { tail -5 gpurun_out/band_r$v.log; exit 1; }
    echo "runtime NO_BAND=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/band_r$v.log)"
  done
done
