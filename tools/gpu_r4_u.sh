# Round 4 (u): K16 loads its hidden partials / step counters before the Wh staging. K16 + rollout tests, probe x3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py tests/test_hip_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_u.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_u.log | head; tail -3 gpurun_out/pytest_u.log; exit 1; }
tail -1 gpurun_out/pytest_u.log
for i in 1 2 3; do
  timeout -k 10 120 python -u benchmarks/native_rollout_probe.py > gpurun_out/probe_u_$i.log 2>&1 || { tail -5 gpurun_out/probe_u_$i.log; exit 1; }
  grep us_per_step gpurun_out/probe_u_$i.log | tail -1
done
