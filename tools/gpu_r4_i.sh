# Round 4 (i): K21 persistent rollout server: parity test vs the graph loop, isolated worker probe, runtime bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "rollout_server or native_rollout_loop" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_i.log 2>&1 || { tail -40 gpurun_out/pytest_i.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_i.log | tail -5
for v in 1 0 1 0; do
  RMM_ROLLOUT_SERVER=$v timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_$v.log 2>&1 || { tail -10 gpurun_out/probe_$v.log; exit 1; }
  echo "server=$v $(tail -1 gpurun_out/probe_$v.log)"
done
for v in 1 0; do
  RMM_ROLLOUT_SERVER=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-gpu-rollout > gpurun_out/bench_i_$v.log 2>&1 || { tail -10 gpurun_out/bench_i_$v.log; exit 1; }
  echo "server=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_i_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/bench_i_$v.log)"
done
