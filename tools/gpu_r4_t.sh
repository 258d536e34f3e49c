# Round 4 (t): native rollout loop with direct kernel launches per step (RMM_ROLLOUT_DIRECT=1) vs graph launches:
# parity test, rollout probe A/B, runtime bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "direct_launch or recapture" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_t.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_t.log | head; tail -3 gpurun_out/pytest_t.log; exit 1; }
tail -1 gpurun_out/pytest_t.log
for m in 1 0 1 0; do
  RMM_ROLLOUT_DIRECT=$m timeout -k 10 120 python -u benchmarks/native_rollout_probe.py > gpurun_out/probe_t_$m.log 2>&1 || { tail -5 gpurun_out/probe_t_$m.log; exit 1; }
  echo "DIRECT=$m $(grep us_per_step gpurun_out/probe_t_$m.log | tail -1)"
done
for m in 1 0; do
  RMM_ROLLOUT_DIRECT=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_t_$m.log 2>&1 || { tail -5 gpurun_out/bench_t_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_t_$m.log').read().strip().splitlines()[-1]); print('DIRECT=$m', d['value'], d['ms_per_step'])"
done
