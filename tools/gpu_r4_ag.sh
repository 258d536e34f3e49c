# Round 4 (ag): one-workgroup K16 for 33-64 rollout rows (4 preloaded rows per wave) — K16 tests, rollout
# parity tests, then probe + runtime bench A/B against the multi-workgroup K16 (RMM_K16_ONE_WG_ROWS=32).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py -k "single_workgroup_advance or heads_sample or direct_launch_matches or shared_weights" -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ag.log 2>&1 || { tail -30 gpurun_out/pytest_ag.log; exit 1; }
tail -2 gpurun_out/pytest_ag.log
for v in 64 32 64 32; do
  RMM_K16_ONE_WG_ROWS=$v timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_ag_$v.log 2>&1 || { tail -10 gpurun_out/probe_ag_$v.log; exit 1; }
  echo "ROWS=$v probe: $(tail -2 gpurun_out/probe_ag_$v.log | tr '\n' ' ')"
done
for v in 64 32 64 32 64 32; do
  RMM_K16_ONE_WG_ROWS=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_ag_$v.log 2>&1 || { tail -5 gpurun_out/bench_ag_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ag_$v.log').read().strip().splitlines()[-1]); print('ROWS=$v', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"
done
