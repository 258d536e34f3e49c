# Round 4 (r): shared (zero-copy) weights through PPO with hybrid workers (test), then bench A/B x2 each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "shared_weights or hybrid_rollouts or recapture" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r.log | head; tail -3 gpurun_out/pytest_r.log; exit 1; }
tail -1 gpurun_out/pytest_r.log
for m in 1 0 1 0; do
  RMM_SHARED_WEIGHTS=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_r_$m.log 2>&1 || { grep -v "^frame" gpurun_out/bench_r_$m.log | tail -5; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_r_$m.log').read().strip().splitlines()[-1]); print('SHARED=$m', d['value'], d['ms_per_step'], d['config'].get('weights_sync'), d['last_stats']['learner_update_s'])"
done
