# Round 4 (ah): multi-workgroup K16 rows per workgroup (RMM_K16_WPW 4 / 2 / 1) at 50 rollout rows — tests,
# probe and runtime bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py -k "single_workgroup_advance" -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ah.log 2>&1 || { tail -30 gpurun_out/pytest_ah.log; exit 1; }
tail -2 gpurun_out/pytest_ah.log
for v in 1 4 2 1 4 2; do
  RMM_K16_WPW=$v timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_ah_$v.log 2>&1 || { tail -10 gpurun_out/probe_ah_$v.log; exit 1; }
  echo "WPW=$v probe: $(tail -1 gpurun_out/probe_ah_$v.log)"
done
for v in 1 4 1 4 1 4; do
  RMM_K16_WPW=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_ah_$v.log 2>&1 || { tail -5 gpurun_out/bench_ah_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ah_$v.log').read().strip().splitlines()[-1]); print('WPW=$v', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"
done
