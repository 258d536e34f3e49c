# Round 4 (ae): sample prefetch behind the update (RMM_PREFETCH_SAMPLE) — shared-weights test, then
# runtime bench A/B interleaved x3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "shared_weights" -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ae.log 2>&1 || { tail -30 gpurun_out/pytest_ae.log; exit 1; }
tail -2 gpurun_out/pytest_ae.log
for m in 1 0 1 0 1 0; do
  RMM_PREFETCH_SAMPLE=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_ae_$m.log 2>&1 || { tail -5 gpurun_out/bench_ae_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ae_$m.log').read().strip().splitlines()[-1]); print('PREFETCH=$m', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"
done
