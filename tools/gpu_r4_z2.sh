# Round 4 (z2): runtime bench A/B of the rollout completion word, interleaved x3.
set -o pipefail
mkdir -p gpurun_out
for m in 1 0 1 0 1 0; do
  RMM_ROLLOUT_SEQ=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_z2_$m.log 2>&1 || { tail -5 gpurun_out/bench_z2_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_z2_$m.log').read().strip().splitlines()[-1]); print('SEQ=$m', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"
done
