# Hybrid rollout layout sweep: rollout workers per learner GPU (envs per worker = 5000 / (100 * w)).
set -o pipefail
mkdir -p gpurun_out
for w in 1 2 5; do
  timeout -k 10 240 python -u bench.py --rollout hybrid --workers-per-learner $w --no-putget --no-fused --no-gpu-rollout > gpurun_out/bench_hybrid_w$w.log 2>&1 || { tail -30 gpurun_out/bench_hybrid_w$w.log; exit 1; }
  echo "w=$w $(tail -1 gpurun_out/bench_hybrid_w$w.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["last_stats"]["learner_update_s"])')"
done
