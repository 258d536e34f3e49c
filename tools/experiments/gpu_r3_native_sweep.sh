# Native rollout loop: layout sweep (workers per learner x double-buffered env groups), runtime PPO ms/iter.
set -o pipefail
mkdir -p gpurun_out
run() {  # $1 label, $2 workers per learner, $3 double buffer, $4 native (1/0)
  local nat=""; [ "$4" = 0 ] && nat=1
  RMM_ROLLOUT_DOUBLE_BUFFER=$3 RMM_NO_NATIVE_ROLLOUT=$nat timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 \
    --no-putget --no-fused --no-gpu-rollout --workers-per-learner $2 > gpurun_out/sw_$1.log 2>&1 || { tail -5 gpurun_out/sw_$1.log; return 1; }
  echo "$1 w=$2 db=$3 native=$4 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_$1.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/sw_$1.log)"
}
for rep in 1 2; do
  run a$rep 2 1 1 || exit 1
  run b$rep 2 0 1 || exit 1
  run c$rep 1 0 1 || exit 1
  run d$rep 1 1 1 || exit 1
  run e$rep 5 0 1 || exit 1
  run f$rep 2 0 0 || exit 1
done
