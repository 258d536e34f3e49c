# hybrid rollout layout A/B on the runtime bench: double buffer on/off x workers per learner
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env, args
  timeout -k 10 400 env $2 python -u bench.py --steps 30 --warmup 5 --no-putget --no-fused --no-gpu-rollout $3 > gpurun_out/lay_$1.log 2>&1 || { tail -5 gpurun_out/lay_$1.log; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lay_$1.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/lay_$1.log)"
}
for i in 1 2; do
run w2_dbl "RMM_ROLLOUT_DOUBLE_BUFFER=1" ""
run w2_single "RMM_ROLLOUT_DOUBLE_BUFFER=0" ""
run w5_single "RMM_ROLLOUT_DOUBLE_BUFFER=0" "--workers-per-learner 5"
run w5_dbl "RMM_ROLLOUT_DOUBLE_BUFFER=1" "--workers-per-learner 5"
run w10_single "RMM_ROLLOUT_DOUBLE_BUFFER=0" "--workers-per-learner 10"
done
