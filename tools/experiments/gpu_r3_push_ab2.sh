# runtime bench A/B (old = separate K19 + multi-workgroup K16), alternating, 5 runs each
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
for v in old new; do
  if [ $v = old ]; then export RMM_NO_FOLD_PUSH=1 RMM_K16_MULTI=1; else unset RMM_NO_FOLD_PUSH RMM_K16_MULTI; fi
  timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/push2_rt_$v.log 2>&1 || { tail -5 gpurun_out/push2_rt_$v.log; exit 1; }
  echo "runtime $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/push2_rt_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/push2_rt_$v.log)"
done
done
