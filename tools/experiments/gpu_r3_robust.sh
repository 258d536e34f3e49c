# Headline robustness on one box: default (native loop, polling) vs blocking wait vs Python loop, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
nproc; cat /proc/loadavg
for rep in 1 2 3; do
  for v in default nospin; do
    case $v in default) e="";; nospin) e="RMM_NATIVE_SPIN=0";; python) e="RMM_NO_NATIVE_ROLLOUT=1";; esac
    env $e timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/rb_$v.log 2>&1 || { tail -5 gpurun_out/rb_$v.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rb_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/rb_$v.log)"
  done
done
cat /proc/loadavg
