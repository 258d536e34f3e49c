# Kernel trace of the fused PPO loop (per-kernel times and gaps of the SGD-step graph) + pipelined-publish A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sgd_prof -o sgd -- python -u bench.py --mode fused --steps 5 --warmup 2 > gpurun_out/sgd_prof.log 2>&1 || { tail -5 gpurun_out/sgd_prof.log; exit 1; }
find gpurun_out/sgd_prof -name "*kernel_trace.csv" | head -3
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/pp_$rep.log 2>&1 || { tail -5 gpurun_out/pp_$rep.log; exit 1; }
  echo "runtime pipelined publish $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pp_$rep.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/pp_$rep.log)"
done
