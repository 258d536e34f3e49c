# Kernel trace + stats of the runtime PPO bench at HEAD (learner actor + hybrid rollout worker).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof -o fp -- python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout > gpurun_out/fprof.log 2>&1 || { tail -5 gpurun_out/fprof.log; exit 1; }
grep '"metric"' gpurun_out/fprof.log | cut -c1-300
find gpurun_out/fprof -name "*kernel_stats.csv" | head -3
