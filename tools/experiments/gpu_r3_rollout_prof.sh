# kernel trace of the hybrid rollout worker (2 env groups, graphs): per-kernel stats
set -o pipefail
mkdir -p gpurun_out/rollprof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rollprof -o roll -- python3 benchmarks/hybrid_step_trace.py graph double > gpurun_out/rollprof/run.log 2>&1 || { tail -20 gpurun_out/rollprof/run.log; exit 1; }
find gpurun_out/rollprof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/rollprof -name "*kernel_stats.csv" | head -1); python3 benchmarks/summarize_prof.py "$f" 20; rm -f $(find gpurun_out/rollprof -name "*.db")
