# Kernel-trace profile of the headline bench (hybrid rollouts: CPU env + GPU policy with K19 frame
# stacks, learner actor), per-process kernel stats summarised.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_hy
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hy -o run -- python3 bench.py --no-putget --no-fused --no-gpu-rollout --steps 5 --warmup 2 > gpurun_out/prof_hy.log 2>&1 || { tail -20 gpurun_out/prof_hy.log; exit 1; }
for f in $(find gpurun_out/prof_hy -name "*kernel_stats.csv"); do echo "## $f" >> gpurun_out/prof_hy_summary.txt; python3 benchmarks/summarize_prof.py $f 25 >> gpurun_out/prof_hy_summary.txt; done
rm -f $(find gpurun_out/prof_hy -name "*.db") $(find gpurun_out/prof_hy -name "*kernel_trace.csv")
head -80 gpurun_out/prof_hy_summary.txt
tail -1 gpurun_out/prof_hy.log | cut -c1-300
