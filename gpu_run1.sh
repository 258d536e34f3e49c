set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppo -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1 && echo PROF_OK
find gpurun_out/prof_ppo -name "*.db" -o -name "*stats*" | head
for f in $(find gpurun_out/prof_ppo -name "*kernel_stats.csv" -o -name "*results.db"); do python3 benchmarks/summarize_prof.py $f 45 > gpurun_out/prof_ppo_summary.txt; done
rm -f $(find gpurun_out/prof_ppo -name "*.db") 
tail -3 gpurun_out/prof_bench.log
