set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_dense.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_ppo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppo -o run -- python3 bench.py --steps 5 --warmup 2 --no-putget > gpurun_out/prof_bench.log 2>&1 && echo PROF_OK
for f in $(find gpurun_out/prof_ppo -name "*kernel_stats.csv" -o -name "*results.db"); do python3 benchmarks/summarize_prof.py $f 40 > gpurun_out/prof_ppo_summary.txt; done
rm -f $(find gpurun_out/prof_ppo -name "*.db")
head -18 gpurun_out/prof_ppo_summary.txt; grep -o '"value": [0-9.]*' gpurun_out/prof_bench.log
