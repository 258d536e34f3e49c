# Round 4 (h): K12 row split: kernel tests (incl. graph == eager, manual == autograd), fused-loop + runtime bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py tests/test_rllib_precision_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1 || { tail -40 gpurun_out/pytest_h.log; exit 1; }
tail -1 gpurun_out/pytest_h.log
for v in 2 0 2 0; do
  RMM_K12_SPLIT=$v timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/k12_$v.log 2>&1 || { tail -5 gpurun_out/k12_$v.log; exit 1; }
  echo "K12_SPLIT=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k12_$v.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_h
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_h.log 2>&1 || { tail -5 gpurun_out/prof_h.log; exit 1; }
for f in $(find gpurun_out/prof_h -name "*kernel_stats.csv"); do python3 benchmarks/summarize_prof.py $f 12 > gpurun_out/prof_h_summary.txt; done
cat gpurun_out/prof_h_summary.txt | cut -c1-150
rm -f $(find gpurun_out/prof_h -name "*.db")
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-putget --no-gpu-rollout > gpurun_out/bench_h.log 2>&1 || { tail -20 gpurun_out/bench_h.log; exit 1; }
grep '"metric"' gpurun_out/bench_h.log | cut -c1-400
