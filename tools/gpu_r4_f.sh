# Round 4 (f): K10 forward bf16 half-image conv1 + float4 trunk reduce: kernel tests, phase timing, fused-loop bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 || { tail -40 gpurun_out/pytest_f.log; exit 1; }
tail -2 gpurun_out/pytest_f.log
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_f.json 2> gpurun_out/trunk_phases_f.err || { tail -5 gpurun_out/trunk_phases_f.err; exit 1; }
cat gpurun_out/trunk_phases_f.json
timeout -k 10 300 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/bench_f_fused.log 2>&1 || { tail -20 gpurun_out/bench_f_fused.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/bench_f_fused.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_f
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_f.log 2>&1 || { tail -5 gpurun_out/prof_f.log; exit 1; }
for f in $(find gpurun_out/prof_f -name "*kernel_stats.csv"); do python3 benchmarks/summarize_prof.py $f 14 > gpurun_out/prof_f_summary.txt; done
cat gpurun_out/prof_f_summary.txt | cut -c1-150
rm -f $(find gpurun_out/prof_f -name "*.db")
