# Round 4 (x): K13s deeper load batches (D k-steps per round trip). Dense/rollout tests, fused loop x2, kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py tests/test_hip_kernels.py tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_x.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_x.log | head; tail -3 gpurun_out/pytest_x.log; exit 1; }
tail -1 gpurun_out/pytest_x.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/fused_x_$i.log 2>&1 || { tail -5 gpurun_out/fused_x_$i.log; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fused_x_$i.log)"
done
timeout -k 10 120 python -u benchmarks/native_rollout_probe.py > gpurun_out/probe_x.log 2>&1 || { tail -5 gpurun_out/probe_x.log; exit 1; }
grep us_per_step gpurun_out/probe_x.log | tail -1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_x
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_x.log 2>&1 || { tail -5 gpurun_out/prof_x.log; exit 1; }
f=$(find gpurun_out/prof_x -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-5
cd "$GRAFT_REPO_ROOT"
for v in 0 1 2 3; do
  RMM_COPY_VARIANT=$v timeout -k 10 120 python -u benchmarks/bench_copy.py 4 > gpurun_out/copy_x_$v.log 2>&1 || { tail -5 gpurun_out/copy_x_$v.log; exit 1; }
  tail -1 gpurun_out/copy_x_$v.log
done
