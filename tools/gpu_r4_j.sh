# Round 4 (j): K21 rollout server phase timeline (workgroup-0 stamps) at 128 / 64 workgroups; K12 split+finalize A/B; fused bench.
set -o pipefail
mkdir -p gpurun_out
true

RMM_K12_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_runtime_gpu.py -m gpu -k "not fused_adam" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_j_k12.log 2>&1 || { tail -30 gpurun_out/pytest_j_k12.log; exit 1; }
echo "k12 split: $(tail -1 gpurun_out/pytest_j_k12.log)"
for w in 128 64; do
  RMM_ROLLOUT_SERVER=1 RMM_ROLLOUT_SERVER_PROF=1 RMM_ROLLOUT_SERVER_WGS=$w timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_j_$w.log 2>&1 || { tail -10 gpurun_out/probe_j_$w.log; exit 1; }
  echo "wgs=$w"; tail -2 gpurun_out/probe_j_$w.log
done
for v in 2 1 2 1; do
  RMM_K12_SPLIT=$v timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/bench_j_$v.log 2>&1 || { tail -5 gpurun_out/bench_j_$v.log; exit 1; }
  echo "K12_SPLIT=$v fused $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_j_$v.log)"
done
