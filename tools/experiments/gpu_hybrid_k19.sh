# K19 device frame stacks: GPU tests for the hybrid worker, the isolated worker probe, and the
# headline bench (hybrid mode only, no extra modes) — each step time-limited, chain stops on failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_runtime_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_runtime_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/hybrid_probe.log 2>&1 || { tail -20 gpurun_out/hybrid_probe.log; exit 1; }
cat gpurun_out/hybrid_probe.log | tail -6
timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_k19.log 2>&1 || { tail -30 gpurun_out/bench_k19.log; exit 1; }
tail -1 gpurun_out/bench_k19.log
