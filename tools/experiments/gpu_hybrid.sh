# Hybrid (CPU env + GPU policy) rollout workers: GPU tests, then the runtime bench in hybrid mode.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "hybrid" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_hybrid.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_hybrid.log; [ $rc -eq 0 ] || { grep -n "^E \|Error" gpurun_out/pytest_hybrid.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --rollout hybrid --no-putget --no-fused --no-gpu-rollout > gpurun_out/bench_hybrid.log 2>&1 || { tail -30 gpurun_out/bench_hybrid.log; exit 1; }
tail -1 gpurun_out/bench_hybrid.log
