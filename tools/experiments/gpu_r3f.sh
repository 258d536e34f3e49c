# LDS-staged coalesced partial stores in K10 backward: numerics + phase timings + fused loop.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_runtime_gpu.py -x -q -k "trunk or manual_step or fp32_reference" --timeout 120 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1 || { tail -30 gpurun_out/pytest_r3f.log; exit 1; }
tail -1 gpurun_out/pytest_r3f.log
timeout -k 10 200 python -u benchmarks/bench_trunk.py 2>&1 | grep '{'
echo "== fused loop"; timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget | cut -c100-200
