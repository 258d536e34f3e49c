# Round 4 (l): K10 prologue — weight loads issued as one batch ahead of the frame loads / LDS zeroing,
# bwd h1 prefetched with the next frame. Tests, phase timing, fused-loop bench, runtime bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 || { tail -40 gpurun_out/pytest_l.log; exit 1; }
tail -1 gpurun_out/pytest_l.log
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_l.json 2> gpurun_out/trunk_phases_l.err || { tail -5 gpurun_out/trunk_phases_l.err; exit 1; }
cat gpurun_out/trunk_phases_l.json
timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/fused_l.log 2>&1 || { tail -5 gpurun_out/fused_l.log; exit 1; }
tail -1 gpurun_out/fused_l.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_l.log 2>&1 || { tail -5 gpurun_out/bench_l.log; exit 1; }
tail -1 gpurun_out/bench_l.log
