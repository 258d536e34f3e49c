# Learner -> GPU rollout worker weights through HBM: runtime GPU tests, phase probe, headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rccl_native.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1 || { tail -40 gpurun_out/pytest_r3e.log; exit 1; }
tail -1 gpurun_out/pytest_r3e.log
timeout -k 10 300 python -u benchmarks/ppo_phase_probe.py 2>&1 | grep '{'
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/bench_r3e.log 2>&1 || { tail -20 gpurun_out/bench_r3e.log; exit 1; }
grep '"metric"' gpurun_out/bench_r3e.log | cut -c1-330
