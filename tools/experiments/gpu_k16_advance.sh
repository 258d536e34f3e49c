# K16 step-advance (no separate counter-increment kernel per rollout step): K16 GPU tests, hybrid
# worker tests, the isolated worker probe and the headline bench — each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_gpu.py -x -v --timeout 120 --timeout-method thread -k "heads_sample" > gpurun_out/pytest_k16.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_k16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_runtime_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_runtime_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/hybrid_probe.log 2>&1 || { tail -20 gpurun_out/hybrid_probe.log; exit 1; }
tail -6 gpurun_out/hybrid_probe.log
timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_k16adv.log 2>&1 || { tail -30 gpurun_out/bench_k16adv.log; exit 1; }
tail -1 gpurun_out/bench_k16adv.log
