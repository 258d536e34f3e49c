# Round 4 (q): the hybrid worker's recapture fix (warm-up steps at row 0, counters restored), then the shared
# (zero-copy) weights runtime bench that faulted in rounds 3/4, then an A/B against the default weight publish.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "hybrid" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_q.log | head; tail -3 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
RMM_SHARED_WEIGHTS=1 RMM_SHARED_WEIGHTS_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_q_shared.log 2>&1 || { grep -v "^frame" gpurun_out/bench_q_shared.log | tail -8; exit 1; }
tail -1 gpurun_out/bench_q_shared.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_q_plain.log 2>&1 || { tail -5 gpurun_out/bench_q_plain.log; exit 1; }
tail -1 gpurun_out/bench_q_plain.log | cut -c1-200
