# Round 4 (m): K10 multi-frame / determinism check after the prologue change, then the eager-vs-graph test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k "trunk" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_m1.log 2>&1; echo "rc=$?"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_m1.log | head -30
timeout -k 10 300 python -u -m pytest tests/test_rllib_gpu.py -k "graph_matches_eager" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_m2.log 2>&1; echo "rc=$?"; grep -E "PASSED|FAILED|Mismatch|Greatest" gpurun_out/pytest_m2.log | head
