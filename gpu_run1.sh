set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "trunk or fused" > gpurun_out/pytest_trunk.log 2>&1; rc=$?; echo "trunk rc=$rc"; tail -25 gpurun_out/pytest_trunk.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1; rc=$?; echo "rl rc=$rc"; tail -5 gpurun_out/pytest_rl.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --breakdown > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -2 gpurun_out/bench.log
