set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "trunk or fused" > gpurun_out/pytest_trunk.log 2>&1; rc=$?; echo "trunk rc=$rc"; tail -3 gpurun_out/pytest_trunk.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/bench_trunk.py > gpurun_out/bench_trunk.log 2>&1; echo "bt rc=$?"; cat gpurun_out/bench_trunk.log | tail -1
