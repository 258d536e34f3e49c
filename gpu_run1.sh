set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shuffle.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_shuffle.log 2>&1; rc=$?; echo "shuffle rc=$rc"; tail -12 gpurun_out/pytest_shuffle.log
