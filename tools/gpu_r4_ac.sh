set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "manual_step or fused_adam" -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ac.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_ac.log; exit $rc
