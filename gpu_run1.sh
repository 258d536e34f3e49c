set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_rllib_gpu.py tests/test_rllib_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_rl.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep -o '"value": [0-9.]*\|"kl": [0-9.]*\|"vf_loss": [0-9.]*\|"put_get_GBps": [0-9.]*' gpurun_out/bench.log
