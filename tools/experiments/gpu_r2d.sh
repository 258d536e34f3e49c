# RLlib runtime GPU tests (hybrid / learner actors / multirank rehearsal) + the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_multirank.py tests/test_rllib_learner_actors.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r2d.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r2d.log; [ $rc -eq 0 ] || { grep -n "^E \|Error" gpurun_out/pytest_r2d.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
