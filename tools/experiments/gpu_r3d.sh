# Multi-rank learner default = one same-stream all-reduce between two graphs: RCCL + gloo multirank
# tests, then the 2-learner RCCL rehearsal bench (compare 141.7 ms/iter with the fork path).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rccl_native.py tests/test_rllib_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1 || { tail -40 gpurun_out/pytest_r3d.log; exit 1; }
grep -E "PASSED|SKIPPED|passed" gpurun_out/pytest_r3d.log | tail -12
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend nccl --steps 3 --warmup 1 --no-putget > gpurun_out/rehearse_rccl_2learners_b.log 2>&1 || { tail -40 gpurun_out/rehearse_rccl_2learners_b.log; exit 1; }
tail -1 gpurun_out/rehearse_rccl_2learners_b.log | cut -c1-300
grep -o '"learner_update_s": [0-9.]*\|"learner_update_s_max": [0-9.]*' gpurun_out/rehearse_rccl_2learners_b.log
