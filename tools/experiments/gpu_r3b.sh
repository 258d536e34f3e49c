# Native RCCL communicator on one GPU (2 ranks, distinct host ids), PPO learner actors with the
# all-reduces inside the SGD-step graph, then the 2-learner bench rehearsal over RCCL.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rccl_native.py tests/test_gpu_objects.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_rccl.log 2>&1 || { tail -60 gpurun_out/pytest_rccl.log; exit 1; }
tail -3 gpurun_out/pytest_rccl.log
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend nccl --steps 3 --warmup 1 --no-putget > gpurun_out/rehearse_rccl_2learners.log 2>&1 || { tail -40 gpurun_out/rehearse_rccl_2learners.log; exit 1; }
tail -1 gpurun_out/rehearse_rccl_2learners.log | cut -c1-900
