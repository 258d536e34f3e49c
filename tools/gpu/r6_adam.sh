# round-6: Adam / ZeRO-1 loads batched (tail Adam, K6, split finalize, peer ZeRO-1): their GPU tests, a fused-loop
# kernel trace, the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_precision_gpu.py tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py tests/test_peer_allreduce.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_adam.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_fused -o fused -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > gpurun_out/prof_fused.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget > gpurun_out/bench_adam.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget >> gpurun_out/bench_adam.log 2>&1 || exit $?
