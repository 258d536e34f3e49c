# round-6: K15x / K16x with their loads batched (tests vs fp64 / torch fp32, rollout parity), a kernel trace of the
# bench, the bench itself, then the multi-rank rehearsals (tools/gpu/r6_multirank2.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_precision_gpu.py tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_heads.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget > gpurun_out/bench_heads.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_heads -o heads -- python3 -u bench.py --steps 5 --warmup 2 --no-putget --no-fused > gpurun_out/prof_heads.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/native_rollout_probe.py 50 100 1 fp32 > gpurun_out/rollout_heads.log 2>&1 || exit $?
bash tools/gpu/r6_multirank2.sh
