# round-6: trunk reduce with the Adam state prefetched and one batch of partial loads; probe: K15x without its
# loss-statistics atomics (RMM_PROBE_K15_NOACC=1, stats wrong: timing only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_precision_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_reduce.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_red -o red -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > gpurun_out/prof_red.log 2>&1 || exit $?
RMM_PROBE_K15_NOACC=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_noacc -o noacc -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > gpurun_out/prof_noacc.log 2>&1 || exit $?
bash tools/gpu/r6_multirank3.sh
