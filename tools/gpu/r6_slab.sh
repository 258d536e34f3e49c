# round-6: K15x loss statistics in a per-workgroup slab (no same-word atomics): tests, fused-loop trace, bench,
# then the multi-rank part 2 (tools/gpu/r6_multirank3.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_precision_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_slab.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_slab -o slab -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > gpurun_out/prof_slab.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget > gpurun_out/bench_slab.log 2>&1 || exit $?
bash tools/gpu/r6_multirank3.sh
