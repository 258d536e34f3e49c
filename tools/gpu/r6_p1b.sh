# round-6: probe pointer as a kernel argument (the device-global one drained vmcnt at each site), frame source
# rows prefetched one frame ahead, conv2 bwd P1b reads hoisted: tests, phase probe, fused trace, bench x2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_precision_gpu.py tests/test_rllib_runtime_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_p1b.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/x3_phase_probe.py > gpurun_out/x3_phase_probe_p1b.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_p1b -o p1b -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > gpurun_out/prof_p1b.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget > gpurun_out/bench_p1b.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-putget >> gpurun_out/bench_p1b.log 2>&1 || exit $?
