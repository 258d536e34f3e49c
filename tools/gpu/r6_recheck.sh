# round-6 re-entry check: the GPU tests, the driver's 1-GPU bench, and a kernel-stats profile of the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r6.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r6.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py >> gpurun_out/bench_r6.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_prof.log 2>&1 || exit $?
find gpurun_out/prof_bench -name "*.csv" ! -name "*stats*" -delete
exit 0
