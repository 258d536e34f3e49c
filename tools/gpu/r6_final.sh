# round-6 check of the tree: the GPU suite, smoke(), and the driver's bench command (twice)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_final.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py >> gpurun_out/bench_final.log 2>&1 || exit $?
