# round-6 GPU check: the GPU tests (optionally a subset: $1 = files / node ids) then a 1-GPU rehearsal of
# the 4-learner data-parallel bench (PeerComm + ZeRO-1 on one device, replica identity reported)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS=${1:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r6.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 4 --same-device --steps 5 --warmup 2 --no-putget > gpurun_out/bench_same4_r6.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_same4_r6.log
exit $rc
