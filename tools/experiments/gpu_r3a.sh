# Round 3 first GPU call: RCCL with 2 ranks on one GPU (distinct NCCL_HOSTID per rank), then the
# new GPU-object leak regression test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rccl_same_gpu_probe.py 2 > gpurun_out/rccl_probe.log 2>&1; rc=$?
tail -20 gpurun_out/rccl_probe.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_objects.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpuobj.log 2>&1 || { tail -30 gpurun_out/pytest_gpuobj.log; exit 1; }
tail -3 gpurun_out/pytest_gpuobj.log
