# GPU object store check: its GPU tests + the standalone store benchmark (1 and 16 GiB puts).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_objects.py tests/test_gpu_store_native.py tests/test_gpu_object_identity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_objstore.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_objstore.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/gpu_object_store_bench.py --sizes 1,4,16 > gpurun_out/objstore_bench.log 2>&1 || { tail -30 gpurun_out/objstore_bench.log; exit 1; }
tail -1 gpurun_out/objstore_bench.log
