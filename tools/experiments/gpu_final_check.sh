# End-of-session GPU check at HEAD: full GPU suite, smoke(), default bench — each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -30 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
