# Full GPU suite + smoke + headline bench at HEAD (each step time-limited, stop at first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r3.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_r3.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3.log 2>&1 || { tail -20 gpurun_out/smoke_r3.log; exit 1; }
tail -1 gpurun_out/smoke_r3.log | cut -c1-200
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3.log 2>&1 || { tail -20 gpurun_out/bench_r3.log; exit 1; }
grep '"metric"' gpurun_out/bench_r3.log | tail -1
