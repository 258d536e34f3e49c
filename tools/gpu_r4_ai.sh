# Round 4 (ai): full GPU suite + smoke + one default bench after the K16 change.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ai.log 2>&1 || { tail -40 gpurun_out/pytest_ai.log; exit 1; }
tail -2 gpurun_out/pytest_ai.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ai.log 2>&1 || { tail -20 gpurun_out/smoke_ai.log; exit 1; }
tail -1 gpurun_out/smoke_ai.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_ai.log 2>&1 || { tail -5 gpurun_out/bench_ai.log; exit 1; }
tail -1 gpurun_out/bench_ai.log
