# Round 4 (o): full GPU suite, smoke and the default bench after the K10 race fix + tail Adam.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_o.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_o.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_o.log 2>&1 || { tail -5 gpurun_out/smoke_o.log; exit 1; }
tail -1 gpurun_out/smoke_o.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_o.log 2>&1 || { tail -5 gpurun_out/bench_o.log; exit 1; }
tail -1 gpurun_out/bench_o.log
