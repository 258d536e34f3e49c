# Round 4 (af): final validation after the sample prefetch default — GPU suite, smoke, default bench x2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_af.log 2>&1 || { tail -40 gpurun_out/pytest_af.log; exit 1; }
tail -3 gpurun_out/pytest_af.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_af.log 2>&1 || { tail -20 gpurun_out/smoke_af.log; exit 1; }
tail -1 gpurun_out/smoke_af.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > gpurun_out/bench_af_$i.log 2>&1 || { tail -5 gpurun_out/bench_af_$i.log; exit 1; }
  tail -1 gpurun_out/bench_af_$i.log
done
