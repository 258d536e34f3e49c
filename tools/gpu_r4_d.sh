# Round 4 (d): K10 phase attribution (graph-replayed), zero-copy weights fault hunt, OOC GPU shuffle.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_d.json 2> gpurun_out/trunk_phases_d.err || { tail -5 gpurun_out/trunk_phases_d.err; exit 1; }
cat gpurun_out/trunk_phases_d.json
for m in none plain store store_ingest; do
  timeout -k 10 240 python3 -u tools/experiments/zero_copy_repro.py $m > gpurun_out/zc_$m.log 2>&1
  rc=$?
  echo "zero_copy $m rc=$rc"; grep -E '^\{' gpurun_out/zc_$m.log | tail -2
  [ $rc -eq 0 ] || { tail -15 gpurun_out/zc_$m.log; exit 1; }
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_shuffle.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_shuffle.log 2>&1 || { tail -30 gpurun_out/pytest_shuffle.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_shuffle.log | tail -5
timeout -k 10 600 python -u benchmarks/gpu_shuffle_ooc.py --quota-gb 8 --factor 4 --rounds 16 --partitions 8 > gpurun_out/shuffle_ooc.log 2>&1 || { tail -30 gpurun_out/shuffle_ooc.log; exit 1; }
tail -1 gpurun_out/shuffle_ooc.log
