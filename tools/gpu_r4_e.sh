# Round 4 (e): K10 phase attribution (graph-replayed), OOC GPU shuffle, then the zero-copy weights runtime experiment (last: may fault).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_e.json 2> gpurun_out/trunk_phases_e.err || { tail -5 gpurun_out/trunk_phases_e.err; exit 1; }
cat gpurun_out/trunk_phases_e.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_shuffle.py tests/test_rllib_dreamer.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_shuffle.log 2>&1 || { tail -30 gpurun_out/pytest_shuffle.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed|'GBps'" gpurun_out/pytest_shuffle.log | tail -6 | cut -c1-1500
timeout -k 10 600 python -u benchmarks/gpu_shuffle_ooc.py --quota-gb 8 --factor 4 --rounds 16 --partitions 16 > gpurun_out/shuffle_ooc.log 2>&1 || { tail -30 gpurun_out/shuffle_ooc.log; exit 1; }
tail -1 gpurun_out/shuffle_ooc.log | cut -c1-2000
RMM_SHARED_WEIGHTS=1 RMM_SHARED_WEIGHTS_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-putget --no-fused --no-gpu-rollout > gpurun_out/shw.log 2>&1
rc=$?
echo "shared-weights rc=$rc"
grep -E "shared-weights|fault|Fault|Error|error" gpurun_out/shw.log | head -20
grep -o '"ms_per_step": [0-9.]*' gpurun_out/shw.log
exit $rc
