# Round 4 (n): K10 conv1-weight race fix + staging, K6 folded into the trunk-reduce launch (tail Adam):
# kernel + learner tests, then the fused loop A/B (RMM_TAIL_ADAM=0/1) and trunk phase timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py -k "tail_adam or parity or graph_matches" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 || { grep -E "FAILED|Error|assert|Mismatch|Greatest" gpurun_out/pytest_n.log | head -30; tail -3 gpurun_out/pytest_n.log; exit 1; }
tail -1 gpurun_out/pytest_n.log
for t in 0 1 0 1; do
  RMM_TAIL_ADAM=$t timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/fused_n_$t.log 2>&1 || { tail -5 gpurun_out/fused_n_$t.log; exit 1; }
  echo "TAIL_ADAM=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fused_n_$t.log)"
done
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_n.json 2> gpurun_out/trunk_phases_n.err || { tail -5 gpurun_out/trunk_phases_n.err; exit 1; }
cat gpurun_out/trunk_phases_n.json
