# Round 4 (z): rollout step completion through K16's host word (RMM_ROLLOUT_SEQ=1) vs events: parity, probe, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_gpu.py -k "direct_launch or heads_sample or recapture" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_z.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_z.log | head; tail -3 gpurun_out/pytest_z.log; exit 1; }
tail -1 gpurun_out/pytest_z.log
for m in 1 0 1 0; do
  RMM_ROLLOUT_SEQ=$m timeout -k 10 120 python -u benchmarks/native_rollout_probe.py > gpurun_out/probe_z_$m.log 2>&1 || { tail -5 gpurun_out/probe_z_$m.log; exit 1; }
  echo "SEQ=$m $(grep us_per_step gpurun_out/probe_z_$m.log | tail -1)"
done
for m in 1 0; do
  RMM_ROLLOUT_SEQ=$m timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-putget --no-fused --no-gpu-rollout --no-fp32 > gpurun_out/bench_z_$m.log 2>&1 || { tail -5 gpurun_out/bench_z_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_z_$m.log').read().strip().splitlines()[-1]); print('SEQ=$m', d['value'], d['ms_per_step'])"
done
