# Round 4 (s): shared weights on by default — runtime / weight-sync GPU tests, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rllib_runtime_gpu.py tests/test_rllib_weights_sync.py tests/test_rllib_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_s.log | tail -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s.log 2>&1 || { tail -5 gpurun_out/smoke_s.log; exit 1; }
tail -1 gpurun_out/smoke_s.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_s.log 2>&1 || { tail -5 gpurun_out/bench_s.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_s.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','runtime_gpu_rollout_samples_per_s','runtime_cpu_rollout_samples_per_s','runtime_fp32_samples_per_s','fused_loop_samples_per_s','put_get_GBps')}, d['config'].get('weights_sync'))"
