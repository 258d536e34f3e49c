# Per-env-group streams in the hybrid rollout worker: hybrid GPU tests, worker probe (shared vs
# per-group streams) and the headline bench at 2 vs 1 HW queues per rollout worker — each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_runtime_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_runtime_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/probe_gs.log 2>&1 || { tail -20 gpurun_out/probe_gs.log; exit 1; }
tail -4 gpurun_out/probe_gs.log
timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_gs_q2.log 2>&1 || { tail -30 gpurun_out/bench_gs_q2.log; exit 1; }
RMM_ROLLOUT_HW_QUEUES=1 timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_gs_q1.log 2>&1 || { tail -30 gpurun_out/bench_gs_q1.log; exit 1; }
RMM_GROUP_STREAMS=0 RMM_ROLLOUT_HW_QUEUES=1 timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_nogs_q1.log 2>&1 || { tail -30 gpurun_out/bench_nogs_q1.log; exit 1; }
for f in bench_gs_q2 bench_gs_q1 bench_nogs_q1; do python -c "import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"; done
