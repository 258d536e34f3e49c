# A/B on one box: K16 step-advance vs the separate counter-increment kernel (RMM_NO_K16_ADVANCE=1):
# isolated hybrid worker probe and the headline bench for each — each step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/probe_adv.log 2>&1 || { tail -20 gpurun_out/probe_adv.log; exit 1; }
RMM_NO_K16_ADVANCE=1 timeout -k 10 200 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/probe_noadv.log 2>&1 || { tail -20 gpurun_out/probe_noadv.log; exit 1; }
echo "== advance"; tail -3 gpurun_out/probe_adv.log; echo "== no advance"; tail -3 gpurun_out/probe_noadv.log
timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_adv.log 2>&1 || { tail -30 gpurun_out/bench_adv.log; exit 1; }
RMM_NO_K16_ADVANCE=1 timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_noadv.log 2>&1 || { tail -30 gpurun_out/bench_noadv.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-gpu-rollout --no-fused --no-putget > gpurun_out/bench_adv2.log 2>&1 || { tail -30 gpurun_out/bench_adv2.log; exit 1; }
for f in bench_adv bench_noadv bench_adv2; do python -c "import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['last_stats']['learner_update_s'])"; done
