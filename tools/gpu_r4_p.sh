# Round 4 (p): the two suite failures after their fixes, then bench twice (box variance check).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_objects.py tests/test_rccl_native.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_p.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_p.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-putget > gpurun_out/bench_p$i.log 2>&1 || { tail -5 gpurun_out/bench_p$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_p$i.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','runtime_gpu_rollout_ms_per_step','fused_loop_samples_per_s')}, d['last_stats']['learner_update_s'])"
done
timeout -k 10 200 python -u benchmarks/native_rollout_probe.py > gpurun_out/probe_p.log 2>&1 || { tail -5 gpurun_out/probe_p.log; exit 1; }
tail -12 gpurun_out/probe_p.log
timeout -k 10 240 python3 -u benchmarks/bench_trunk.py > gpurun_out/trunk_phases_p.json 2> gpurun_out/trunk_phases_p.err || { tail -5 gpurun_out/trunk_phases_p.err; exit 1; }
cat gpurun_out/trunk_phases_p.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_p.log 2>&1 || { tail -5 gpurun_out/prof_p.log; exit 1; }
find gpurun_out/prof_p -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -14 {} | cut -d, -f1-8'
