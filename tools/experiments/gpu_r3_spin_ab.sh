# rollout step wait: event poll (spin) vs blocking synchronize; probe + runtime bench
set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  RMM_ROLLOUT_SPIN=$v timeout -k 10 240 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/spin_probe_$v.log 2>&1 || { tail -5 gpurun_out/spin_probe_$v.log; exit 1; }
  echo "SPIN=$v"; grep "n=" gpurun_out/spin_probe_$v.log | grep "graphs=True"
done
for i in 1 2 3; do for v in 0 1; do
  RMM_ROLLOUT_SPIN=$v timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/spin_rt_$v.log 2>&1 || { tail -5 gpurun_out/spin_rt_$v.log; exit 1; }
  echo "runtime SPIN=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/spin_rt_$v.log)"
done; done
