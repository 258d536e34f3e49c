# Native rollout loop: env step split over 1/2/4 CPU threads, event polling vs blocking wait (isolated
# 50-env hybrid worker), then the runtime bench at the new defaults.
set -o pipefail
mkdir -p gpurun_out
for sp in 1 0; do
  for th in 1 2 4; do
    RMM_NATIVE_SPIN=$sp RMM_ENV_THREADS=$th timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/et_${th}_$sp.log 2>&1 || { tail -5 gpurun_out/et_${th}_$sp.log; exit 1; }
    echo "threads=$th spin=$sp $(tail -1 gpurun_out/et_${th}_$sp.log)"
  done
done
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/et_rt_$rep.log 2>&1 || { tail -5 gpurun_out/et_rt_$rep.log; exit 1; }
  echo "runtime default $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/et_rt_$rep.log) $(grep -o '"cpus_per_rollout_worker": [0-9]*' gpurun_out/et_rt_$rep.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/et_rt_$rep.log)"
  RMM_ENV_THREADS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/et_rt1_$rep.log 2>&1 || { tail -5 gpurun_out/et_rt1_$rep.log; exit 1; }
  echo "runtime threads=1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/et_rt1_$rep.log)"
done
