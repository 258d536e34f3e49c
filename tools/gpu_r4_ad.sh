# Round 4 (ad): K13s slice count sweep on the fused loop (RMM_K13S_S applies to the SGD and rollout K13s).
set -o pipefail
mkdir -p gpurun_out
for sl in 0 2 8 0 2 8; do
  RMM_K13S_S=$sl timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/fused_ad_$sl.log 2>&1 || { tail -5 gpurun_out/fused_ad_$sl.log; exit 1; }
  echo "S=$sl $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fused_ad_$sl.log)"
done
