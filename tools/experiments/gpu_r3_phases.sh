set -o pipefail
mkdir -p gpurun_out
for n in 50 12; do
  timeout -k 10 120 python -u benchmarks/native_rollout_probe.py $n 100 1 > gpurun_out/ph_$n.log 2>&1 || { tail -5 gpurun_out/ph_$n.log; exit 1; }
  tail -1 gpurun_out/ph_$n.log
done
