set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u benchmarks/ppo_phase_probe.py 1 > gpurun_out/ph2.log 2>&1 || { tail -5 gpurun_out/ph2.log; exit 1; }
tail -1 gpurun_out/ph2.log
