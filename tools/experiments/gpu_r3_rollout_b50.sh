# One hybrid worker in isolation at the bench layout (50 envs, 1 group, native loop) vs variants, then a
# kernel trace of the 50-env policy step and the runtime phase probe at the new default layout.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/rp_50_1.log 2>&1 && tail -1 gpurun_out/rp_50_1.log || exit 1
RMM_NO_NATIVE_ROLLOUT=1 timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/rp_50_1py.log 2>&1 && tail -1 gpurun_out/rp_50_1py.log || exit 1
timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 25 100 1 > gpurun_out/rp_25_1.log 2>&1 && tail -1 gpurun_out/rp_25_1.log || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_prof -o rp -- python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/rp_prof.log 2>&1 || { tail -5 gpurun_out/rp_prof.log; exit 1; }
f=$(find gpurun_out/rp_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-220
timeout -k 10 200 python -u benchmarks/ppo_phase_probe.py 1 > gpurun_out/rp_phase.log 2>&1 || { tail -5 gpurun_out/rp_phase.log; exit 1; }
tail -1 gpurun_out/rp_phase.log
