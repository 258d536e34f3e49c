# Kernel-trace profiles of the two halves of the headline step, each in ONE process so rocprofv3
# sees every kernel: (1) the hybrid rollout worker in isolation (K19 + K10/K13/K16 policy step),
# (2) the fused PPO learner loop (SGD-step kernels).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_probe gpurun_out/prof_fused
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o run -- python3 benchmarks/hybrid_rollout_probe.py > gpurun_out/prof_probe.log 2>&1 || { tail -20 gpurun_out/prof_probe.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_fused.log 2>&1 || { tail -20 gpurun_out/prof_fused.log; exit 1; }
for d in prof_probe prof_fused; do
  for f in $(find gpurun_out/$d -name "*kernel_stats.csv"); do echo "## $d" >> gpurun_out/prof_k19_summary.txt; python3 benchmarks/summarize_prof.py $f 20 >> gpurun_out/prof_k19_summary.txt; done
done
rm -f $(find gpurun_out/prof_probe gpurun_out/prof_fused -name "*.db") $(find gpurun_out/prof_probe gpurun_out/prof_fused -name "*kernel_trace.csv")
cat gpurun_out/prof_k19_summary.txt | head -60
