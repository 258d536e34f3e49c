# PPO step kernels (fused single-process loop = the learner + rollout kernels of the runtime
# path): kernel-trace stats, then one PMC pass with MFMA counters (own run, no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_ppo gpurun_out/pmc_ppo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ppo -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_bench.log 2>&1 || { tail -5 gpurun_out/prof_bench.log; exit 1; }
for f in $(find gpurun_out/prof_ppo -name "*kernel_stats.csv"); do python3 benchmarks/summarize_prof.py $f 40 > gpurun_out/prof_ppo_summary.txt; done
head -30 gpurun_out/prof_ppo_summary.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_ppo -o run -- python3 bench.py --mode fused --steps 2 --warmup 1 --no-putget > gpurun_out/pmc_bench.log 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_bench.log; exit 1; }
python3 benchmarks/mfma_report.py gpurun_out/pmc_ppo 30 > gpurun_out/mfma_report.txt 2>&1
cat gpurun_out/mfma_report.txt
rm -f $(find gpurun_out/pmc_ppo gpurun_out/prof_ppo -name "*.db")
