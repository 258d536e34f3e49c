set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_ppo
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES FETCH_SIZE --kernel-trace -d gpurun_out/pmc_ppo -o run -- python3 bench.py --steps 2 --warmup 1 --no-putget > gpurun_out/pmc_bench.log 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmc_bench.log; exit 1; }
python3 benchmarks/pmc_summary.py gpurun_out/pmc_ppo > gpurun_out/pmc_ppo_summary.txt 2>&1
rm -f $(find gpurun_out/pmc_ppo -name "*.db")
head -30 gpurun_out/pmc_ppo_summary.txt
