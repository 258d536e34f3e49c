# Counter list + kernel-trace profile of the runtime bench (GPU rollout actors + learner actor).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -i "mfma\|SQ_INSTS_VALU\b\|SQ_BUSY\|LDS_BANK" gpurun_out/counters_list.txt | head -40 > gpurun_out/counters_mfma.txt || true
rm -rf gpurun_out/prof_rt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rt -o run -- python3 bench.py --rollout gpu --no-putget --no-fused --no-gpu-rollout --steps 5 --warmup 2 > gpurun_out/prof_rt.log 2>&1 || { tail -20 gpurun_out/prof_rt.log; exit 1; }
for f in $(find gpurun_out/prof_rt -name "*kernel_stats.csv"); do python3 benchmarks/summarize_prof.py $f 40 >> gpurun_out/prof_rt_summary.txt; done
rm -f $(find gpurun_out/prof_rt -name "*.db") 
head -45 gpurun_out/prof_rt_summary.txt
tail -1 gpurun_out/prof_rt.log | cut -c1-400
