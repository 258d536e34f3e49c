# Round 4 (aa): K12 row split with the finalize deferred into the trunk-reduce launch (finalize + Adam per element).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu.py -k "tail_adam or parity or graph_matches" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_aa.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_aa.log | head; tail -3 gpurun_out/pytest_aa.log; exit 1; }
tail -1 gpurun_out/pytest_aa.log
for m in 2 1 2 1; do
  RMM_K12_SPLIT=$m timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget > gpurun_out/fused_aa_$m.log 2>&1 || { tail -5 gpurun_out/fused_aa_$m.log; exit 1; }
  echo "SPLIT=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fused_aa_$m.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_aa
RMM_K12_SPLIT=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aa -o run -- python3 bench.py --mode fused --steps 5 --warmup 2 --no-putget > gpurun_out/prof_aa.log 2>&1 || { tail -5 gpurun_out/prof_aa.log; exit 1; }
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/prof_aa/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r['Percentage'])>1: print(round(float(r['AverageNs'])/1000,2), r['Calls'], r['Name'][:70])
"
