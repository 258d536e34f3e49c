# gos bench (stack dump if it stalls) then the multi-rank learner probes (tools/gpu/r6_batch4.sh)
cd $GRAFT_REPO_ROOT
bash tools/gpu/r6_gos.sh
grep -q "^rc=0" gpurun_out/gos_bench_r6.log || exit 1
bash tools/gpu/r6_batch4.sh
