# round-6 multi-rank rehearsals, second part: 8 ranks on the one GPU in "one" mode (the shared-device default:
# fork mode's concurrent collective launches of 8 processes cannot all be resident on one device), the 4-learner
# runtime bench with replica identity, and a kernel trace of the 2-rank fork mode
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/multirank_r6b.log
: > $L
echo "== RMM_PEER_BLOCKS=8 RMM_PEER_ZERO1_BLOCKS=8 RMM_PEER_MODE=one world=8" >> $L
RMM_PEER_BLOCKS=8 RMM_PEER_ZERO1_BLOCKS=8 RMM_PEER_MODE=one RMM_PEER_TIMEOUT_S=30 timeout -k 10 300 python -u benchmarks/peer_fork_probe.py --world 8 --updates 3 >> $L 2>&1 || exit $?
echo "== bench.py --gpus 4 --same-device" >> $L
timeout -k 10 400 python -u bench.py --gpus 4 --same-device --steps 5 --warmup 2 --no-putget >> $L 2>&1 || exit $?
RMM_PEER_MODE=fork timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_fork2 -o fork2 -- python3 -u benchmarks/peer_fork_probe.py --world 2 --updates 2 > gpurun_out/peer_fork_probe_prof.log 2>&1 || exit $?
python tools/trace_overlap.py gpurun_out/prof_fork2 > gpurun_out/fork2_overlap.txt 2>&1
python tools/trace_overlap.py gpurun_out/prof_fork2 --kernel k_peer_allreduce >> gpurun_out/fork2_overlap.txt 2>&1
find gpurun_out/prof_fork2 -name "*.csv" -size +2M -delete
exit 0
