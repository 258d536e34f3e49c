# round-6 multi-rank rehearsals on the box's one GPU: the learner step over PeerComm in "one" and "fork" mode
# (2 / 4 / 8 ranks, ZeRO-1 workgroups from occupancy), the 4-learner runtime bench with replica identity,
# and a kernel trace of the fork mode (ZeRO-1 on the comm stream beside the trunk backward)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/multirank_r6.log
: > $L
for cfg in "one 2" "fork 2" "fork 4" "fork 8"; do
  set -- $cfg
  echo "== RMM_PEER_MODE=$1 world=$2" >> $L
  RMM_PEER_MODE=$1 timeout -k 10 300 python -u benchmarks/peer_fork_probe.py --world $2 --updates 5 >> $L 2>&1 || exit $?
done
echo "== bench.py --gpus 4 --same-device" >> $L
timeout -k 10 400 python -u bench.py --gpus 4 --same-device --steps 5 --warmup 2 --no-putget >> $L 2>&1 || exit $?
RMM_PEER_MODE=fork timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_fork2 -o fork2 -- python3 -u benchmarks/peer_fork_probe.py --world 2 --updates 2 > gpurun_out/peer_fork_probe_prof.log 2>&1 || exit $?
python tools/trace_overlap.py gpurun_out/prof_fork2 > gpurun_out/fork2_overlap.txt 2>&1
python tools/trace_overlap.py gpurun_out/prof_fork2 --kernel k_peer_allreduce >> gpurun_out/fork2_overlap.txt 2>&1
exit 0
