# round-6 batch 4: multi-rank learner step over PeerComm (2 ranks on the box's GPU), "one" vs "fork" mode, and a
# kernel trace of the fork mode with the overlap of each ZeRO-1 launch against the trunk backward
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in one fork; do
  echo "RMM_PEER_MODE=$m" >> gpurun_out/peer_fork_probe_r6.log
  RMM_PEER_MODE=$m timeout -k 10 240 python -u benchmarks/peer_fork_probe.py --world 2 >> gpurun_out/peer_fork_probe_r6.log 2>&1 || exit $?
done
RMM_PEER_MODE=fork timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_fork2 -o fork2 -- python3 -u benchmarks/peer_fork_probe.py --world 2 --updates 2 > gpurun_out/peer_fork_probe_prof.log 2>&1 || exit $?
python tools/trace_overlap.py gpurun_out/prof_fork2 > gpurun_out/fork2_overlap.txt 2>&1
python tools/trace_overlap.py gpurun_out/prof_fork2 --kernel k_peer_allreduce >> gpurun_out/fork2_overlap.txt 2>&1
rm -rf gpurun_out/prof_fork2/*/*/*.csv.gz 2>/dev/null
exit 0
