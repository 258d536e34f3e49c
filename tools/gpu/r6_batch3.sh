# round-6 batch 3: spill probe (packed vs device-placed chunks), the object-store bench's spill rows, and the
# fork-mode multi-rank learner probe under a kernel trace (ranks exit normally, so rocprofv3 flushes)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/spill_probe.py --gb 1 --reps 3 > gpurun_out/spill_probe_r6b.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/gpu_object_store_bench.py --sizes 1 --iters 2 > gpurun_out/gos_bench_r6.log 2>&1 || exit $?
RMM_PEER_MODE=fork timeout -k 10 300 python -u benchmarks/peer_fork_probe.py --world 2 > gpurun_out/peer_fork_probe_r6.log 2>&1 || exit $?
RMM_PEER_MODE=fork timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_fork2 -o fork2 -- python3 -u benchmarks/peer_fork_probe.py --world 2 --updates 2 > gpurun_out/peer_fork_probe_prof.log 2>&1
echo "rc=$?" >> gpurun_out/peer_fork_probe_prof.log
