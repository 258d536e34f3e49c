# round-6: spill line-rate probe, 8-learner 1-GPU rehearsal, and a kernel trace of the fork-mode 2-learner
# rehearsal (ZeRO-1 launch on the comm stream beside the trunk backward)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/spill_probe.py --gb 1 --reps 3 > gpurun_out/spill_probe_r6.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --gpus 8 --same-device --steps 5 --warmup 2 --no-putget > gpurun_out/bench_same8_r6.log 2>&1 || exit $?
RMM_PEER_MODE=fork RMM_NO_FORKSERVER=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_fork2 -o fork2 -- python3 -u bench.py --gpus 2 --same-device --steps 3 --warmup 1 --no-putget > gpurun_out/bench_fork2_r6.log 2>&1
echo "rc=$?" >> gpurun_out/bench_fork2_r6.log
