# round-6: x3 phase-timestamp probe (last SGD step of one update), twice, then the multi-rank part 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u benchmarks/x3_phase_probe.py > gpurun_out/x3_phase_probe.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/x3_phase_probe.py >> gpurun_out/x3_phase_probe.log 2>&1 || exit $?
bash tools/gpu/r6_multirank3.sh
