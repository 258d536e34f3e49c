# round-6: runtime bench variance (per-iteration wall times, worker sample() time), 3 runs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-putget --no-fused > gpurun_out/var_$i.log 2>&1 || exit $?
done
