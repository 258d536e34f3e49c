# round-6 A/B: learner + rollout worker pinned to the GPU's NUMA-local CPUs (default) vs left to the OS
# (RMM_NUMA_PIN=0); runtime bench alternating, 3 runs each; then the GPU tests that drive the rollout worker
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python tools/numa_probe.py > gpurun_out/numa.log 2>&1
lscpu > gpurun_out/lscpu.log 2>&1
L=gpurun_out/numa_ab.log
: > $L
for i in 1 2 3; do
  for f in 1 0; do
    echo "== RMM_NUMA_PIN=$f run $i" >> $L
    RMM_NUMA_PIN=$f timeout -k 10 300 python -u bench.py --no-putget --no-fused 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
