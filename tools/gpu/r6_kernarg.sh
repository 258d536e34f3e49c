# round-6 A/B: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the runtime default, fused loop and
# runtime bench alternating, plus the rollout probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/kernarg_ab.log
: > $L
for i in 1 2; do
  for f in 0 1; do
    echo "== HIP_FORCE_DEV_KERNARG=$f run $i" >> $L
    if [ $f = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    timeout -k 10 200 python -u benchmarks/native_rollout_probe.py 50 100 1 fp32 2>&1 | grep us_per_step >> $L || exit 1
    timeout -k 10 200 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget 2>&1 | grep '"metric"' >> $L || exit 1
    timeout -k 10 300 python -u bench.py --no-putget --no-fused 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
