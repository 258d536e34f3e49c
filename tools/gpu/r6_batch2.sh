# round-6 batch 2: new kernel tests (fused K13x+K16x, forked dense Adam), the rollout probe A/B, then the
# spill probe and the multi-rank rehearsals (tools/gpu/r6_multirank.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_x3_kernels.py tests/test_rllib_runtime_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "fused or dense_adam_fork or tail_adam or direct_launch" > gpurun_out/gpu_tests_b2.log 2>&1 || exit $?
for f in 0 1; do
  RMM_ROLLOUT_FUSED_HEADS=$f timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 fp32 >> gpurun_out/rollout_fused_ab.log 2>&1 || exit $?
done
for f in 0 1 0 1; do
  echo "RMM_X3_DENSE_ADAM_FORK=$f" >> gpurun_out/dense_adam_fork_ab.log
  RMM_X3_DENSE_ADAM_FORK=$f timeout -k 10 300 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget >> gpurun_out/dense_adam_fork_ab.log 2>&1 || exit $?
done
bash tools/gpu/r6_multirank.sh
