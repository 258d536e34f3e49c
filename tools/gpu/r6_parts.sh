# round-6 probe: rollout K16x as ONE 1024-thread workgroup (4 rows per wave, step advance after a barrier; no
# per-workgroup system fence + ticket) for B = 50 (RMM_PROBE_K16_ONE=1) vs 13 workgroups, rollout probe alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/k16one_ab.log
: > $L
for i in 1 2 3; do
  for f in 0 1; do
    echo "== K16_ONE=$f run $i" >> $L
    if [ $f = 1 ]; then export RMM_PROBE_K16_ONE=1; else unset RMM_PROBE_K16_ONE; fi
    timeout -k 10 200 python -u benchmarks/native_rollout_probe.py 50 100 1 fp32 2>&1 | grep us_per_step >> $L || exit 1
  done
done
unset RMM_PROBE_K16_ONE
timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "direct or rollout" > gpurun_out/k16one_tests.log 2>&1
RMM_PROBE_K16_ONE=1 timeout -k 10 400 python -u -m pytest tests/test_rllib_runtime_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "direct or rollout" >> gpurun_out/k16one_tests.log 2>&1
