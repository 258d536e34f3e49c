# K10 backward partials in bf16 (default) vs fp32 (RMM_TRUNK_PARTIAL_FP32=1), new k-major dW2 layout:
# kernel tests, isolated backward timing, fused-loop and runtime A/B.
set -o pipefail
mkdir -p gpurun_out
true > gpurun_out/bp_pytest.log
rc=$?; tail -2 gpurun_out/bp_pytest.log; grep -E "FAILED|Error" gpurun_out/bp_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  RMM_TRUNK_PARTIAL_FP32=$v timeout -k 10 120 python -u benchmarks/bench_trunk.py --only bwd --B 500 > gpurun_out/bp_k_$v.log 2>&1 || { tail -5 gpurun_out/bp_k_$v.log; exit 1; }
  echo "FP32=$v $(tail -1 gpurun_out/bp_k_$v.log)"
done
for rep in 1 2; do
  for v in 1 0; do
    RMM_TRUNK_PARTIAL_FP32=$v timeout -k 10 120 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget > gpurun_out/bp_f_$v.log 2>&1 || { tail -5 gpurun_out/bp_f_$v.log; exit 1; }
    echo "fused FP32=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bp_f_$v.log)"
  done
done
for v in 1 0; do
  RMM_TRUNK_PARTIAL_FP32=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-putget --no-fused --no-gpu-rollout > gpurun_out/bp_r_$v.log 2>&1 || { tail -5 gpurun_out/bp_r_$v.log; exit 1; }
  echo "runtime FP32=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bp_r_$v.log) $(grep -o '"learner_update_s": [0-9.]*' gpurun_out/bp_r_$v.log)"
done
