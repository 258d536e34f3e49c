set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  RMM_TRUNK_PARTIAL_FP32=$v timeout -k 10 200 python -u -m pytest tests/test_rllib_runtime_gpu.py -q --timeout 120 --timeout-method thread -k "manual_step or fused_adam or clip_matches or action0" > gpurun_out/bpd_$v.log 2>&1
  echo "FP32=$v rc=$? $(tail -1 gpurun_out/bpd_$v.log)"
  grep -E "^E .*(max|assert|diff)" gpurun_out/bpd_$v.log | head -4
done
