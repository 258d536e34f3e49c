# Dense Adam overlapped with the trunk backward with a capped grid: fused loop per cap.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -q -k "manual_step" --timeout 150 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || { tail -40 gpurun_out/pytest_split.log; exit 1; }
RMM_SPLIT_ADAM_BLOCKS=32 timeout -k 10 300 python -u -m pytest tests/test_rllib_runtime_gpu.py -x -q -k "manual_step" --timeout 150 --timeout-method thread >> gpurun_out/pytest_split.log 2>&1 || { tail -40 gpurun_out/pytest_split.log; exit 1; }
grep passed gpurun_out/pytest_split.log
for cap in 0 16 32 64 128 0; do
echo "== cap $cap"; RMM_SPLIT_ADAM_BLOCKS=$cap timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget | cut -c100-200
done
