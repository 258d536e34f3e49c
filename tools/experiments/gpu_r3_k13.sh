# K13 XCD-aware tile order + pipelined K10 trunk fwd/bwd: correctness, isolated K13 A/B, fused-loop
# A/B (K13 order), and the per-SGD-step kernel timeline.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -k "dense or trunk" --timeout 120 --timeout-method thread > gpurun_out/pytest_k13.log 2>&1 || { tail -30 gpurun_out/pytest_k13.log; exit 1; }
tail -1 gpurun_out/pytest_k13.log
echo "== K13 remap"; timeout -k 10 120 python -u benchmarks/bench_dense_fwd.py
echo "== K13 raster"; RMM_K13_NOREMAP=1 timeout -k 10 120 python -u benchmarks/bench_dense_fwd.py
echo "== fused loop remap"; timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget | cut -c1-200
echo "== fused loop raster"; RMM_K13_NOREMAP=1 timeout -k 10 200 python -u bench.py --mode fused --steps 10 --warmup 3 --no-putget | cut -c1-200
rm -rf gpurun_out/prof_tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tl -o run -- python3 bench.py --mode fused --steps 3 --warmup 1 --no-putget > gpurun_out/prof_tl.log 2>&1 || { tail -5 gpurun_out/prof_tl.log; exit 1; }
python3 benchmarks/step_timeline.py gpurun_out/prof_tl > gpurun_out/timeline_r3b.txt 2>&1
cat gpurun_out/timeline_r3b.txt
rm -rf gpurun_out/prof_tl
