# Kernel-trace timeline of the fused PPO loop (learner SGD steps + rollout steps): per-step span,
# kernel busy time and inter-kernel gaps (benchmarks/step_timeline.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tl -o run -- python3 bench.py --mode fused --steps 3 --warmup 1 --no-putget > gpurun_out/prof_tl.log 2>&1 || { tail -5 gpurun_out/prof_tl.log; exit 1; }
python3 benchmarks/step_timeline.py gpurun_out/prof_tl > gpurun_out/timeline_r3.txt 2>&1
cat gpurun_out/timeline_r3.txt
rm -f $(find gpurun_out/prof_tl -name "*.db")
timeout -k 10 300 python -u -m pytest tests/test_raysort.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_raysort.log 2>&1 || { tail -40 gpurun_out/pytest_raysort.log; exit 1; }
tail -2 gpurun_out/pytest_raysort.log
