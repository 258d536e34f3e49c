# GPU suite, smoke, runtime bench (CPU rollouts), runtime bench (GPU rollout actors).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -n "^E " gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-putget --no-fused > gpurun_out/bench_cpu.log 2>&1 || { tail -30 gpurun_out/bench_cpu.log; exit 1; }
tail -1 gpurun_out/bench_cpu.log
timeout -k 10 300 python -u bench.py --rollout gpu --no-putget --no-fused > gpurun_out/bench_gpu.log 2>&1 || { tail -30 gpurun_out/bench_gpu.log; exit 1; }
tail -1 gpurun_out/bench_gpu.log
