# Round 4 (k): K21 with per-XCD hierarchical barriers + relaxed done_seq: parity, timeline at 64/128/256 WGs, runtime A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_rllib_runtime_gpu.py -k "rollout_server" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
for w in 64 128 256; do
  RMM_ROLLOUT_SERVER=1 RMM_ROLLOUT_SERVER_PROF=1 RMM_ROLLOUT_SERVER_WGS=$w timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_k_$w.log 2>&1 || { tail -10 gpurun_out/probe_k_$w.log; exit 1; }
  echo "wgs=$w"; tail -2 gpurun_out/probe_k_$w.log
done
RMM_ROLLOUT_SERVER=0 timeout -k 10 120 python -u benchmarks/native_rollout_probe.py 50 100 1 > gpurun_out/probe_k_graph.log 2>&1 || { tail -10 gpurun_out/probe_k_graph.log; exit 1; }
echo "graph: $(tail -1 gpurun_out/probe_k_graph.log)"
