# Hybrid worker probe (graph vs eager launches) + kernel traces of one worker's rollout steps.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/hybrid_rollout_probe.py > gpurun_out/probe_graphs.log 2>&1 || { tail -20 gpurun_out/probe_graphs.log; exit 1; }
tail -6 gpurun_out/probe_graphs.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_graph -o run -- python3 benchmarks/hybrid_step_trace.py graph > gpurun_out/trace_graph.log 2>&1 || { tail -20 gpurun_out/trace_graph.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_eager -o run -- python3 benchmarks/hybrid_step_trace.py eager > gpurun_out/trace_eager.log 2>&1 || { tail -20 gpurun_out/trace_eager.log; exit 1; }
find gpurun_out/trace_graph gpurun_out/trace_eager -name "*kernel_trace.csv" | head
