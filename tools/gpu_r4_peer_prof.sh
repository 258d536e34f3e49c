# Round 4: peer all-reduce timing sweep (sizes x workgroups, 2 and 3 ranks on one GPU) + a kernel
# trace of each rank process (rank processes started from bash, each under its own rocprofv3).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_rllib_gpu.py -k parity_counters -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || { tail -30 gpurun_out/pytest_parity.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_parity.log | tail -2
timeout -k 10 300 python -u -m ray_memory_management_amd.parallel.peer_selftest --world 2 --sweep --iters 200 --out gpurun_out/sweep2 > gpurun_out/sweep2.log 2>&1 || { tail -30 gpurun_out/sweep2.log; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/sweep2/rank0.json'))
for r in d['sweep']: print(r)"
timeout -k 10 300 python -u -m ray_memory_management_amd.parallel.peer_selftest --world 3 --sweep --iters 100 --out gpurun_out/sweep3 > gpurun_out/sweep3.log 2>&1 || { tail -30 gpurun_out/sweep3.log; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/sweep3/rank0.json'))
for r in d['sweep']: print(r)"
rm -rf gpurun_out/prof_peer gpurun_out/peerprof; mkdir -p gpurun_out/peerprof
ST=gpurun_out/peerprof/store
for r in 0 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_peer/r$r -o run -- python3 -m ray_memory_management_amd.parallel.peer_selftest --world 2 --rank $r --store $ST --out gpurun_out/peerprof --iters 100 > gpurun_out/peerprof/r$r.log 2>&1 &
done
wait %1 || { tail -20 gpurun_out/peerprof/r0.log; exit 1; }
wait %2 || { tail -20 gpurun_out/peerprof/r1.log; exit 1; }
for f in $(find gpurun_out/prof_peer -name "*kernel_stats.csv"); do echo "== $f"; python3 benchmarks/summarize_prof.py $f 12; done
rm -f $(find gpurun_out/prof_peer -name "*.db")
