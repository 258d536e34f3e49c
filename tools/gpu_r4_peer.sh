# Round 4: peer-memory all-reduce self-test (2 and 3 ranks on one GPU), GPU tests, 2-learner rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m ray_memory_management_amd.parallel.peer_selftest --world 2 --out gpurun_out/peer2 > gpurun_out/peer2.log 2>&1 || { tail -30 gpurun_out/peer2.log; exit 1; }
tail -1 gpurun_out/peer2.log | cut -c1-1500
timeout -k 10 240 python -u -m ray_memory_management_amd.parallel.peer_selftest --world 3 --out gpurun_out/peer3 > gpurun_out/peer3.log 2>&1 || { tail -30 gpurun_out/peer3.log; exit 1; }
tail -1 gpurun_out/peer3.log | cut -c1-600
timeout -k 10 400 python -u -m pytest tests/test_peer_allreduce.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1 || { tail -40 gpurun_out/pytest_peer.log; exit 1; }
grep -E "passed|failed|peer all-reduce" gpurun_out/pytest_peer.log | tail -5
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --dist-backend nccl --steps 5 --warmup 2 --no-putget > gpurun_out/rehearse_peer.log 2>&1 || { tail -30 gpurun_out/rehearse_peer.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_peer.log | tail -1 | cut -c1-3000
