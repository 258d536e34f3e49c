# Multi-learner rehearsal on a 1-GPU box: 2 learner actors on the same GPU, 2x hybrid rollout workers,
# the code path the 8-GPU SCALE run takes (placement-group bundles, learner group, per-step gradient
# all-reduce). (1) the production backend: PeerComm (peer-memory all-reduce, --dist-backend nccl);
# (2) gloo (GroupComm); (3) the torchrun launch shape with 2 ranks (rank 0 drives the runtime).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --steps 5 --warmup 2 --no-putget ${BENCH_ARGS:-} > gpurun_out/rehearse_peer.log 2>&1 || { tail -30 gpurun_out/rehearse_peer.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_peer.log | tail -1 | cut -c1-400
grep -o '"comm": "[A-Za-z]*"' gpurun_out/rehearse_peer.log | head -1
[ -n "${PEER_ONLY:-}" ] && exit 0
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-putget ${BENCH_ARGS:-} > gpurun_out/rehearse_2learners.log 2>&1 || { tail -30 gpurun_out/rehearse_2learners.log; exit 1; }
tail -1 gpurun_out/rehearse_2learners.log | cut -c1-400
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/rehearse_torchrun.log 2>&1 || { tail -30 gpurun_out/rehearse_torchrun.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_torchrun.log | tail -1 | cut -c1-400
