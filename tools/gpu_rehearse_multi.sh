# Multi-learner rehearsal on a 1-GPU box: 2 learner actors on the same GPU (gloo), 2x2 hybrid rollout
# workers, the same code path the 8-GPU SCALE run takes (placement-group bundles, learner group,
# gradient all-reduce), then the torchrun launch shape with 2 ranks (rank 0 drives the runtime).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-putget > gpurun_out/rehearse_2learners.log 2>&1 || { tail -30 gpurun_out/rehearse_2learners.log; exit 1; }
tail -1 gpurun_out/rehearse_2learners.log | cut -c1-600
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/rehearse_torchrun.log 2>&1 || { tail -30 gpurun_out/rehearse_torchrun.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_torchrun.log | tail -1 | cut -c1-600
