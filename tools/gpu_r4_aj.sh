# Round 4 (aj): 2-learner rehearsal on one MI355X after the sample prefetch default (torchrun launch shape, RCCL
# ranks on the same device -> PeerComm in-graph all-reduce, shared weights), then the gloo variant.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --same-device --steps 5 --warmup 2 > gpurun_out/rehearse_aj.log 2>&1 || { tail -30 gpurun_out/rehearse_aj.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_aj.log | tail -1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-putget > gpurun_out/rehearse_aj_gloo.log 2>&1 || { tail -30 gpurun_out/rehearse_aj_gloo.log; exit 1; }
tail -1 gpurun_out/rehearse_aj_gloo.log | cut -c1-900
