# Round 4 (v): 2-learner rehearsal on one GPU (both learner actors on GPU 0: peer all-reduce, shared weights,
# direct rollout launches), then the 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --same-device --no-putget > gpurun_out/bench_v2.log 2>&1 || { grep -v "^frame" gpurun_out/bench_v2.log | tail -8; exit 1; }
grep '"metric"' gpurun_out/bench_v2.log | tail -1 | cut -c1-400
