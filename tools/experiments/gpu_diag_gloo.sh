set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/diag_gloo_torchrun.py > gpurun_out/diag_direct.log 2>&1 || { tail -20 gpurun_out/diag_direct.log; exit 1; }
grep allreduce gpurun_out/diag_direct.log
timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29544 tools/diag_gloo_torchrun.py > gpurun_out/diag_torchrun.log 2>&1 || { tail -20 gpurun_out/diag_torchrun.log; exit 1; }
grep allreduce gpurun_out/diag_torchrun.log
