# Order check: torchrun launch first, then the direct launch; list leftover runtime processes between.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/order_torchrun.log 2>&1 || { tail -30 gpurun_out/order_torchrun.log; exit 1; }
grep '"metric"' gpurun_out/order_torchrun.log | tail -1 | cut -c1-200
sleep 2
ps -eo pid,ppid,stat,etime,cmd | grep -v grep | grep -E "ray_memory_management_amd|worker_main|node.py" > gpurun_out/order_leftovers.txt || true
echo "leftover runtime processes: $(wc -l < gpurun_out/order_leftovers.txt)"
head -5 gpurun_out/order_leftovers.txt | cut -c1-200
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-putget > gpurun_out/order_direct.log 2>&1 || { tail -30 gpurun_out/order_direct.log; exit 1; }
grep '"metric"' gpurun_out/order_direct.log | tail -1 | cut -c1-200
python3 -c "
import json
for f in ['gpurun_out/order_torchrun.log','gpurun_out/order_direct.log']:
    l=[x for x in open(f) if x.startswith('{\"metric')][-1]
    d=json.loads(l); print(f, d['ms_per_step'], d['last_stats'].get('learner_update_s'))
"
