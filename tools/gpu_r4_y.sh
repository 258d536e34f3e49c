# Round 4 (y): host cost of a kernel launch / event record on the box (rollout-step launch phase attribution).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "
import torch
from ray_memory_management_amd._native import require_hip
h = require_hip()
s = torch.cuda.Stream()
torch.cuda.synchronize()
for n in (100, 1000, 1000):
    print('launch_us, event_record_us, launch_200x512_us:', [round(x, 2) for x in h.launch_overhead_probe(n, s.cuda_stream)])
" > gpurun_out/launch_y.log 2>&1 || { tail -5 gpurun_out/launch_y.log; exit 1; }
cat gpurun_out/launch_y.log
