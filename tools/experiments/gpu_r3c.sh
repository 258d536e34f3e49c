# Native RCCL communicator on one GPU (2 ranks, distinct host ids): eager fork/join tests, the
# learner actors, the 2-learner bench rehearsal over RCCL; LAST (may crash): an RCCL all-reduce
# captured on the capture stream itself (no fork) to learn whether capture works at all here.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rccl_native.py tests/test_gpu_objects.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_rccl.log 2>&1 || { tail -60 gpurun_out/pytest_rccl.log; exit 1; }
tail -3 gpurun_out/pytest_rccl.log
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --dist-backend nccl --steps 3 --warmup 1 --no-putget > gpurun_out/rehearse_rccl_2learners.log 2>&1 || { tail -40 gpurun_out/rehearse_rccl_2learners.log; exit 1; }
tail -1 gpurun_out/rehearse_rccl_2learners.log | cut -c1-1200
python - <<'PY'
import os
src = open("tests/test_rccl_native.py").read()
start = src.index('_CHILD = r"""') + len('_CHILD = r"""')
child = src[start:src.index('"""', start)].format(root=os.getcwd())
open("gpurun_out/rccl_child.py", "w").write(child)
PY
d=$(mktemp -d)
for r in 0 1; do
  RMM_RCCL_SAME_DEVICE=1 RMM_RCCL_IN_GRAPH=1 RMM_RCCL_FORK=0 timeout -k 10 120 python -X faulthandler gpurun_out/rccl_child.py $r 2 $d/store > gpurun_out/ingraph_r$r.out 2> gpurun_out/ingraph_r$r.err &
done
wait
echo "in-graph (no fork) results:"; cat gpurun_out/ingraph_r0.out gpurun_out/ingraph_r1.out; grep -h "Fatal\|File" gpurun_out/ingraph_r0.err | head -5
