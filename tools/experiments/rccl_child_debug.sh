# Debug the RcclComm 2-rank same-GPU child: faulthandler + RCCL INFO logs per rank.
set -o pipefail
mkdir -p gpurun_out/rccl_dbg
python - <<'PY'
import os, sys, tempfile
sys.path.insert(0, os.getcwd())
src = open("tests/test_rccl_native.py").read()
start = src.index('_CHILD = r"""') + len('_CHILD = r"""')
end = src.index('"""', start)
child = src[start:end].format(root=os.getcwd())
open("gpurun_out/rccl_dbg/child.py", "w").write(child)
PY
d=$(mktemp -d)
for r in 0 1; do
  RMM_RCCL_SAME_DEVICE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,NET,ENV timeout -k 10 120 python -X faulthandler gpurun_out/rccl_dbg/child.py $r 2 $d/store > gpurun_out/rccl_dbg/r$r.out 2> gpurun_out/rccl_dbg/r$r.err &
done
wait
echo "rc done"; tail -5 gpurun_out/rccl_dbg/r0.out; tail -40 gpurun_out/rccl_dbg/r0.err; tail -15 gpurun_out/rccl_dbg/r1.err
