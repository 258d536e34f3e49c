set -o pipefail
mkdir -p gpurun_out
for g in graphs eager; do
  DBG_UPDATES=2 DBG_ITERS=3 RMM_SGD_CHAIN=3 timeout -k 10 120 python -u tools/experiments/split_fin_debug.py $g > gpurun_out/splitdbg_g.log 2>&1 || { tail -8 gpurun_out/splitdbg_g.log; exit 1; }
  echo "== $g"; grep -v amdgpu.ids gpurun_out/splitdbg_g.log | grep -v "max|d| 0.000e+00"
done
