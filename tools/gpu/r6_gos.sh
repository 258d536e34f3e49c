# GPU object-store bench alone, with progress lines and a Python stack dump if it stalls
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
timeout -s ABRT -k 10 170 python -u benchmarks/gpu_object_store_bench.py --sizes 1 --iters 2 > gpurun_out/gos_bench_r6.log 2>&1
echo "rc=$?" >> gpurun_out/gos_bench_r6.log
