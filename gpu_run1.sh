set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python benchmarks/gpu_shuffle.py --rows-per-gpu 8000000 --row-bytes 256 > gpurun_out/gpu_shuffle.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/gpu_shuffle.log
