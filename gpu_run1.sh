set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u benchmarks/train_resnet50.py --workers 1 --batch 256 --steps 20 --warmup 5 > gpurun_out/resnet50.log 2>&1; echo "rc=$?"
tail -5 gpurun_out/resnet50.log; cat gpurun_out/resnet50_progress.log
