# Round 4 (c): learner roofline, then the rest of (b): 3-rank peer sweep, fp32 + bf16 bench, GPU shuffle tests + OOC run.
set -o pipefail
bash tools/gpu_r4_roofline.sh || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m ray_memory_management_amd.parallel.peer_selftest --world 3 --sweep --iters 100 --out gpurun_out/sweep3 > gpurun_out/sweep3.log 2>&1 || { tail -5 gpurun_out/sweep3.log; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/sweep3/rank0.json'))
for r in d['sweep']: print(r)"
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-putget > gpurun_out/bench_r4c.log 2>&1 || { tail -30 gpurun_out/bench_r4c.log; exit 1; }
grep '"metric"' gpurun_out/bench_r4c.log | tail -1 | cut -c1-3000
timeout -k 10 400 python -u -m pytest tests/test_gpu_shuffle.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_shuffle.log 2>&1 || { tail -30 gpurun_out/pytest_shuffle.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_shuffle.log | tail -5
timeout -k 10 600 python -u benchmarks/gpu_shuffle_ooc.py --quota-gb 8 --factor 4 --rounds 16 --partitions 8 > gpurun_out/shuffle_ooc.log 2>&1 || { tail -30 gpurun_out/shuffle_ooc.log; exit 1; }
tail -1 gpurun_out/shuffle_ooc.log
