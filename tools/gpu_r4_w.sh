# Round 4 (w): K1 copy variants (GPU store put path) vs hipMemcpyAsync / torch copy_, read-only / write-only rates.
set -o pipefail
mkdir -p gpurun_out
for v in 0 2; do
  RMM_COPY_VARIANT=$v timeout -k 10 120 python -u benchmarks/bench_copy.py 4 > gpurun_out/copy_w_$v.log 2>&1 || { tail -5 gpurun_out/copy_w_$v.log; exit 1; }
  tail -1 gpurun_out/copy_w_$v.log
done
