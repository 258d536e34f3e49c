# K13s split-K dense layer: timing sweep over configurations and slice counts at M = 500
# (each run its own process: the overrides are read once)
set -o pipefail
mkdir -p gpurun_out
for c in 3 5 6; do
  for s in 2 3 4 6; do
    export RMM_K13S_CFG=$c RMM_K13S_S=$s
    timeout -k 10 120 python -u benchmarks/bench_dense_fwd.py > gpurun_out/k13s_c${c}_S$s.log 2>&1 || { tail -20 gpurun_out/k13s_c${c}_S$s.log; exit 1; }
    echo "cfg=$c S=$s"; grep '^{"M500' gpurun_out/k13s_c${c}_S$s.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); (m,r),=d.items()
    cons = r.get('k15_part_us', r.get('k16_part_us')); base = r.get('k15_us', r.get('k16_us'))
    print(m, 'S', r['S'], 'k13', r['k13_us'], 'k13s', r['k13s_us'], 'cons', base, '->', cons, 'total', round(r['k13_us']+base,2), '->', round(r['k13s_us']+cons,2), 'err', '%.1e' % r['max_abs_err_vs_fp32'])
"
  done
done
unset RMM_K13S_CFG RMM_K13S_S
timeout -k 10 120 python -u benchmarks/bench_dense_fwd.py > gpurun_out/k13s_default.log 2>&1 && echo default && cat gpurun_out/k13s_default.log | grep '^{"M'
