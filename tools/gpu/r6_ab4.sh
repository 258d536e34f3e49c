# round-6 same-box A/B: ab_old/ (80b8b07) vs the current tree; fused loop x3 alternating, runtime x2, kernel traces
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/ab4_r6.log
: > $L
for i in 1 2 3; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    echo "== $v fused $i" >> $L
    (cd $d && timeout -k 10 200 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget) 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
for i in 1 2; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    echo "== $v runtime $i" >> $L
    (cd $d && timeout -k 10 300 python -u bench.py --no-putget --no-fused) 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
for v in old new; do
  d=.; [ $v = old ] && d=ab_old
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_ab_$v -o ab_$v -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > $R/gpurun_out/prof_ab_$v.log 2>&1) || exit $?
  python tools/rocpd_stats.py gpurun_out/prof_ab_$v/ab_${v}_results.db 14 > gpurun_out/prof_ab_$v.txt
  rm -rf gpurun_out/prof_ab_$v
done
