# round-6 same-box A/B/C: ab_old/ (80b8b07), current tree (new2), ab_new3/ (new2 + h1 stored from LDS in 16-B
# vectors): fused-loop bench alternating, then a kernel trace of each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/ab3_r6.log
: > $L
for i in 1 2; do
  for v in old new2 new3; do
    d=.; [ $v = old ] && d=ab_old; [ $v = new3 ] && d=ab_new3
    echo "== $v fused $i" >> $L
    (cd $d && timeout -k 10 200 python -u bench.py --mode fused --steps 20 --warmup 3 --no-putget) 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
for v in old new2 new3; do
  d=.; [ $v = old ] && d=ab_old; [ $v = new3 ] && d=ab_new3
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_ab_$v -o ab_$v -- python3 -u bench.py --mode fused --steps 10 --warmup 2 --no-putget > $R/gpurun_out/prof_ab_$v.log 2>&1) || exit $?
  python tools/rocpd_stats.py gpurun_out/prof_ab_$v/ab_${v}_results.db 14 > gpurun_out/prof_ab_$v.txt
  rm -rf gpurun_out/prof_ab_$v
done
