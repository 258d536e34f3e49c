# round-6 same-box A/B: ab_old/ = the tree at 80b8b07 (K15x / K16x batching only) vs the current tree; fused loop
# and the runtime bench, alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/ab_r6.log
: > $L
for i in 1 2; do
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
