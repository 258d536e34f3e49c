# round-6 same-box A/B of the runtime path: ab_old/ (8ea933a, before the runtime-semantics / ref-counting
# fixes) vs the current tree; bench.py runtime mode x3 alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/ab5_r6.log
: > $L
for i in 1 2 3; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    echo "== $v runtime $i" >> $L
    (cd $d && timeout -k 10 300 python -u bench.py --no-putget --no-fused) 2>&1 | grep '"metric"' >> $L || exit 1
  done
done
