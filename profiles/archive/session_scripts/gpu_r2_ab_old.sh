#!/bin/bash
# Interleaved A/B on one box: this tree (production poll settings) vs the
# tree at the start of the round-2 latency work (_ab_old, its own 5 ms settings)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2ab
mkdir -p $O
for i in 1 2 3; do
  for v in new old; do
    d=$R; [ $v = old ] && d=$R/_ab_old
    (cd $d && timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err)
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
