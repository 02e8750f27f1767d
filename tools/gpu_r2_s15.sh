#!/bin/bash
# Round 2: does the workload validation's GPU work slow the plugin pod? full vs quick workload, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s15
mkdir -p $O
cd $R
for i in 1 2; do
  for v in full quick; do
    extra=""
    [ $v = quick ] && extra="--quick-workload"
    timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 1 --kubelet-status-s 0 $extra --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
