#!/bin/bash
# A/B: pod-resources channel opened early vs at first use, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s23
mkdir -p $O
cd $R
for i in 1 2; do
  for v in pre lazy; do
    e=""; [ $v = lazy ] && e="AMDGPU_EXPERIMENT_NO_PRECONNECT=1"
    env $e timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 1 --kubelet-status-s 0 --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
