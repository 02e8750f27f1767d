#!/bin/bash
# Round 2: bench at production poll settings (1 s agent poll, 10 s kubelet status tick)
# vs the old fast-poll configuration, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s10
mkdir -p $O
cd $R
for i in 1 2; do
  for v in prod fast; do
    extra=""
    [ $v = fast ] && extra="--agent-poll-s 0.005 --kubelet-status-s 0"
    timeout -k 10 400 python3 -u bench.py --steps 8 --warmup 2 $extra --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
