#!/bin/bash
# RCCL rehearsal at N=1 (the multi-GPU critical path): RCCL in its own process
# per GPU (separate, default) vs in the kernel-check process (shared), interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s25
mkdir -p $O
cd $R
for i in 1 2; do
  for v in separate shared; do
    timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 1 --kubelet-status-s 0 --rccl-single-gpu --rccl-process $v --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
