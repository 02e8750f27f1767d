#!/bin/bash
# Round 2: GPU tier, then A/B of the held workload exit (default) vs immediate exit, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s24
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in hold nohold; do
    e="AMDGPU_VALIDATOR_HOLD_EXIT=1"; [ $v = nohold ] && e="AMDGPU_VALIDATOR_HOLD_EXIT=0"
    env $e timeout -k 10 400 python3 -u bench.py --steps 8 --warmup 1 --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
