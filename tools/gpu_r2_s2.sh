#!/bin/bash
# Round 2: GPU tier after the driver/hook changes, then interleaved A/B of the
# validator start gate (prespawn) against the previous ordering
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s2
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in pre nopre; do
    flag=""; [ $v = nopre ] && flag="--no-prespawn"
    timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 $flag --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c1-220 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
