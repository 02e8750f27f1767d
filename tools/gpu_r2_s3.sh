#!/bin/bash
# Round 2: validator result at its report (pipes closed) vs at its exit, interleaved A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s3
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py tests/test_launcher.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in early exit; do
    e=1; [ $v = exit ] && e=0
    AMDGPU_VALIDATOR_REPORT_EARLY=$e timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --detail $O/ab_${v}_$i.json > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cut -c100-140 $O/ab_${v}_$i.out)"
    [ $rc -ne 0 ] && { tail -5 $O/ab_${v}_$i.err; exit $rc; }
  done
done
exit 0
