#!/bin/bash
# Round 2: GPU tier + bench at production settings after the inotify / SDMA changes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2s14}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 2 --detail $O/bench_$i.json > $O/bench_$i.out 2> $O/bench_$i.err
  rc=$?; echo "bench $i rc=$rc $(cut -c100-140 $O/bench_$i.out)"
  [ $rc -ne 0 ] && { tail -5 $O/bench_$i.err; exit $rc; }
done
exit 0
