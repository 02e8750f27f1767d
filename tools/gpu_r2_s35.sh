#!/bin/bash
# Round 2: GPU tier and the default-shape bench after the driver-recovery, admission-retry and shutdown changes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s35
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.out
[ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
exit 0
