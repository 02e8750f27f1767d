#!/bin/bash
# Round 2, last: what the driver runs at round end (GPU tests, smoke, default bench) at HEAD
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s36
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py > $O/bench.out 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-250 $O/bench.out
exit $rc
