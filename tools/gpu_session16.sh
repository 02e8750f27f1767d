#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest $R/tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/startup_timing.py > $O/startup.json 2>&1
rc=$?; echo "startup rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 1 --detail $O/detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
exit $rc
