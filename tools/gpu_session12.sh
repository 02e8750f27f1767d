#!/bin/bash
# Full GPU test tier + 1-GPU bench (each GPU step under its own time limit)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest $R/tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
exit $rc
