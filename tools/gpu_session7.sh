#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --steps 5 --warmup 1 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -5 $O/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/__graft_entry__.py smoke > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
exit $rc
