#!/bin/bash
# GPU session 4: kernel tests, end-to-end bench (N=1), rocprof of the bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest $R/tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -20 $O/bench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-counter-gate > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $O/prof.log; ls $O/prof
exit $rc
