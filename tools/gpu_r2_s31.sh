#!/bin/bash
# Round 2 (re-entry): GPU tier, smoke, default bench and a kernel-stats profile at HEAD
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s31
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.out
[ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
AMDGPU_VALIDATOR_TEARDOWN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 > $O/prof_bench.out 2> $O/prof_bench.err
rc=$?; echo "rocprof rc=$rc"
exit $rc
