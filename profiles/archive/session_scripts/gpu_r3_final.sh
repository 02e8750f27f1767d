#!/bin/bash
# End-of-round check on one MI355X: GPU test tier, smoke(), driver-style bench (20 steps + 5 warm-up).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r3_final}; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json
exit $rc
