#!/bin/bash
# First GPU session: fixtures, kernel numerics, kernel micro-bench, rocprof stats.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date)"
timeout -k 10 240 python3 $R/tools/capture_fixtures.py $O/fixtures > $O/fixtures.log 2>&1 || echo "fixtures rc=$?"
echo "fixtures done $(date)"
timeout -k 10 480 python3 -m pytest $R/tests/test_kernels_gpu.py -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)"; tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/kernel_bench.py > $O/kbench.json 2> $O/kbench.err
rc=$?; echo "kbench rc=$rc $(date)"; cat $O/kbench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o kb --output-format csv -- python3 $R/tools/kernel_bench.py --quick > $O/prof1.log 2>&1
rc=$?; echo "rocprof rc=$rc $(date)"
exit $rc
