#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest $R/tests/test_kernels_gpu.py -x -q > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/kernel_bench.py > $O/kbench.json 2> $O/kbench.err
rc=$?; echo "kbench rc=$rc"; cat $O/kbench.json; tail -3 $O/kbench.err
exit $rc
