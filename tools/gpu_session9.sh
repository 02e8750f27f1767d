#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -m pytest $R/tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 $O/pytest_gpu.log
exit $rc
