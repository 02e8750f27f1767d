#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s13
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest $R/tests/test_kernels_gpu.py -x -q -k "hbm or gemm" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/hbm_sweep.py > $O/hbm_sweep.json 2> $O/hbm_sweep.err
rc=$?; echo "sweep rc=$rc"; head -30 $O/hbm_sweep.json; grep -A12 '"4294967296"' $O/hbm_sweep.json
exit $rc
