#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s17
mkdir -p $O
timeout -k 10 300 python3 $R/tools/gemm_stamps.py > $O/stamps.json 2> $O/stamps.err
rc=$?; echo "rc=$rc"; cat $O/stamps.json; tail -5 $O/stamps.err
