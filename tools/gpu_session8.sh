#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/exit_check.py > $O/exit.jsonl 2> $O/exit.err
rc=$?; echo "exit-check rc=$rc"; cut -c1-1500 $O/exit.jsonl
exit $rc
