#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 $R/tools/validator_timing.py > $O/timing.jsonl 2> $O/timing.err
rc=$?; echo "timing rc=$rc"; cat $O/timing.jsonl | cut -c1-600; tail -5 $O/timing.err
exit $rc
