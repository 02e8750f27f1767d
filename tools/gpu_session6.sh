#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/validator_timing.py > $O/timing.jsonl 2> $O/timing.err
rc=$?; echo "timing rc=$rc"; cut -c1-400 $O/timing.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -20 $O/bench.err
exit $rc
