#!/bin/bash
# One driver-style bench run on the MI355X with the per-step breakdown kept.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r3_bench}; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps ${STEPS:-10} --warmup 2 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $O/bench.json
exit $rc
