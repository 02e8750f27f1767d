#!/bin/bash
# Round 2: GPU tier, default bench and the RCCL-rehearsal bench after the NFD readiness / sandbox changes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s32
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.out
[ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --kubelet-status-s 0 --rccl-single-gpu --detail $O/rehearsal.json > $O/rehearsal.out 2> $O/rehearsal.err
rc=$?; echo "rehearsal rc=$rc"; cut -c1-400 $O/rehearsal.out
[ $rc -ne 0 ] && { tail -5 $O/rehearsal.err; exit $rc; }
exit 0
