#!/bin/bash
# Full GPU tier + N=1 headline bench (what the driver runs at round end),
# then the N=1 bench with the RCCL validation process rehearsed (the critical
# path of a multi-GPU node: tools/rccl_init_probe.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-full}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; tail -3 $O/bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --rccl-single-gpu --detail $O/bench_rccl_detail.json > $O/bench_rccl.json 2> $O/bench_rccl.err
rc=$?; echo "bench rccl rehearsal rc=$rc"; cat $O/bench_rccl.json; tail -3 $O/bench_rccl.err
exit $rc
