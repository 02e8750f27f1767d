#!/bin/bash
# GPU tier, then the RCCL start-up probe and the rehearsed bench (device-side RCCL checks)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-dev}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/rccl_init_probe.py $O 3 > $O/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep '"gfx950-rccl", "round": [0-2]' $O/probe.log | cut -c1-330
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 1 --rccl-single-gpu --detail $O/bench_rccl_detail.json > $O/bench_rccl.json 2> $O/bench_rccl.err
rc=$?; echo "bench rccl rc=$rc"; cut -c1-420 $O/bench_rccl.json
exit $rc
