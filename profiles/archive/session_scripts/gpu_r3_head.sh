#!/bin/bash
# Round-3 HEAD check on one MI355X: GPU tier, driver-style bench, rocprofv3 kernel stats of a bench run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3_head}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 10 --warmup 2 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
[ $rc -ne 0 ] && exit $rc
[ -n "${SKIP_PROF:-}" ] && exit 0
mkdir -p /tmp/rv1
cd /tmp
AMDGPU_VALIDATOR_TEARDOWN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    $R/amdgpu_operator/_native/amdgpu-validator --rendezvous /tmp/rv1 --steps hip,vecadd,gemm,mfma,hbm,xgmi > $O/validator_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $O/validator_prof.log | cut -c1-400
exit $rc
