#!/bin/bash
# rocprofv3 kernel-trace stats of the validator's kernel steps and of its RCCL
# step on the gfx950-trimmed RCCL (one MI355X).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rocprof}
mkdir -p $O /tmp/rv1 /tmp/rv2
cd /tmp && export TMPDIR=/tmp
V=$R/amdgpu_operator/_native/amdgpu-validator
AMDGPU_VALIDATOR_TEARDOWN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kernels -o run -- $V --rendezvous /tmp/rv1 \
    --steps hip,vecadd,gemm,mfma,hbm,xgmi > $O/kernels.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -2 $O/kernels.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
AMDGPU_VALIDATOR_TEARDOWN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rccl -o run -- $V --rendezvous /tmp/rv2 \
    --steps hip,rccl > $O/rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -2 $O/rccl.log | cut -c1-300
find $O -name "*kernel_stats.csv" | head
exit $rc
