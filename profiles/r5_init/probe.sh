#!/bin/bash
# HIP vs HSA start-up cost on the box, one process at a time
set -o pipefail
export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/r5_init
mkdir -p $O
N=amdgpu_operator/_native
TIMEFORMAT="%R s wall"
for i in 1 2 3 4; do
  { time timeout -k 5 30 $N/amdgpu-gpu-check > $O/check.$i.json; } 2> $O/check.$i.time || exit 1
  { time timeout -k 5 30 $N/amdgpu-validator --rendezvous /tmp/rv-init --steps hip > $O/hip.$i.json; } 2> $O/hip.$i.time || exit 1
  { time timeout -k 5 30 $N/amdgpu-validator --rendezvous /tmp/rv-init --steps hip,vecadd > $O/vec.$i.json; } 2> $O/vec.$i.time || exit 1
done
echo probes done
cd /tmp && export TMPDIR=/tmp AMDGPU_VALIDATOR_CLEAN_EXIT=1
timeout -k 10 90 rocprofv3 --hip-trace --hsa-trace --kernel-trace --memory-copy-trace -d $GRAFT_REPO_ROOT/$O/trace -o run --output-format csv -- $GRAFT_REPO_ROOT/$N/amdgpu-validator --rendezvous /tmp/rv-init2 --steps hip,vecadd > $GRAFT_REPO_ROOT/$O/traced.json 2> $GRAFT_REPO_ROOT/$O/traced.err
echo rc=$?
