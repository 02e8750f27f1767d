#!/bin/bash
# built by: /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/native/co_load_probe.cpp -o tools/native/co_load_probe
# RCCL start-up on the GPU box: trimmed vs system library (validator rccl
# step, phase-timed) and the bare cost of loading RCCL's gfx950 code object.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rccl_load}
mkdir -p $O
cd $R
python3 -c "
from amdgpu_operator.toolkit import fatbin as F
_, e, b = F.fatbin_of('amdgpu_operator/_native/rccl-gfx950/librccl.so.1')
t, co = F.code_object(b, e, 'gfx950'); open('/tmp/rccl_gfx950.co', 'wb').write(co)" || exit 1
for i in 1 2 3; do
  timeout -k 5 60 tools/native/co_load_probe /tmp/rccl_gfx950.co >> $O/co_load.jsonl 2>> $O/co_load.err || exit $?
done
cat $O/co_load.jsonl
timeout -k 10 400 python3 -u tools/rccl_init_probe.py $O 3 > $O/probe.log 2>&1
rc=$?; tail -30 $O/probe.log; exit $rc
