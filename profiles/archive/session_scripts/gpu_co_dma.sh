#!/bin/bash
# Does ROCr's HSA_CO_DMACOPY_SIZE (code-object segment copy by DMA) speed up
# loading RCCL's gfx950 code object?  co_load_probe under several settings.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-co_dma}
mkdir -p $O
cd $R
python3 -c "
from amdgpu_operator.toolkit import fatbin as F
_, e, b = F.fatbin_of('amdgpu_operator/_native/rccl-gfx950/librccl.so.1')
t, co = F.code_object(b, e, 'gfx950'); open('/tmp/rccl_gfx950.co', 'wb').write(co)" || exit 1
for r in 1 2; do
  for v in unset 0 1 4096 1048576; do
    if [ $v = unset ]; then
      out=$(timeout -k 5 60 tools/native/co_load_probe /tmp/rccl_gfx950.co) || exit $?
    else
      out=$(HSA_CO_DMACOPY_SIZE=$v timeout -k 5 60 tools/native/co_load_probe /tmp/rccl_gfx950.co) || exit $?
    fi
    echo "{\"HSA_CO_DMACOPY_SIZE\": \"$v\", \"round\": $r, \"probe\": $out}" | tee -a $O/co_dma.jsonl
  done
done
