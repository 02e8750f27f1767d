#!/bin/bash
# AQL-packet counter gate variants on the GPU box (bounded, diagnostics)
cd /tmp
N=/root/repo/amdgpu_operator/_native
O=/root/repo/gpurun_out
i=0
for v in "" "AMDGPU_AQL_GATE_READ=1" "AQLPROFILE_READ_API=1 AMDGPU_AQL_GATE_READ=1" "AMDGPU_AQL_GATE_NO_PROFILING=1"; do
  i=$((i+1))
  env AMDGPU_AQL_GATE_BUF_MULT=4 $v timeout -k 5 60 $N/amdgpu-validator --rendezvous /tmp/rva$i --steps hip,gemm --counter-gate > $O/aql_v$i.json 2> $O/aql_v$i.err
  rc=$?; echo "variant $i [$v] rc=$rc $(grep -o '"counter_gate[^}]*' $O/aql_v$i.json | cut -c1-400)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
