#!/bin/bash
# Fresh-process start-up: ROCr alone (hsa_init_probe: one kernel via AQL) vs
# the HIP runtime (hip_init_probe: first kernel), interleaved, 6 runs each;
# prints each probe's JSON line plus the spawn-to-exit wall time in ms
cd ${GRAFT_REPO_ROOT:-$(pwd)}
H=tools/native/hsa_init_probe
P=tools/native/hip_init_probe
for i in 1 2 3 4 5 6; do
  for b in $H $P; do
    s=$(date +%s%N)
    o=$(timeout -k 5 30 $b amdgpu_operator/_native/validator_kernels.co) || { echo "$b failed: $o"; exit 1; }
    e=$(date +%s%N)
    echo "$(basename $b) wall_ms=$(( (e - s) / 1000000 )) $o"
  done
done
