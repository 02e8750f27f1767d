#!/bin/bash
# Same A/B as rccl_thp_probe.sh for the kernel-check validator (HIP) and the
# plugin pod's HSA check: process wall and the validator's own step times.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=amdgpu_operator/_native/amdgpu-validator
C=amdgpu_operator/_native/amdgpu-gpu-check
run() {
  local name=$1; shift
  local s=$(date +%s%N)
  local o
  o=$(env "$@" timeout -k 5 60 $V --steps hip,vecadd,gemm,mfma,hbm --rendezvous /tmp/thpw-rv --run-id $name-$RANDOM 2>&1) || { echo "$name FAILED: $(echo "$o" | tail -2)"; exit 1; }
  local e=$(date +%s%N)
  echo "$name validator wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({x["name"]: x.get("seconds") for x in d["steps"]})')"
  s=$(date +%s%N)
  o=$(env "$@" HSA_ENABLE_SDMA=0 timeout -k 5 30 $C 2>&1) || { echo "$name gpu-check FAILED: $(echo "$o" | tail -2)"; exit 1; }
  e=$(date +%s%N)
  echo "$name gpu-check wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("seconds"))')"
}
for i in 1 2 3 4 5 6; do
  run base X=1
  run hugetlb1 GLIBC_TUNABLES=glibc.malloc.hugetlb=1
done
