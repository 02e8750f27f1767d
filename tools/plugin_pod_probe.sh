#!/bin/bash
# The plugin-validation pod's process (amdgpu-validator --steps hip,vecadd,
# 1 Mi elements) under runtime settings, interleaved, 6 rounds, 0.3 s apart:
# spawn-to-exit wall (ms), the validator's step times and its stream creation
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=amdgpu_operator/_native/amdgpu-validator
run() {  # name, env..., -- args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  local s=$(date +%s%N)
  local o
  o=$(env "${envs[@]}" timeout -k 5 60 $V --rendezvous /tmp/ppp-rv "$@" 2>&1) || { echo "$name FAILED: $o"; exit 1; }
  local e=$(date +%s%N)
  echo "$name wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({x["name"]: round(x["seconds"]*1e3,1) for x in d["steps"]}, "stream", round(d.get("stream_create_s",0)*1e3,1), "total", round(d.get("seconds",0)*1e3,1))')"
}
A="--steps hip,vecadd --vecadd-elems 1048576"
for i in 1 2 3 4 5 6; do
  for v in "base" "devkarg0 HIP_FORCE_DEV_KERNARG=0" "fgskarg ROC_USE_FGS_KERNARG=1" \
           "skipcopy ROC_SKIP_KERNEL_ARG_COPY=1" "coherent HIP_HOST_COHERENT=1"; do
    set -- $v
    name=$1; shift
    run $name HSA_ENABLE_SDMA=0 "$@" -- $A
    sleep 0.3
  done
done
