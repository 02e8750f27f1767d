#!/bin/bash
# ncclCommInitRank cost of the validator's RCCL step (1 rank) under RCCL
# settings (off-node, algorithm tables, buffer and FIFO sizes, channel count), interleaved,
# 5 rounds: lib_load_s, comm_init_s and the process wall (ms)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=amdgpu_operator/_native/amdgpu-validator
run() {
  local name=$1; shift
  local s=$(date +%s%N)
  local o
  o=$(env "$@" timeout -k 5 60 $V --steps hip,rccl --rccl-elems 1048576 --rendezvous /tmp/rep-rv --run-id $name-$RANDOM 2>&1) || { echo "$name FAILED: $(echo "$o" | tail -2)"; exit 1; }
  local e=$(date +%s%N)
  echo "$name wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=[x for x in d["steps"] if x["name"]=="rccl"][0]; print({k: r.get(k) for k in ("lib_load_s","comm_init_s","init_wait_s","library")})')"
}
for i in 1 2 3 4 5; do
  run base X=1
  run noib NCCL_IB_DISABLE=1
  run fifo4k NCCL_WORK_FIFO_DEPTH=4096
  run buf1m NCCL_BUFFSIZE=1048576
  run ch4 NCCL_MAX_NCHANNELS=4
  run runtime_connect NCCL_RUNTIME_CONNECT=1
done
