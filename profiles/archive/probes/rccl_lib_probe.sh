#!/bin/bash
# ncclCommInitRank (1 rank) with the gfx950-only RCCL stored zstd-compressed
# (default) vs uncompressed, interleaved, 6 rounds
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=amdgpu_operator/_native/amdgpu-validator
run() {
  local name=$1; shift
  local s=$(date +%s%N)
  local o
  o=$(env "$@" timeout -k 5 60 $V --steps hip,rccl --rccl-elems 1048576 --rendezvous /tmp/rlp-rv --run-id $name-$RANDOM 2>&1) || { echo "$name FAILED: $(echo "$o" | tail -2)"; exit 1; }
  local e=$(date +%s%N)
  echo "$name wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=[x for x in d["steps"] if x["name"]=="rccl"][0]; print({k: r.get(k) for k in ("lib_load_s","comm_init_s","library")})')"
}
RAW=$(pwd)/amdgpu_operator/_native/rccl-gfx950-raw/librccl.so.1
for i in 1 2 3 4 5 6; do
  run zstd X=1
  run raw AMDGPU_RCCL_LIBRARY=$RAW
done
