#!/bin/bash
# ncclCommInitRank of the validator's RCCL step (1 rank) with glibc's malloc
# asked for transparent huge pages (GLIBC_TUNABLES=glibc.malloc.hugetlb=1):
# the communicator set-up is mostly system time loading RCCL's 108 MB code
# object, i.e. page faults on freshly allocated buffers.  Interleaved, 6 rounds.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
echo "thp: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null) defrag: $(cat /sys/kernel/mm/transparent_hugepage/defrag 2>/dev/null)"
V=amdgpu_operator/_native/amdgpu-validator
run() {
  local name=$1; shift
  local s=$(date +%s%N)
  local o
  o=$(env "$@" timeout -k 5 60 $V --steps hip,rccl --rccl-elems 1048576 --rendezvous /tmp/thp-rv --run-id $name-$RANDOM 2>&1) || { echo "$name FAILED: $(echo "$o" | tail -2)"; exit 1; }
  local e=$(date +%s%N)
  echo "$name wall_ms=$(( (e - s) / 1000000 )) $(echo "$o" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=[x for x in d["steps"] if x["name"]=="rccl"][0]; print({k: r.get(k) for k in ("comm_init_s","init_wait_s")})')"
}
for i in 1 2 3 4 5 6; do
  run base X=1
  run hugetlb1 GLIBC_TUNABLES=glibc.malloc.hugetlb=1
done
