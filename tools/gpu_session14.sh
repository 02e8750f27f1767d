#!/bin/bash
# time-to-Ready breakdown on the current code + validator process timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s14
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 1 --detail $O/detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
V=$R/amdgpu_operator/_native/amdgpu-validator
for i in 1 2 3; do
  /usr/bin/time -f "wall %e s" timeout -k 10 60 $V --rendezvous /tmp/rv$i --run-id r$i --steps hip,vecadd,gemm,hbm,xgmi --gemm 4096 --counter-gate > $O/val$i.json 2>> $O/val_time.txt
  echo "val$i rc=$?"
done
AMDGPU_VALIDATOR_COUNTERS=1 timeout -k 10 60 $V --rendezvous /tmp/rv9 --run-id r9 --steps hip,vecadd,gemm,hbm,xgmi --gemm 4096 --counter-gate > $O/val_gate.json 2>> $O/val_time.txt
echo "gate rc=$?"
cat $O/val_time.txt | grep wall
