#!/bin/bash
# Rehearsed multi-GPU critical path (RCCL validation at N=1): RCCL in its own
# process vs inside the kernel-check process, interleaved bench runs.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rccl_ab}
mkdir -p $O
cd $R
for r in 1 2; do
  for mode in separate shared; do
    timeout -k 10 240 python3 -u bench.py --steps 6 --warmup 1 --rccl-single-gpu --rccl-process $mode \
        --detail $O/${mode}_$r.detail.json > $O/${mode}_$r.json 2> $O/${mode}_$r.err
    rc=$?; echo "$mode round $r rc=$rc: $(python3 -c "import json,sys; d=json.load(open('$O/${mode}_$r.json')); print(d['value'], d['config']['time_to_ready_s'])" 2>&1)"
    [ $rc -ne 0 ] && { tail -5 $O/${mode}_$r.err; exit $rc; }
  done
done
exit 0
